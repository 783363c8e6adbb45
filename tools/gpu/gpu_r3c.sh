set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -k rccl -x -v --timeout 300 --timeout-method thread > gpurun_out/rccl_tests.log 2>&1 &&
bash tools/probe/comm_contention_probe.sh 16 > gpurun_out/comm_contention.log 2>&1 &&
bash tools/prof_run.sh r3c &&
timeout -k 10 200 python -u tools/probe/qkv_plan_probe.py > gpurun_out/qkv_plan_probe.log 2>&1 &&
timeout -k 10 200 python -u tools/probe/ffn_epilogue_probe.py > gpurun_out/ffn_epi_probe.log 2>&1
