set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_split_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests_i.log 2>&1 &&
timeout -k 10 200 python -u tools/probe/ffn_epilogue_probe.py > gpurun_out/ffn_epi4.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_i.log 2>&1 &&
bash tools/prof_run.sh r3i > gpurun_out/prof_r3i.log 2>&1
