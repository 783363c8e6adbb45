set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/probe/wgrad_group_probe.py > gpurun_out/wgrad_group_probe.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_d.log 2>&1 &&
HX_WGRAD_GROUP=0 timeout -k 10 300 python -u bench.py > gpurun_out/bench_d_nogroup.log 2>&1 &&
bash tools/prof_run.sh r3d &&
bash tools/probe/comm_contention_probe.sh 16 > gpurun_out/comm_contention.log 2>&1
