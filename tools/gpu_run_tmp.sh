set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_gp.log 2>&1 &&
tail -n 1 gpurun_out/bench_gp.log | cut -c 1-250 &&
bash tools/prof_run.sh gp
