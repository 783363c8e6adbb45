set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/bench_gemm_split.py > gpurun_out/gemm_split.log 2>&1 &&
timeout -k 10 300 python -u bench.py --fp32-gemm bf16x3 > gpurun_out/bench_bf16x3.log 2>&1 &&
timeout -k 10 300 python -u bench.py --fp32-gemm bf16x6 > gpurun_out/bench_bf16x6.log 2>&1 &&
bash tools/prof_run.sh x3 --fp32-gemm bf16x3 && bash tools/prof_run.sh x6 --fp32-gemm bf16x6
