set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe/ffn_epilogue_probe.py > gpurun_out/ffn_epi3.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_split_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_g.log 2>&1
