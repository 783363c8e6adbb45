# round 4, first call: the fp16x3 kernels' numerics, the fp16x3 bench + kernel trace, then the tree's state
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_f16_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r4a_f16.log 2>&1 &&
timeout -k 10 300 python -u bench.py --fp32-gemm fp16x3 > gpurun_out/r4a_bench_f16.log 2>&1 &&
bash tools/prof_run.sh r4a_f16 --fp32-gemm fp16x3 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r4a_bench.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a_gputests.log 2>&1
