set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_k0.log 2>&1 &&
timeout -k 10 300 python -u bench.py --overlap-wgrad > gpurun_out/bench_k1.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_k2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --overlap-wgrad > gpurun_out/bench_k3.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "side or overlap or reducer or matches" > gpurun_out/side_tests.log 2>&1
