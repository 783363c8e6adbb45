set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_j0.log 2>&1 &&
timeout -k 10 300 python -u bench.py --overlap-wgrad > gpurun_out/bench_j1.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_j2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --overlap-wgrad > gpurun_out/bench_j3.log 2>&1
