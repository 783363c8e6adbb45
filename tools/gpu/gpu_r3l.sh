set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests_l.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_l.log 2>&1 &&
bash tools/prof_run.sh r3l > gpurun_out/prof_r3l.log 2>&1
