set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/o_def0.log 2>&1 &&
HX_WGRAD_DEFER=0 timeout -k 10 300 python -u bench.py > gpurun_out/o_nodef0.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/o_def1.log 2>&1 &&
HX_WGRAD_DEFER=0 timeout -k 10 300 python -u bench.py > gpurun_out/o_nodef1.log 2>&1
