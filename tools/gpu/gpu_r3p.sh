set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/p_def0.log 2>&1 &&
HX_WGRAD_SLOT_PCT=50 timeout -k 10 300 python -u bench.py > gpurun_out/p_50a.log 2>&1 &&
HX_WGRAD_SLOT_PCT=75 timeout -k 10 300 python -u bench.py > gpurun_out/p_75a.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/p_def1.log 2>&1 &&
HX_WGRAD_SLOT_PCT=50 timeout -k 10 300 python -u bench.py > gpurun_out/p_50b.log 2>&1 &&
HX_WGRAD_SLOT_PCT=75 timeout -k 10 300 python -u bench.py > gpurun_out/p_75b.log 2>&1
