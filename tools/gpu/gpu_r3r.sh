set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r_p0a.log 2>&1 &&
HX_SIDE_PRIO=-1 timeout -k 10 300 python -u bench.py > gpurun_out/r_phia.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r_p0b.log 2>&1 &&
HX_SIDE_PRIO=-1 timeout -k 10 300 python -u bench.py > gpurun_out/r_phib.log 2>&1
