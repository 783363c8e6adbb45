# round 5 (j): the whole GPU suite and the 1-GPU bench on the per-row-scale tree
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 900 gpurun_out/r5j_gpu_suite.log python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests &&
run_step 300 gpurun_out/r5j_bench.log python -u bench.py
echo done
