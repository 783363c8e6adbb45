# round 5 (af): whole GPU suite, smoke and bench on the cleaned kernel table
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 900 gpurun_out/r5af_gpu_suite.log python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests &&
run_step 300 gpurun_out/r5af_smoke.log python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
run_step 300 gpurun_out/r5af_bench.log python -u bench.py
echo done
