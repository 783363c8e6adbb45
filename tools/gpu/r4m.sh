# round 4 (m): full GPU suite + smoke on the final tree
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 1000 gpurun_out/r4m_gpu_tests.log python -u -m pytest tests/ -m gpu -v --timeout 200 --timeout-method thread
run_step 150 gpurun_out/r4m_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
echo done
