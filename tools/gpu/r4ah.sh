# round 4 (ah): full GPU suite + smoke + fp32 headline bench on the tree with the bf16 GELU epilogues
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 1000 gpurun_out/r4ah_gpu_tests.log python -u -m pytest tests/ -m gpu -v --timeout 200 --timeout-method thread
run_step 150 gpurun_out/r4ah_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run_step 200 gpurun_out/r4ah_bench.log python -u bench.py
echo done
