# round 5 (ag): weight gradient on 32-token stages -- tests, repeated A/B vs 16-token stages (cfg 2)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5ag_gemmtests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py &&
WGRAD_PLANS=1:0,2:0,1:0,2:0,1:0,2:0 run_step 300 gpurun_out/r5ag_wgrad_ab.log python -u tools/probe/gemm_f16_bench.py
echo done
