# round 5 (w): weight-gradient plans at T = 16384 (token splits vs slab traffic)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
WGRAD_PLANS=plan,1:3,1:4,1:6,1:8,1:12,0:1,0:2,0:3 run_step 300 gpurun_out/r5w_wgrad_plans.log python -u tools/probe/gemm_f16_bench.py
echo done
