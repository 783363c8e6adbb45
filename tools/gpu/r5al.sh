# round 5 (al): weight-gradient split counts at T = 4096 (batch 32), repeated A/B on one box
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
T=4096 WGRAD_PLANS=1:0,1:4,1:2,0:0,1:0,1:4,1:2,0:0 run_step 300 gpurun_out/r5al_wgrad_t4096.log python -u tools/probe/gemm_f16_bench.py
echo done
