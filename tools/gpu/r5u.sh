# round 5 (u): NER-sized GEMMs (M = 1536): tile / split-K plans, weight-gradient plans
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
T=1536 CFGS=2,2:1,3,3:1,4,4:1,6,6:1 run_step 300 gpurun_out/r5u_m1536_sweep.log python -u tools/probe/gemm_f16_bench.py &&
T=1536 WGRAD_PLANS=plan,1:1,1:2,1:3,0:1,0:2,0:4 run_step 300 gpurun_out/r5u_m1536_wgrad.log python -u tools/probe/gemm_f16_bench.py
echo done
