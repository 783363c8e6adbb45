# round 4 (ab): weight-gradient tile / split sweep (HX_WGRAD_F16 forces cfg:nsplit for every shape)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 150 gpurun_out/r4ab_plan.log python -u tools/probe/gemm_f16_bench.py
HX_WGRAD_F16=0:4 run_step 150 gpurun_out/r4ab_0_4.log python -u tools/probe/gemm_f16_bench.py
HX_WGRAD_F16=0:8 run_step 150 gpurun_out/r4ab_0_8.log python -u tools/probe/gemm_f16_bench.py
HX_WGRAD_F16=1:12 run_step 150 gpurun_out/r4ab_1_12.log python -u tools/probe/gemm_f16_bench.py
HX_WGRAD_F16=1:5 run_step 150 gpurun_out/r4ab_1_5.log python -u tools/probe/gemm_f16_bench.py
echo done
