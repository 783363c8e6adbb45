# round 5 (z): repeated same-box A/B of the batch-32 tile plan (2 vs 1) and the GELU store policy
# (6 plain vs 11 non-temporal stores everywhere; the default now = nt for the GELU epilogues)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
T=4096 CFGS=2,1,2,1,2,1 run_step 300 gpurun_out/r5z_m4096_ab.log python -u tools/probe/gemm_f16_bench.py &&
CFGS=6,11,6,11 run_step 300 gpurun_out/r5z_store_ab.log python -u tools/probe/gemm_f16_bench.py
echo done
