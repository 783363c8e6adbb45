# round 5 (aq): repeated A/B of the 256 x 192 tile (cfg 1) vs 128 x 192 at two workgroups per CU (cfg 4)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
CFGS=1,4,1,4,1,4 run_step 300 gpurun_out/r5aq_cfg14_ab.log python -u tools/probe/gemm_f16_bench.py
echo done
