# round 5 (g): timing diagnostics -- no split VALU (10), + no DMA (11), + no barrier (12) vs cfg 6
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
CFGS=6,10,11,12,8,6 run_step 300 gpurun_out/r5g_sweep.log python -u tools/probe/gemm_f16_bench.py
echo done
