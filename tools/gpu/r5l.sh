# round 5 (l): epilogue / prologue share of the fp16x3 GEMM (HX_GEMM_DIAG 1: no epilogue, 2: no k loop)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
CFGS=6 run_step 200 gpurun_out/r5l_full.log python -u tools/probe/gemm_f16_bench.py &&
HX_GEMM_DIAG=1 CFGS=6 run_step 200 gpurun_out/r5l_noepi.log python -u tools/probe/gemm_f16_bench.py &&
HX_GEMM_DIAG=2 CFGS=6 run_step 200 gpurun_out/r5l_noloop.log python -u tools/probe/gemm_f16_bench.py
echo done
