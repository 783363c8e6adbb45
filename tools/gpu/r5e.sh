# round 5 (e): timing diagnostics -- no k-loop DMA (cfg 8), 128-B-row DMA pieces (cfg 9) vs cfg 6; counter list
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
CFGS=6,8,9,6,8,9 run_step 300 gpurun_out/r5e_sweep.log python -u tools/probe/gemm_f16_bench.py
run_step 60 gpurun_out/r5e_counters.log rocprofv3 -L
echo done
