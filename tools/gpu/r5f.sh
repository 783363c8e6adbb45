# round 5 (f): timing diagnostics -- no k-loop DMA (cfg 8), 128-B-row DMA pieces (cfg 9) vs cfg 6; TA / TD / TCP counters
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
CFGS=6,8,9,6,8,9 run_step 300 gpurun_out/r5f_sweep.log python -u tools/probe/gemm_f16_bench.py
HX_GEMM_F16_CFG=6 ONLY=qkv run_step 90 gpurun_out/r5f_pmc.log rocprofv3 --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCP_TA_ADDR_STALL_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16" --output-format csv -d gpurun_out/pmc_r5f -o run -- python3 tools/probe/gemm_f16_bench.py
HX_GEMM_F16_CFG=6 ONLY=qkv run_step 90 gpurun_out/r5f_pmc2.log rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_BUSY_avr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16" --output-format csv -d gpurun_out/pmc_r5f2 -o run -- python3 tools/probe/gemm_f16_bench.py
echo done
