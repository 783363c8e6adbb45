# round 4 (o): SQ counters of the two-waves-per-SIMD fp16x3 attention backward; phase-2 kernel trace
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 90 gpurun_out/r4o_pmc1.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex attn_bwd --output-format csv -d gpurun_out/pmc_r4o1 -o run -- python3 tools/probe/attn_bwd_probe.py
run_step 90 gpurun_out/r4o_pmc2.log rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_COUNT --kernel-include-regex attn_bwd --output-format csv -d gpurun_out/pmc_r4o2 -o run -- python3 tools/probe/attn_bwd_probe.py
run_step 300 gpurun_out/r4o_prof_p2.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4o_p2 -o run -- python3 bench.py --seq 512 --batch 32 --max-pred 80 --steps 5 --warmup 3
echo done
