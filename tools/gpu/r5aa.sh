# round 5 (aa): counters of the current fp16x3 GEMM / wgrad on the FFN-down shapes (three passes)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
ONLY=ffn_down run_step 90 gpurun_out/r5aa_pmc1.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d /tmp/pmc_r5aa1 -o run -- python3 tools/probe/gemm_f16_bench.py &&
python tools/pmc_summary.py /tmp/pmc_r5aa1/run_counter_collection.csv > gpurun_out/r5aa_pmc1.md &&
ONLY=ffn_down run_step 90 gpurun_out/r5aa_pmc2.log timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d /tmp/pmc_r5aa2 -o run -- python3 tools/probe/gemm_f16_bench.py &&
python tools/pmc_summary.py /tmp/pmc_r5aa2/run_counter_collection.csv > gpurun_out/r5aa_pmc2.md &&
ONLY=ffn_down run_step 90 gpurun_out/r5aa_pmc3.log timeout -s KILL 80 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d /tmp/pmc_r5aa3 -o run -- python3 tools/probe/gemm_f16_bench.py &&
python tools/pmc_summary.py /tmp/pmc_r5aa3/run_counter_collection.csv > gpurun_out/r5aa_pmc3.md
echo done
