# round 4 (r): SQ / TCC counters of the fp16x3 GEMMs (QKV shape: forward, data gradient, weight gradient)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
ONLY=qkv run_step 90 gpurun_out/r4r_pmc1.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d gpurun_out/pmc_r4r1 -o run -- python3 tools/probe/gemm_f16_bench.py
ONLY=qkv run_step 90 gpurun_out/r4r_pmc2.log rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_COUNT --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d gpurun_out/pmc_r4r2 -o run -- python3 tools/probe/gemm_f16_bench.py
ONLY=qkv run_step 90 gpurun_out/r4r_pmc3.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d gpurun_out/pmc_r4r3 -o run -- python3 tools/probe/gemm_f16_bench.py
echo done
