# round 5 (b): SQ / TCC counters of the pipelined fp16x3 GEMM (QKV shape), both large-tile wave layouts
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
for cfg in 0 1; do
HX_GEMM_F16_CFG=$cfg ONLY=qkv run_step 90 gpurun_out/r5b_pmc1_c$cfg.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d gpurun_out/pmc_r5b1_c$cfg -o run -- python3 tools/probe/gemm_f16_bench.py
HX_GEMM_F16_CFG=$cfg ONLY=qkv run_step 90 gpurun_out/r5b_pmc2_c$cfg.log rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_COUNT --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d gpurun_out/pmc_r5b2_c$cfg -o run -- python3 tools/probe/gemm_f16_bench.py
HX_GEMM_F16_CFG=$cfg ONLY=qkv run_step 90 gpurun_out/r5b_pmc3_c$cfg.log rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-include-regex "gemm_f16|wgrad_f16" --output-format csv -d gpurun_out/pmc_r5b3_c$cfg -o run -- python3 tools/probe/gemm_f16_bench.py
done
HX_GEMM_F16_CFG=1 run_step 200 gpurun_out/r5b_gemm_bench_c1.log python -u tools/probe/gemm_f16_bench.py
echo done
