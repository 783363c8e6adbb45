# round 4 (j): fp16x3 attention forward + backward tests, kernel probe, SQ counters of the
# attention backward kernels (x6 / f16 / fp32)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 240 gpurun_out/r4j_attn_test.log python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_kernels_gpu.py -k "attention_f16 or attention_x6" tests/test_gemm_f16_gpu.py::test_gemm_f16_split_k_beta_bias
run_step 120 gpurun_out/r4j_attn_probe.log python -u tools/probe/attn_bwd_probe.py
export TMPDIR=/tmp
run_step 90 gpurun_out/r4j_pmc1.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex attn --output-format csv -d gpurun_out/pmc_r4j1 -o run -- python3 tools/probe/attn_bwd_probe.py
run_step 90 gpurun_out/r4j_pmc2.log rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_COUNT --kernel-include-regex attn --output-format csv -d gpurun_out/pmc_r4j2 -o run -- python3 tools/probe/attn_bwd_probe.py
echo done
