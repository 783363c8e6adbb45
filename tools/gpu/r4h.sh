# round 4 (h): counters of the fp16x3 GEMM / weight-gradient kernels (qkv shapes), one pass each
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 60 gpurun_out/r4h_counters.txt rocprofv3 -L
ONLY=qkv run_step 90 gpurun_out/r4h_pmc1.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_r4h1 -o run -- python3 tools/probe/gemm_f16_bench.py
ONLY=qkv run_step 90 gpurun_out/r4h_pmc2.log rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_r4h2 -o run -- python3 tools/probe/gemm_f16_bench.py
echo done
