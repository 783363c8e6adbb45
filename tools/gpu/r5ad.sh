# round 5 (ad): attention kernels -- standalone times and counters (fwd / bwd fp16x3, B128 S128)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 120 gpurun_out/r5ad_attn_times.log python -u tools/bench_kernels.py --only attn &&
run_step 90 gpurun_out/r5ad_pmc1.log timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "attn_(fwd|bwd)_f16" --output-format csv -d /tmp/pmc_r5ad1 -o run -- python3 tools/bench_kernels.py --only attn &&
python tools/pmc_summary.py /tmp/pmc_r5ad1/run_counter_collection.csv > gpurun_out/r5ad_pmc1.md &&
run_step 90 gpurun_out/r5ad_pmc2.log timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --kernel-include-regex "attn_(fwd|bwd)_f16" --output-format csv -d /tmp/pmc_r5ad2 -o run -- python3 tools/bench_kernels.py --only attn &&
python tools/pmc_summary.py /tmp/pmc_r5ad2/run_counter_collection.csv > gpurun_out/r5ad_pmc2.md
echo done
