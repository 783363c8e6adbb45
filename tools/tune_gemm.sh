#!/bin/bash
# Re-tune the shipped GEMM solution table on an MI355X (see hetseq_9cme_amd/ops/gemm_tuning.py);
# merge the resulting CSVs with tools/merge_gemm_tables.py afterwards.
set -e
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > $O/t10_table_fp32.log 2>&1
# bf16 online tuning is not run: a library candidate faulted (illegal address) during bf16 tuning on ROCm 7.2
timeout -k 10 600 python bench.py --steps 6 --warmup 3 --model large --gemm-tuning online --gemm-tuning-file $O/tune_fp32_large.csv > $O/t10_large.log 2>&1
timeout -k 10 500 python bench.py --steps 6 --warmup 3 --model large --precision bf16 --gemm-tuning online --gemm-tuning-file $O/tune_bf16_large.csv > $O/t10_large_bf16.log 2>&1
tail -n1 $O/t10_*.log
