#!/bin/bash
# Re-tune the shipped fp32 GEMM solution table on an MI355X (hetseq_9cme_amd/ops/gemm_tuning.py),
# then merge:  python tools/merge_gemm_tables.py hetseq_9cme_amd/tuning/gemm_gfx950.csv OUT/tune_*0.csv
# (the device ordinal is appended to each file name).
#
# Only fp32 is tuned: on ROCm 7.2 a library candidate faulted (illegal address) while
# TunableOp benchmarked the bf16 shapes, so bf16 keeps the library heuristics.
set -e
export TMPDIR=/tmp
OUT=${OUT:-${GRAFT_REPO_ROOT:-.}/gpurun_out}
mkdir -p "$OUT"
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS:-120}
# BERT-base phase 1 (128 x 128 tokens per GPU) and phase 2 (32 x 512): same GEMM shapes
timeout -k 10 900 python bench.py --steps 6 --warmup 3 --gemm-tuning retune \
    --gemm-tuning-file "$OUT/tune_fp32_base.csv" > "$OUT/tune_fp32_base.log" 2>&1
# BERT-large phase 1 (new shapes are added on top of the shipped table)
timeout -k 10 900 python bench.py --steps 4 --warmup 2 --model large --gemm-tuning online \
    --gemm-tuning-file "$OUT/tune_fp32_large.csv" > "$OUT/tune_fp32_large.log" 2>&1
tail -n1 "$OUT"/tune_fp32_*.log
