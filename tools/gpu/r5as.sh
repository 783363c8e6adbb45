#!/bin/bash
# A/B: GEMM A operand pre-split into fp16 pieces vs split in the k loop, plus its numerics tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py \
  -k "presplit or pieces_out" > gpurun_out/r5as_tests.log 2>&1 &&
PIECES_AB=5 timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5as_pieces_ab.log 2>&1
