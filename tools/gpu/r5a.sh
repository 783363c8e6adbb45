# round 5 (a): the pipelined per-row-scaled fp16x3 GEMM -- GEMM tests, GEMM bench
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 400 gpurun_out/r5a_gemmtests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 200 gpurun_out/r5a_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
echo done
