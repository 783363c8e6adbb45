# round 4 (w): s_setprio pair around the GEMM MFMA clusters (guide T5) -- tests, GEMM bench, bench
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4w_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 150 gpurun_out/r4w_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 200 gpurun_out/r4w_bench.log python -u bench.py
echo done
