# round 4 (s): four-stage DMA ring in gemm_f16_k -- GEMM tests, GEMM bench, headline bench
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4s_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 150 gpurun_out/r4s_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 200 gpurun_out/r4s_bench.log python -u bench.py
run_step 200 gpurun_out/r4s_bench_bf16.log python -u bench.py --precision bf16
echo done
