# round 4 (aa): fp16x3 GEMM with a four-stage ring and the next stage's fragments read under the
# current stage's MFMAs -- tests, GEMM bench, benches (A/B against the saved baseline numbers)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4aa_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 150 gpurun_out/r4aa_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 200 gpurun_out/r4aa_bench.log python -u bench.py
run_step 240 gpurun_out/r4aa_bench_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
echo done
