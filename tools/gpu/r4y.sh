# round 4 (y): plan with the 256 x 256 tile for wide shallow products -- tests, GEMM bench, benches
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4y_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 150 gpurun_out/r4y_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 200 gpurun_out/r4y_bench.log python -u bench.py
run_step 200 gpurun_out/r4y_bench_bf16.log python -u bench.py --precision bf16
HX_GEMM_F16_CFG=0 run_step 200 gpurun_out/r4y_bench_cfg0.log python -u bench.py
run_step 240 gpurun_out/r4y_bench_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
echo done
