# round 4 (x): 256 x 256 tile (cfg 5) -- bf16 plan, fp16x3 sweep; tests; benches
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4x_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 150 gpurun_out/r4x_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
T=16384 CFGS=0:1,5:1 run_step 240 gpurun_out/r4x_sweep.log python -u tools/probe/gemm_f16_bench.py
run_step 200 gpurun_out/r4x_bench_bf16.log python -u bench.py --precision bf16
run_step 200 gpurun_out/r4x_bench.log python -u bench.py
echo done
