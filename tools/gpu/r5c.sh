# round 5 (c): ring depth 5 vs 4, wave layouts -- GEMM tests, per-shape sweep
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5c_gemmtests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py -k "every_tile or forward or dgrad or gelu"
CFGS=1,6,0,4 run_step 300 gpurun_out/r5c_sweep.log python -u tools/probe/gemm_f16_bench.py
echo done
