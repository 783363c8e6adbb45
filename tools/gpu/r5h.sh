# round 5 (h): v_fma_mix split between pass-1/2 MFMAs -- GEMM tests (ramps) + tile sweep
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5h_gemmtests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py &&
CFGS=0,1,6,10,4,2 run_step 300 gpurun_out/r5h_sweep.log python -u tools/probe/gemm_f16_bench.py
echo done
