# round 5 (i): GEMM tests + split-placement sweep, then the whole GPU suite and the 1-GPU bench
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5i_gemmtests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py &&
CFGS=0,9,6,8,10 run_step 300 gpurun_out/r5i_sweep.log python -u tools/probe/gemm_f16_bench.py &&
run_step 900 gpurun_out/r5i_gpu_suite.log python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests &&
run_step 300 gpurun_out/r5i_bench.log python -u bench.py
echo done
