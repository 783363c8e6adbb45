# round 5 (bx): token-type gradient kernel -- tests (kernel + embedding / model paths), bench fp32 / bf16
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_determinism_gpu.py tests/test_parity_gpu.py > gpurun_out/r5bx_tests.log 2>&1 || exit 1
run_step 300 gpurun_out/r5bx_fp32.log python -u bench.py &&
run_step 300 gpurun_out/r5bx_bf16.log python -u bench.py --precision bf16
echo done
