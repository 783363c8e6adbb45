# round 5 (am): --precision bf16 with the plain / beta products on hipBLASLt (A/B: HX_BF16_LIB=0 = all on
# the hand-written kernel), then the GPU suite
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
for i in 1 2; do
HX_BF16_LIB=0 run_step 300 gpurun_out/r5am_bf16_own_$i.log python -u bench.py --precision bf16 &&
run_step 300 gpurun_out/r5am_bf16_lib_$i.log python -u bench.py --precision bf16 || exit 1
done
run_step 900 gpurun_out/r5am_gpu_suite.log python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests
echo done
