# round 5 (ap): attention forward with the K / V bias in registers -- tests, phase-1 and phase-2 times
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 400 gpurun_out/r5ap_kerneltests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py &&
run_step 120 gpurun_out/r5ap_attn_p1.log python -u tools/bench_kernels.py --only attn &&
run_step 120 gpurun_out/r5ap_attn_p2.log python -u tools/bench_kernels.py --only attn --batch 32 --seq 512
echo done
