# round 5 (ai): attention kernels with the QKV bias staged in LDS and transposing max-reductions --
# tests and standalone times
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 400 gpurun_out/r5ai_kerneltests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py &&
run_step 120 gpurun_out/r5ai_attn_times.log python -u tools/bench_kernels.py --only attn &&
run_step 300 gpurun_out/r5ai_bench.log python -u bench.py
echo done
