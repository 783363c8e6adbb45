# round 5 (at): LayerNorm-written GEMM operand pieces -- numerics tests, then the headline step
# A/B (HX_PRESPLIT=0 / 1, alternated twice on one box)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5at_tests.log 2>&1 || exit 1
for i in 1 2; do
HX_PRESPLIT=0 run_step 300 gpurun_out/r5at_off_$i.log python -u bench.py &&
HX_PRESPLIT=1 run_step 300 gpurun_out/r5at_on_$i.log python -u bench.py || exit 1
done
echo done
