# round 5 (bn): 256 wgrad tile for the attention-output gradient -- tests, step A/B
# (HX_WGRAD_FEW256=0 / 1, alternated twice), batch 32 check
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py \
  -k "wgrad" > gpurun_out/r5bn_tests.log 2>&1 || exit 1
ONLY=attn_out WGRAD_PLANS=plan,0:14,plan,0:14 timeout -k 10 120 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5bn_plan.log 2>&1 &&
for i in 1 2; do
HX_WGRAD_FEW256=0 run_step 300 gpurun_out/r5bn_old_$i.log python -u bench.py &&
HX_WGRAD_FEW256=1 run_step 300 gpurun_out/r5bn_new_$i.log python -u bench.py || exit 1
done
run_step 300 gpurun_out/r5bn_b32.log python -u bench.py --batch 32
echo done
