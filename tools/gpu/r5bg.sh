# round 5 (bg): LayerNorm dropout decisions recorded in the forward, replayed in the backward --
# tests, kernel probe, headline / bf16 step A/B (HX_LN_DROP_RECORD=0 / 1)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_gemm_f16_gpu.py -k "ln or layernorm or layer_norm or bert or model" > gpurun_out/r5bg_tests.log 2>&1 || exit 1
for i in 1 2; do
HX_LN_DROP_RECORD=0 run_step 300 gpurun_out/r5bg_bf16_old_$i.log python -u bench.py --precision bf16 &&
HX_LN_DROP_RECORD=1 run_step 300 gpurun_out/r5bg_bf16_new_$i.log python -u bench.py --precision bf16 || exit 1
done
HX_LN_DROP_RECORD=0 run_step 300 gpurun_out/r5bg_fp32_old.log python -u bench.py &&
HX_LN_DROP_RECORD=1 run_step 300 gpurun_out/r5bg_fp32_new.log python -u bench.py
echo done
