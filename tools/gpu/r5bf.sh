# round 5 (bf): Q/K/V bias in the projection GEMM's epilogue (attention adds nothing, still returns
# the bias gradient) -- GPU suite, then headline / bf16 step A/B (HX_QKV_BIAS_EPILOGUE=0 / 1)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bf_tests.log 2>&1 || exit 1
for i in 1 2; do
HX_QKV_BIAS_EPILOGUE=0 run_step 300 gpurun_out/r5bf_fp32_old_$i.log python -u bench.py &&
HX_QKV_BIAS_EPILOGUE=1 run_step 300 gpurun_out/r5bf_fp32_new_$i.log python -u bench.py || exit 1
done
HX_QKV_BIAS_EPILOGUE=0 run_step 300 gpurun_out/r5bf_bf16_old.log python -u bench.py --precision bf16 &&
HX_QKV_BIAS_EPILOGUE=1 run_step 300 gpurun_out/r5bf_bf16_new.log python -u bench.py --precision bf16
echo done
