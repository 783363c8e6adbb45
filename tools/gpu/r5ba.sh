# round 5 (ba): LayerNorm backward with two rows of look-ahead -- tests, old / new builds alternated
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_gemm_f16_gpu.py -k "ln or layernorm or layer_norm" > gpurun_out/r5ba_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in old new; do
    HX_EXT_SO=tools/probe/ab/_C_$v.so timeout -k 10 120 python -u tools/probe/ln_probe.py >> gpurun_out/r5ba_ln_ab.log 2>&1 || exit 1
  done
done
echo done
