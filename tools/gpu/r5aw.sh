# round 5 (aw): attention backward with conflict-free dS / staging LDS accesses -- numerics tests,
# then old / new builds alternated (separate processes) on one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention or attn" > gpurun_out/r5aw_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for v in old new; do
    timeout -k 10 120 python -u tools/probe/ext_ab.py tools/probe/ab/_C_$v.so attn_bwd >> gpurun_out/r5aw_ab.log 2>&1 || exit 1
  done
done
for v in old new; do
  timeout -k 10 120 python -u tools/probe/ext_ab.py tools/probe/ab/_C_$v.so attn_fwd >> gpurun_out/r5aw_ab.log 2>&1 || exit 1
done
echo done
