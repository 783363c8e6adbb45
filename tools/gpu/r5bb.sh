# round 5 (bb): LayerNorm kernels with and without dropout (Philox regeneration cost)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for k in 0.9 1.0; do
    KEEP=$k HX_EXT_SO=tools/probe/ab/_C_old.so timeout -k 10 120 python -u tools/probe/ln_probe.py >> gpurun_out/r5bb_ln_keep.log 2>&1 || exit 1
  done
done
echo done
