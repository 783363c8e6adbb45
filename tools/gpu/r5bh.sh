# round 5 (bh): attention forward at three waves per SIMD (old / new builds alternated)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in old new; do
    NO_BIAS=1 timeout -k 10 120 python -u tools/probe/ext_ab.py tools/probe/ab/_C_$v.so attn_fwd >> gpurun_out/r5bh_ab.log 2>&1 || exit 1
  done
done
echo done
