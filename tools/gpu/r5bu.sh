# round 5 (bu): phase-2 attention backward -- cost of the dQ atomics (diagnostic build with plain
# stores, wrong sums) vs the real kernel, alternated
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in old new; do
    S=512 timeout -k 10 120 python -u tools/probe/ext_ab.py tools/probe/ab/_C_$v.so attn_bwd >> gpurun_out/r5bu_ab.log 2>&1 || exit 1
  done
done
echo done
