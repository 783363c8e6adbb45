# batch 32 (4096 token rows): --overlap-wgrad (the low-priority, CU-reserving side stream) vs the
# default compute stream only, alternated REPS times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-4}); do
  for arm in off on; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --batch 32 $([ $arm = on ] && echo --overlap-wgrad) $BENCH_ARGS > gpurun_out/b32_$arm.log 2>&1 || { tail -20 gpurun_out/b32_$arm.log; exit 1; }
    echo "b32 $BENCH_ARGS overlap=$arm rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b32_$arm.log)"
  done
done
