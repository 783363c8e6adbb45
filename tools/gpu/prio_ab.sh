# A/B of stream priorities for the weight-gradient overlap, alternated REPS times:
#   base   -- compute (default) and side stream at normal priority
#   chigh  -- the training step on a high-priority stream (HX_COMPUTE_PRIO=1)
#   slow   -- the side stream at LOW priority (HX_SIDE_PRIO=low; HIP range printed first)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -c "from hetseq_9cme_amd.ops._ext import C; print('HIP stream priority range (least, greatest):', C().stream_priority_range())"
for rep in $(seq 1 ${REPS:-3}); do
  for arm in ${ARMS:-base chigh slow}; do
    case $arm in
      base) e="HX_SIDE_PRIO=normal";; chigh) e="HX_SIDE_PRIO=normal HX_COMPUTE_PRIO=1";; slow) e="HX_SIDE_PRIO=low";; both) e="HX_COMPUTE_PRIO=1 HX_SIDE_PRIO=low";;
    esac
    env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $BENCH_ARGS > gpurun_out/prio_${arm}_$rep.log 2>&1 || { tail -20 gpurun_out/prio_${arm}_$rep.log; exit 1; }
    echo "bench $BENCH_ARGS $arm rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/prio_${arm}_$rep.log)"
  done
done
