# Generic alternated A/B over environment settings: ARMS="name1:VAR=v,VAR2=w name2:VAR=x ..." (an
# arm with no assignments is "name:"); bench.py --steps 20 --warmup 5 $BENCH_ARGS, REPS rounds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for arm in $ARMS; do
    name=${arm%%:*}; vars=${arm#*:}
    env $(echo "$vars" | tr ',' ' ') timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $BENCH_ARGS > gpurun_out/envab_$name.log 2>&1 || { tail -20 gpurun_out/envab_$name.log; exit 1; }
    echo "bench $BENCH_ARGS $name rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/envab_$name.log)"
  done
done
