# Weight-gradient / GEMM plans for fewer workgroup slots than CUs (bench.py --reserve-cus R: the
# one-workgroup-per-CU side-stream weight gradients then leave R CUs free for the compute stream's
# LayerNorm / attention backward), alternated REPS times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for r in ${RS:-0 16 32}; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --reserve-cus $r $BENCH_ARGS > gpurun_out/res_$r.log 2>&1 || { tail -20 gpurun_out/res_$r.log; exit 1; }
    echo "bench $BENCH_ARGS reserve=$r rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/res_$r.log)"
  done
done
