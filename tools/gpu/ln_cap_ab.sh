# LayerNorm grid caps (HX_LN_FWD_CAP / HX_LN_BWD_CAP: workgroups of 4 row-waves; below the row
# count the waves grid-stride with one row of look-ahead): LN tests at the smallest caps, the
# kernel probe over FCAPS x BCAPS, then the headline bench alternated over BENCH_CAPS REPS times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
HX_LN_FWD_CAP=64 HX_LN_BWD_CAP=64 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_f16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "layernorm or embed_ln or ln" > gpurun_out/ln_tests.log 2>&1 || { tail -30 gpurun_out/ln_tests.log; exit 1; }
echo "tests caps 64: $(tail -1 gpurun_out/ln_tests.log)"
for f in ${FCAPS:-4096 2048 1024 512}; do
  for b in ${BCAPS:-512}; do
    HX_LN_FWD_CAP=$f HX_LN_BWD_CAP=$b timeout -k 10 120 python -u tools/probe/ln_probe.py >> gpurun_out/ln_probe.log 2>&1 || { tail -20 gpurun_out/ln_probe.log; exit 1; }
  done
done
cat gpurun_out/ln_probe.log
for rep in $(seq 1 ${REPS:-2}); do
  for fb in ${BENCH_CAPS:-4096:512}; do
    f=${fb%%:*}; b=${fb##*:}
    HX_LN_FWD_CAP=$f HX_LN_BWD_CAP=$b timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $BENCH_ARGS > gpurun_out/ln_bench_${f}_${b}_$rep.log 2>&1 || { tail -20 gpurun_out/ln_bench_${f}_${b}_$rep.log; exit 1; }
    echo "bench $BENCH_ARGS fwd=$f bwd=$b rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ln_bench_${f}_${b}_$rep.log)"
  done
done
