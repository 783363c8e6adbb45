# A/B of which waves issue the large GEMM tile's LDS-DMA (HX_GEMM_DMA_WAVES: 0 every wave, 4 waves
# 0-3, 12 waves 4-7): GEMM tests under each switch, then the headline bench alternated REPS times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for dw in ${TDWS:-}; do
  HX_GEMM_DMA_WAVES=$dw timeout -k 10 300 python -u -m pytest tests/test_gemm_f16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/dw_tests_$dw.log 2>&1 || { tail -30 gpurun_out/dw_tests_$dw.log; exit 1; }
  echo "tests dma_waves=$dw: $(tail -1 gpurun_out/dw_tests_$dw.log)"
done
for rep in $(seq 1 ${REPS:-3}); do
  for dw in 0 ${DWS:-4 12}; do
    HX_GEMM_DMA_WAVES=$dw timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $BENCH_ARGS > gpurun_out/dw_bench_${dw}_$rep.log 2>&1 || { tail -20 gpurun_out/dw_bench_${dw}_$rep.log; exit 1; }
    echo "bench $BENCH_ARGS dma_waves=$dw rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dw_bench_${dw}_$rep.log)"
  done
done
