# The low-priority weight-gradient side stream below its 8192-row default: GPU tests that cover the
# side stream (graph capture, RCCL reducer, kernels), then --overlap-wgrad vs the default at batch 32
# (4096 rows), BERT-large seq 128 / seq 512 (4096 rows) and NER (graph-captured updates)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_dist_gpu.py tests/test_train_graph_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/prio_tests.log 2>&1 || { tail -30 gpurun_out/prio_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/prio_tests.log)"
for arm in off on; do
  timeout -k 10 400 python -u tools/bench_ner.py --steps 40 --repeats 3 $([ $arm = on ] && echo --overlap-wgrad) > gpurun_out/ner_$arm.log 2>&1 || { tail -20 gpurun_out/ner_$arm.log; exit 1; }
  echo "ner overlap=$arm $(grep -o '"s_per_update_min_median_max": \[[0-9., ]*\]' gpurun_out/ner_$arm.log)"
done
for rep in $(seq 1 ${REPS:-4}); do
  for arm in off on; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --batch 32 $([ $arm = on ] && echo --overlap-wgrad) > gpurun_out/b32_$arm.log 2>&1 || { tail -20 gpurun_out/b32_$arm.log; exit 1; }
    echo "b32 overlap=$arm rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b32_$arm.log)"
  done
done
for rep in 1 2; do
  for arm in off on; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --model large --batch 32 $([ $arm = on ] && echo --overlap-wgrad) > gpurun_out/l128_$arm.log 2>&1 || { tail -20 gpurun_out/l128_$arm.log; exit 1; }
    echo "large128 overlap=$arm rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/l128_$arm.log)"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --model large --seq 512 --batch 8 --max-pred 80 $([ $arm = on ] && echo --overlap-wgrad) > gpurun_out/l512_$arm.log 2>&1 || { tail -20 gpurun_out/l512_$arm.log; exit 1; }
    echo "large512 overlap=$arm rep=$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/l512_$arm.log)"
  done
done
