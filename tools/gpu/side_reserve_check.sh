set -o pipefail; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_dist_gpu.py tests/test_train_graph_gpu.py tests/test_gemm_f16_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v2_tests.log 2>&1 || { tail -30 gpurun_out/v2_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/v2_tests.log)"
ARMS="r0:HX_SIDE_RESERVE=0 auto:" REPS=2 BENCH_ARGS="--model large --batch 32" bash tools/gpu/env_ab.sh || exit 1
ARMS="r0:HX_SIDE_RESERVE=0 auto:" REPS=1 BENCH_ARGS="--model large --seq 512 --batch 8 --max-pred 80" bash tools/gpu/env_ab.sh || exit 1
ARMS="auto:" REPS=2 bash tools/gpu/env_ab.sh || exit 1
timeout -k 10 400 python -u tools/bench_ner.py --steps 40 --repeats 3 > gpurun_out/v2_ner.log 2>&1 || { tail -20 gpurun_out/v2_ner.log; exit 1; }
echo "ner $(grep -o '"s_per_update_min_median_max": \[[0-9., ]*\]' gpurun_out/v2_ner.log)"
