# round 4 (u): fp16x3 attention at fine-tuning sizes -- NER (eager / graph), graph-update tests,
# attention op tests, headline bench
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r4u_tests.log python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_train_graph_gpu.py tests/test_kernels_gpu.py -k "graph or attention"
run_step 200 gpurun_out/r4u_ner.log python -u tools/bench_ner.py --steps 40
run_step 200 gpurun_out/r4u_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step
run_step 200 gpurun_out/r4u_bench.log python -u bench.py
echo done
