# round 5 (o): NER graph-replay update -- host time split (batch fetch vs train_step call) and a
# cProfile of 20 replayed updates
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5o_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step --cprofile gpurun_out/r5o_ner_graph_cprof.txt &&
run_step 300 gpurun_out/r5o_ner_eager.log python -u tools/bench_ner.py --steps 40
echo done
