# round 5 (bi): NER fine-tuning update with the final tree (eager, graph, graph + reducer)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5bi_ner_eager.log python -u tools/bench_ner.py &&
run_step 300 gpurun_out/r5bi_ner_graph.log python -u tools/bench_ner.py --graph-train-step &&
run_step 300 gpurun_out/r5bi_ner_graph_reducer.log python -u tools/bench_ner.py --graph-train-step --force-reducer &&
run_step 300 gpurun_out/r5bi_ner_eager2.log python -u tools/bench_ner.py
echo done
