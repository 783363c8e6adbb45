# round 5 (ab): status numbers -- headline, bf16, NER eager / graph / graph + reducer
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5ab_bench.log python -u bench.py &&
run_step 300 gpurun_out/r5ab_bf16.log python -u bench.py --precision bf16 &&
run_step 300 gpurun_out/r5ab_ner_eager.log python -u tools/bench_ner.py --steps 40 &&
run_step 300 gpurun_out/r5ab_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step &&
run_step 300 gpurun_out/r5ab_ner_graph_reducer.log python -u tools/bench_ner.py --steps 40 --graph-train-step --force-reducer
echo done
