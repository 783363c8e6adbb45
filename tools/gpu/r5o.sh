# round 5 (o): NER graph-replay update -- host time split (batch fetch vs train_step call) and a
# cProfile of 20 replayed updates; narrower fold blocks (kernel tests + step trace)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 400 gpurun_out/r5o_kerneltests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py &&
run_step 300 gpurun_out/r5o_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step --cprofile gpurun_out/r5o_ner_graph_cprof.txt &&
run_step 300 gpurun_out/r5o_ner_eager.log python -u tools/bench_ner.py --steps 40 &&
run_step 300 gpurun_out/r5o_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_r5o -o run -- python3 bench.py --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_r5o/run_results.db --steps 6 --marker adam_k --top 40 > gpurun_out/r5o_step_profile.md
echo done
