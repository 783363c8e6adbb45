# round 5 (n): headline bench + kernel trace (wgrad interleave, nt GELU stores, vector fold);
# NER graph-replay update time and its kernel trace (traces in /tmp, summaries in gpurun_out)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5n_bench.log python -u bench.py &&
run_step 300 gpurun_out/r5n_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_r5n -o run -- python3 bench.py --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_r5n/run_results.db --steps 6 --marker adam_k --top 40 > gpurun_out/r5n_step_profile.md &&
run_step 300 gpurun_out/r5n_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step &&
run_step 300 gpurun_out/r5n_ner_prof.log rocprofv3 --kernel-trace -d /tmp/prof_r5n_ner -o run -- python3 tools/bench_ner.py --steps 20 --graph-train-step &&
python tools/prof_summary.py /tmp/prof_r5n_ner/run_results.db --steps 10 --marker adam --top 40 > gpurun_out/r5n_ner_profile.md &&
python tools/ner_gaps.py /tmp/prof_r5n_ner/run_results.db > gpurun_out/r5n_ner_gaps.txt
echo done
