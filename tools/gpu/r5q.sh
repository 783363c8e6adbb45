# round 5 (q): NER captured-update device time; batch-32 and phase-2 kernel traces
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5q_ner_graph.log python -u tools/bench_ner.py --steps 30 --graph-train-step &&
run_step 300 gpurun_out/r5q_b32_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_r5q_b32 -o run -- python3 bench.py --batch 32 --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_r5q_b32/run_results.db --steps 6 --marker adam_k --top 40 > gpurun_out/r5q_b32_profile.md &&
run_step 400 gpurun_out/r5q_p2_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_r5q_p2 -o run -- python3 bench.py --seq 512 --batch 32 --max-pred 80 --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_r5q_p2/run_results.db --steps 6 --marker adam_k --top 40 > gpurun_out/r5q_p2_profile.md
echo done
