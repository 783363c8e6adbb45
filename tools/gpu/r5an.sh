# round 5 (an): headline trace after the attention changes; batch 32, phase 2 and NER numbers
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5an_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_r5an -o run -- python3 bench.py --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_r5an/run_results.db --steps 6 --marker adam_k --top 40 > gpurun_out/r5an_step_profile.md &&
run_step 300 gpurun_out/r5an_bench.log python -u bench.py &&
run_step 300 gpurun_out/r5an_b32.log python -u bench.py --batch 32 &&
run_step 400 gpurun_out/r5an_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80 &&
run_step 300 gpurun_out/r5an_ner.log python -u tools/bench_ner.py --steps 40 &&
run_step 300 gpurun_out/r5an_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step
echo done
