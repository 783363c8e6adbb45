# round 5 (ae): captured-update replay at batch 128 and 32 vs eager (same box)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5ae_b128_eager.log python -u bench.py &&
run_step 300 gpurun_out/r5ae_b128_graph.log python -u bench.py --graph-train-step &&
run_step 300 gpurun_out/r5ae_b32_eager.log python -u bench.py --batch 32 &&
run_step 300 gpurun_out/r5ae_b32_graph.log python -u bench.py --batch 32 --graph-train-step
echo done
