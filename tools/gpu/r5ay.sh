# round 5 (ay): --precision bf16 eager vs graph-captured update (alternated twice on one box)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
for i in 1 2; do
run_step 300 gpurun_out/r5ay_bf16_eager_$i.log python -u bench.py --precision bf16 &&
run_step 300 gpurun_out/r5ay_bf16_graph_$i.log python -u bench.py --precision bf16 --graph-train-step || exit 1
done
echo done
