# round 5 (ca): batch 32 eager vs graph-captured update (alternated twice), headline graph check
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
for i in 1 2; do
run_step 300 gpurun_out/r5ca_b32_eager_$i.log python -u bench.py --batch 32 &&
run_step 300 gpurun_out/r5ca_b32_graph_$i.log python -u bench.py --batch 32 --graph-train-step || exit 1
done
run_step 300 gpurun_out/r5ca_b128_graph.log python -u bench.py --graph-train-step
echo done
