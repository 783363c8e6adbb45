# round 4 (ak): final-tree benches (headline, batch 32, phase 2, bf16, NER eager / graph)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4ak_bench.log python -u bench.py
run_step 200 gpurun_out/r4ak_bench_b32.log python -u bench.py --batch 32
run_step 240 gpurun_out/r4ak_bench_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
run_step 200 gpurun_out/r4ak_bench_bf16.log python -u bench.py --precision bf16
run_step 200 gpurun_out/r4ak_ner.log python -u tools/bench_ner.py --steps 40
run_step 200 gpurun_out/r4ak_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step
echo done
