# round 4 (n): benches on the final tree (headline, fp16x3 attention, batch 32, phase 2 both
# attention kernels, bf16, NER eager / graph) and the headline kernel trace
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4n_bench.log python -u bench.py
run_step 200 gpurun_out/r4n_bench_attnx6.log python -u bench.py --fp32-attention x6
run_step 200 gpurun_out/r4n_bench_b32.log python -u bench.py --batch 32
run_step 240 gpurun_out/r4n_bench_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
run_step 240 gpurun_out/r4n_bench_p2_x6.log python -u bench.py --seq 512 --batch 32 --max-pred 80 --fp32-attention x6
run_step 200 gpurun_out/r4n_bench_bf16.log python -u bench.py --precision bf16
run_step 200 gpurun_out/r4n_ner.log python -u tools/bench_ner.py --steps 40
run_step 200 gpurun_out/r4n_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step
export TMPDIR=/tmp
run_step 240 gpurun_out/r4n_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4n -o run -- python3 bench.py --steps 5 --warmup 3
echo done
