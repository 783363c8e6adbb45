# round 5 (r): M = 4096 (batch 32) tile plans; NER captured update: kernels + memory copies
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
T=4096 CFGS=2,4,6,6:2,6:4,0,1 run_step 300 gpurun_out/r5r_m4096_sweep.log python -u tools/probe/gemm_f16_bench.py &&
run_step 300 gpurun_out/r5r_ner_prof.log rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/prof_r5r_ner -o run -- python3 tools/bench_ner.py --steps 20 --graph-train-step &&
python tools/trace_tables.py /tmp/prof_r5r_ner/run_results.db > gpurun_out/r5r_ner_tables.txt &&
python tools/ner_gaps.py /tmp/prof_r5r_ner/run_results.db --last 1000 > gpurun_out/r5r_ner_gaps.txt
echo done
