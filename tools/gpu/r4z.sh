# round 4 (z): kernel traces of the verdict's three library-free checks -- phase 1 batch 32,
# NER fine-tuning, --precision bf16 (no Cijk_* library GEMM above 0.05 ms/step)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 240 gpurun_out/r4z_prof_b32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4z_b32 -o run -- python3 bench.py --batch 32 --steps 5 --warmup 3
run_step 240 gpurun_out/r4z_prof_ner.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4z_ner -o run -- python3 tools/bench_ner.py --steps 6 --warmup 2
run_step 240 gpurun_out/r4z_prof_bf16.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4z_bf16 -o run -- python3 bench.py --precision bf16 --steps 5 --warmup 3
echo done
