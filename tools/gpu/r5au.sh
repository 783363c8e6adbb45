# round 5 (au): step kernel profiles with and without the LayerNorm-written GEMM pieces
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
HX_PRESPLIT=0 run_step 300 gpurun_out/r5au_prof_off.log rocprofv3 --kernel-trace --stats -d /tmp/prof_off -o run -- python3 bench.py --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_off/run_results.db --steps 6 --marker adam_k --top 45 > gpurun_out/r5au_profile_off.md &&
HX_PRESPLIT=1 run_step 300 gpurun_out/r5au_prof_on.log rocprofv3 --kernel-trace --stats -d /tmp/prof_on -o run -- python3 bench.py --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_on/run_results.db --steps 6 --marker adam_k --top 45 > gpurun_out/r5au_profile_on.md
echo done
