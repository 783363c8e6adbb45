# round 5 (ac): --precision bf16 kernel trace
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5ac_bf16_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_r5ac -o run -- python3 bench.py --precision bf16 --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_r5ac/run_results.db --steps 6 --marker adam_k --top 45 > gpurun_out/r5ac_bf16_profile.md
echo done
