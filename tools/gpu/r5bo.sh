# round 5 (bo): batch-32 step profile
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5bo_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_bo -o run -- python3 bench.py --batch 32 --steps 10 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_bo/run_results.db --steps 11 --marker adam_k --top 40 > gpurun_out/r5bo_b32_step_profile.md
echo done
