# round 5 (ax): --precision bf16 step profile with the library products (the default)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5ax_bf16_bench.log python -u bench.py --precision bf16 &&
run_step 300 gpurun_out/r5ax_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_ax -o run -- python3 bench.py --precision bf16 --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_ax/run_results.db --steps 6 --marker adam_k --top 45 > gpurun_out/r5ax_bf16_step_profile.md
echo done
