# round 5 (x): headline bench + trace with the 85 %-fill weight-gradient plan; wgrad plan check
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5x_bench.log python -u bench.py &&
run_step 300 gpurun_out/r5x_prof.log rocprofv3 --kernel-trace --stats -d /tmp/prof_r5x -o run -- python3 bench.py --steps 5 --warmup 3 &&
python tools/prof_summary.py /tmp/prof_r5x/run_results.db --steps 6 --marker adam_k --top 40 > gpurun_out/r5x_step_profile.md &&
WGRAD_PLANS=plan run_step 300 gpurun_out/r5x_wgrad_plan.log python -u tools/probe/gemm_f16_bench.py
echo done
