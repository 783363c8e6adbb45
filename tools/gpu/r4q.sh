# round 4 (q): headline kernel trace with the weight gradients on the compute stream (new default)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r4q_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4q -o run -- python3 bench.py --steps 5 --warmup 3
echo done
