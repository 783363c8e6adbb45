# round 5 (k): headline kernel trace on the per-row-scale tree
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5k_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5k -o run -- python3 bench.py --steps 5 --warmup 3
echo done
