# round 5 (bz): the non-package kernels of one headline step, with their neighbours
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
export TMPDIR=/tmp
run_step 300 gpurun_out/r5bz_prof.log rocprofv3 --kernel-trace -d /tmp/prof_bz -o run -- python3 bench.py --steps 3 --warmup 2 &&
python tools/small_kernels.py /tmp/prof_bz/run_results.db > gpurun_out/r5bz_small_kernels.txt
echo done
