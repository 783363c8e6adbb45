# round 4 (v): headline bench repeat on one box (default, x6 attention, default again)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4v_bench1.log python -u bench.py
run_step 200 gpurun_out/r4v_bench_x6.log python -u bench.py --fp32-attention x6
run_step 200 gpurun_out/r4v_bench2.log python -u bench.py
run_step 200 gpurun_out/r4v_bench_ov.log python -u bench.py --overlap-wgrad
echo done
