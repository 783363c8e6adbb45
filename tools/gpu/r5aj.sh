# round 5 (aj): attention backward cost of the bias gradient and the scale producers
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 120 gpurun_out/r5aj_attn_times.log python -u tools/bench_kernels.py --only attn
echo done
