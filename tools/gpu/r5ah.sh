# round 5 (ah): attention forward cost of the scale producers and the QKV bias
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 120 gpurun_out/r5ah_attn_times.log python -u tools/bench_kernels.py --only attn
echo done
