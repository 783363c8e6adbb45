# round 4 (l): locate the fp16x3 attention backward's ramp-case dQ error
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 120 gpurun_out/r4l_ramp.log python -u tools/probe/attn_ramp_probe.py
echo done
