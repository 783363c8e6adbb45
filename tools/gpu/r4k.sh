# round 4 (k): attention kernels after the DPP wave max / V fragments in LDS / branchy rescale
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 240 gpurun_out/r4k_attn_test.log python -u -m pytest -v --timeout 100 --timeout-method thread tests/test_kernels_gpu.py -k "attention_f16"
run_step 120 gpurun_out/r4k_attn_probe.log python -u tools/probe/attn_bwd_probe.py
echo done
