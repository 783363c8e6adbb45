# round 5 (y): weight-gradient split counts A/B on one box, repeated
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
WGRAD_PLANS=1:6,1:7,1:8,1:9,1:6,1:7,1:8,1:9 run_step 300 gpurun_out/r5y_wgrad_ab.log python -u tools/probe/gemm_f16_bench.py
echo done
