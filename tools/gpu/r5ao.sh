# round 5 (ao): attention kernels at phase 2 (B32 S512)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 120 gpurun_out/r5ao_attn_p2.log python -u tools/bench_kernels.py --only attn --batch 32 --seq 512
echo done
