# round 5 (av): headline step A/B of the LayerNorm-written GEMM pieces: off / forward only / forward
# and backward, alternated three times on one box
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
for i in 1 2 3; do
HX_PRESPLIT=0 run_step 300 gpurun_out/r5av_p0_$i.log python -u bench.py &&
HX_PRESPLIT=1 run_step 300 gpurun_out/r5av_p1_$i.log python -u bench.py &&
HX_PRESPLIT=2 run_step 300 gpurun_out/r5av_p2_$i.log python -u bench.py || exit 1
done
echo done
