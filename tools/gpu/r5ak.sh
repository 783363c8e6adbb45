# round 5 (ak): weight-gradient side stream A/B (repeated, one box) with the faster attention
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
for i in 1 2; do
run_step 300 gpurun_out/r5ak_off_$i.log python -u bench.py &&
run_step 300 gpurun_out/r5ak_on_$i.log python -u bench.py --overlap-wgrad || exit 1
done
echo done
