# round 5 (bt): phase-2 config (seq 512, batch 32, 80 predictions) with the final tree
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 400 gpurun_out/r5bt_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80 &&
run_step 400 gpurun_out/r5bt_p2_b.log python -u bench.py --seq 512 --batch 32 --max-pred 80
echo done
