# round 5 (ce): producer-side dQKV maxima at S > 128 -- attention tests, phase-2 bench (twice)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention or attn" > gpurun_out/r5ce_tests.log 2>&1 || exit 1
run_step 400 gpurun_out/r5ce_p2_1.log python -u bench.py --seq 512 --batch 32 --max-pred 80 &&
run_step 400 gpurun_out/r5ce_p2_2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
echo done
