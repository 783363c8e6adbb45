# round 4 (t): 300-update BERT-base parity with the fp16x3 attention (default) and the x6 one;
# GEMM tests on the final gemm_f16 (ring depth as a constant)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4t_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 900 gpurun_out/r4t_parity.log python -u tools/parity_run.py --updates 300 --modes native,native#2,fp16x3,fp16x3:x6 --out gpurun_out/r4t_parity
echo done
