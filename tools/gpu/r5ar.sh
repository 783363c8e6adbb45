# round 5 (ar): staggered wave halves (cfg 7) -- tests, repeated A/B vs cfg 1
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5ar_gemmtests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py &&
CFGS=1,7,1,7,1,7 run_step 300 gpurun_out/r5ar_stagger_ab.log python -u tools/probe/gemm_f16_bench.py
echo done
