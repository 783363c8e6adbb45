# round 5 (be): one barrier per two k steps (cfg 7 / 8) -- tile tests, then repeated A/B vs cfg 1 / 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py \
  -k "every_tile or presplit" > gpurun_out/r5be_tests.log 2>&1 || exit 1
CFGS=1,7,1,7,1,7 timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5be_cfg7_ab.log 2>&1 &&
T=4096 CFGS=2,8,1,7,2,8,1,7 timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5be_cfg8_m4096_ab.log 2>&1
echo done
