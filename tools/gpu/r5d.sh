# round 5 (d): DMA pieces interleaved with MFMAs (cfg 1) vs a DMA burst (cfg 6), 5-stage ring (cfg 7)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5d_gemmtests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py -k "every_tile or forward or gelu"
CFGS=1,6,7,0,1,6 run_step 300 gpurun_out/r5d_sweep.log python -u tools/probe/gemm_f16_bench.py
echo done
