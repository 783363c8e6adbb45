# round 5 (br): small-M tile plan (decoder at batch 32) -- GEMM tests, decoder plan check, batch-32 /
# headline benches
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py > gpurun_out/r5br_tests.log 2>&1 || exit 1
M=640 CFGS=plan,1,2 timeout -k 10 200 python -u tools/probe/decoder_tiles.py > gpurun_out/r5br_decoder.log 2>&1 &&
run_step 300 gpurun_out/r5br_b32_1.log python -u bench.py --batch 32 &&
run_step 300 gpurun_out/r5br_b128.log python -u bench.py &&
run_step 300 gpurun_out/r5br_b32_2.log python -u bench.py --batch 32
echo done
