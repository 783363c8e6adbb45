# attention kernels on one GPU: numerics tests, then fp32 / bf16 micro-benchmarks (phase 1 and phase 2 shapes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "attention or bf16" > gpurun_out/attn_tests.log 2>&1
rc=$?
timeout -k 10 120 python -u tools/bench_kernels.py --only attn,attn_bf16 > gpurun_out/attn_bench.log 2>&1 &&
timeout -k 10 120 python -u tools/bench_kernels.py --only attn,attn_bf16 --batch 32 --seq 512 >> gpurun_out/attn_bench.log 2>&1
exit $rc
