set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1
echo "tests rc=$?"
for m in bf16x3 bf16x6; do
timeout -k 10 300 python -u bench.py --fp32-gemm $m > gpurun_out/bench_$m.log 2>&1 || exit 1
done
