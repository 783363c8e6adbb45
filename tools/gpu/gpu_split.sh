set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1 &&
for b in 32 128; do for m in bf16x6 bf16x3; do
timeout -k 10 300 python -u bench.py --batch $b --fp32-gemm $m > gpurun_out/b_${b}_$m.log 2>&1 || exit 1
echo "batch $b $m $(tail -n 1 gpurun_out/b_${b}_$m.log | cut -c 150-230)"
done; done
