set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --fp32-gemm bf16x3 --overlap-wgrad > gpurun_out/b_ov.log 2>&1 || exit 1
echo "overlap $(tail -n 1 gpurun_out/b_ov.log | cut -c 150-230)"
timeout -k 10 200 python -u bench.py --fp32-gemm bf16x3 > gpurun_out/b_noov.log 2>&1 || exit 1
echo "no-overlap $(tail -n 1 gpurun_out/b_noov.log | cut -c 150-230)"
