# round 5 (cf): validation of the committed tree -- full GPU suite, smoke(), headline / bf16 / batch-32 bench
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5cf_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5cf_smoke.log 2>&1 || exit 1
run_step 300 gpurun_out/r5cf_bench.log python -u bench.py &&
run_step 300 gpurun_out/r5cf_bench_bf16.log python -u bench.py --precision bf16 &&
run_step 300 gpurun_out/r5cf_bench_b32.log python -u bench.py --batch 32
echo done
