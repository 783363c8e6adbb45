# round 4 (ag): bf16 plan on cfg 1 + fused bf16 FFN: tests, bench, and the same bench with the bf16
# FFN fusion switched off (A/B in one call), then a bf16 kernel trace
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 500 gpurun_out/r4ag_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "bf16 or gelu or ffn" tests/
run_step 200 gpurun_out/r4ag_bench_bf16.log python -u bench.py --precision bf16
run_step 200 gpurun_out/r4ag_bench_bf16_unfused.log python -u -c "import sys, runpy; import hetseq_9cme_amd.ops.fused as f; f._ffn_bf16_ok = lambda *a: False; sys.argv = ['bench.py', '--precision', 'bf16']; runpy.run_path('bench.py', run_name='__main__')"
run_step 200 gpurun_out/r4ag_bench_bf16b.log python -u bench.py --precision bf16
run_step 200 gpurun_out/r4ag_bench_bf16_unfusedb.log python -u -c "import sys, runpy; import hetseq_9cme_amd.ops.fused as f; f._ffn_bf16_ok = lambda *a: False; sys.argv = ['bench.py', '--precision', 'bf16']; runpy.run_path('bench.py', run_name='__main__')"
export TMPDIR=/tmp
run_step 240 gpurun_out/r4ag_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4ag -o run -- python3 bench.py --precision bf16 --steps 5 --warmup 3
echo done
