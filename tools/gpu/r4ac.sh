# round 4 (ac): bf16 backward reusing the forward's batched W^T (no per-weight conversion in
# the backward): bf16 GPU tests, bf16 bench x2 and a bf16 kernel trace
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 400 gpurun_out/r4ac_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "bf16" tests/
run_step 200 gpurun_out/r4ac_bench_bf16.log python -u bench.py --precision bf16
run_step 200 gpurun_out/r4ac_bench_bf16b.log python -u bench.py --precision bf16
export TMPDIR=/tmp
run_step 240 gpurun_out/r4ac_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4ac -o run -- python3 bench.py --precision bf16 --steps 5 --warmup 3
echo done
