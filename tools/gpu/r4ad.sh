# round 4 (ad): bf16 FFN with the GELU in the bf16 GEMM epilogues (no bias_act passes) + the
# backward reusing the forward's W^T: bf16 / GELU GPU tests, bf16 bench x2, bf16 kernel trace
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 500 gpurun_out/r4ad_tests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu -k "bf16 or gelu or ffn" tests/
run_step 200 gpurun_out/r4ad_bench_bf16.log python -u bench.py --precision bf16
run_step 200 gpurun_out/r4ad_bench_bf16b.log python -u bench.py --precision bf16
export TMPDIR=/tmp
run_step 240 gpurun_out/r4ad_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4ad -o run -- python3 bench.py --precision bf16 --steps 5 --warmup 3
echo done
