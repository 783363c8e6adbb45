# round 4 (p): weight-gradient side stream A/B with the two-waves-per-SIMD attention (phase 1, phase 2)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4p_bench.log python -u bench.py
run_step 200 gpurun_out/r4p_bench_noov.log python -u bench.py --no-overlap-wgrad
run_step 240 gpurun_out/r4p_bench_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
run_step 240 gpurun_out/r4p_bench_p2_noov.log python -u bench.py --seq 512 --batch 32 --max-pred 80 --no-overlap-wgrad
run_step 200 gpurun_out/r4p_bench_b32_noov.log python -u bench.py --batch 32 --no-overlap-wgrad
echo done
run_step 200 gpurun_out/r4p_bench_bf16.log python -u bench.py --precision bf16
HX_GEMM_F16_CFG=1 run_step 200 gpurun_out/r4p_bench_bf16_cfg1.log python -u bench.py --precision bf16
echo done2
