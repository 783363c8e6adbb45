# round 4 (af): FFN epilogue probe (bf16 dgelu dmode 0 added) and the bf16 step on the 64 x 96-wave
# 256 x 192 tile (cfg 1) for every GEMM vs the plan
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r4af_probe.log python -u tools/probe/ffn_epilogue_probe.py
run_step 200 gpurun_out/r4af_bench_bf16.log python -u bench.py --precision bf16
HX_GEMM_F16_CFG=1 run_step 200 gpurun_out/r4af_bench_bf16_cfg1.log python -u bench.py --precision bf16
echo done
