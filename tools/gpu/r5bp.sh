# round 5 (bp): split-K at batch 32 (M = 4096): plan vs forced slab counts on the 256 x 192 tile, repeated
set -o pipefail
mkdir -p gpurun_out
T=4096 CFGS=plan,1:1,1:2,1:3,1:4,plan,1:1,1:2,1:3,1:4 timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5bp_b32_splitk.log 2>&1
echo done
