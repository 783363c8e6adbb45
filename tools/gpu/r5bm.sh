# round 5 (bm): attention-output weight gradient (768 x 768 over 16384 tokens): split / tile sweep,
# repeated
set -o pipefail
mkdir -p gpurun_out
ONLY=attn_out WGRAD_PLANS=plan,0:8,0:10,0:14,0:18,0:24,1:9,1:16,1:28,plan,0:8,0:10,0:14,0:18,0:24,1:9,1:16,1:28 \
  timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5bm_attn_out_wgrad.log 2>&1
echo done
