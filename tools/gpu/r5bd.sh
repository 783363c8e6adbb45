# round 5 (bd): tile plans at the NER shapes (M = 1536 token rows): forward / dgrad per tile config,
# split-K variants, weight-gradient plans
set -o pipefail
mkdir -p gpurun_out
T=1536 CFGS=plan,2,3,0,1,plan,3,2 timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5bd_ner_tiles.log 2>&1 &&
T=1536 CFGS=2:2,3:2,2:3,2:1 timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5bd_ner_splitk.log 2>&1 &&
T=1536 WGRAD_PLANS=plan,0:1,0:2,0:4,1:1,plan timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/r5bd_ner_wgrad.log 2>&1
echo done
