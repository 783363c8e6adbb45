# round 4: fp16x3 across the BASELINE configs + 300-update parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --fp32-gemm fp16x3 --batch 32 > gpurun_out/r4b_bench_f16_b32.log 2>&1 &&
timeout -k 10 300 python -u bench.py --fp32-gemm fp16x3 --seq 512 --batch 32 --max-pred 80 > gpurun_out/r4b_bench_f16_p2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --precision bf16 > gpurun_out/r4b_bench_bf16.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_ner.py --fp32-gemm fp16x3 --steps 40 > gpurun_out/r4b_ner_f16.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_ner.py --fp32-gemm fp16x3 --steps 40 --graph-train-step --force-reducer > gpurun_out/r4b_ner_f16_graph_reducer.log 2>&1 &&
timeout -k 10 900 python -u tools/parity_run.py --updates 300 --modes native,native#2,bf16x6,fp16x3 --out gpurun_out/r4b_parity > gpurun_out/r4b_parity.log 2>&1
