# round 4 (i): fp16x3 attention backward (test + probe); split-K / NER-size sweeps; two-stage
# weight gradient; bench (default, graph-replayed update); NER
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 240 gpurun_out/r4i_attn_test.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_kernels_gpu.py -k "attention_f16 or attention_x6_backward"
run_step 120 gpurun_out/r4i_attn_probe.log python -u tools/probe/attn_bwd_probe.py
run_step 200 gpurun_out/r4i_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
T=2048 CFGS=2:1,2:2,2:4,3:1,3:2,plan run_step 150 gpurun_out/r4i_sweep2048.log python -u tools/probe/gemm_f16_bench.py
run_step 150 gpurun_out/r4i_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 200 gpurun_out/r4i_bench.log python -u bench.py
run_step 200 gpurun_out/r4i_bench_graph.log python -u bench.py --graph-train-step
run_step 200 gpurun_out/r4i_ner.log python -u tools/bench_ner.py --steps 40
echo done
