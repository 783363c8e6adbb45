# round 4 (c): bf16 row-limit fix + graph/reducer tests, standalone GEMM speeds, bf16 / NER /
# phase-2 kernel traces
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r4c_tests.log python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gemm_f16_gpu.py tests/test_determinism_gpu.py tests/test_train_graph_gpu.py
run_step 180 gpurun_out/r4c_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 300 gpurun_out/r4c_bench_bf16.log python -u bench.py --precision bf16
run_step 300 gpurun_out/r4c_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step
run_step 450 gpurun_out/r4c_prof_bf16.log bash tools/prof_run.sh r4c_bf16 --precision bf16
run_step 450 gpurun_out/r4c_prof_ner.log bash tools/prof_ner.sh r4c_ner
run_step 450 gpurun_out/r4c_prof_ner_gr.log bash tools/prof_ner.sh r4c_ner_gr --graph-train-step --force-reducer
run_step 450 gpurun_out/r4c_prof_p2.log bash tools/prof_run.sh r4c_p2 --seq 512 --batch 32 --max-pred 80
echo done
