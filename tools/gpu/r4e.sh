# round 4 (e): one GEMM family (bf16x6 / bf16x3 linear paths, GradPlanes, pieces removed) + the GEMM
# main loop with cross-barrier fragment prefetch: GEMM tests + speeds first, then the GPU suite,
# smoke, headline + bf16 bench, NER eager / graph with and without the wgrad side stream
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4e_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
run_step 180 gpurun_out/r4e_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 120 gpurun_out/r4e_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run_step 300 gpurun_out/r4e_bench.log python -u bench.py
run_step 300 gpurun_out/r4e_bench_bf16.log python -u bench.py --precision bf16
run_step 900 gpurun_out/r4e_gputests.log python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
run_step 240 gpurun_out/r4e_ner.log python -u tools/bench_ner.py --steps 40
run_step 240 gpurun_out/r4e_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step
run_step 240 gpurun_out/r4e_ner_graph_noside.log python -u tools/bench_ner.py --steps 40 --graph-train-step --no-overlap-wgrad
run_step 240 gpurun_out/r4e_ner_noside.log python -u tools/bench_ner.py --steps 40 --no-overlap-wgrad
echo done
