# round 5 (m): interleaved wgrad split (tests + per-shape times); epilogue store cache policy
# (cfg 11 nt, 12 sc0 sc1 vs 6), full and epilogue-only; vectorised fold (kernel tests)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5m_gemmtests.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py &&
run_step 400 gpurun_out/r5m_kerneltests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py &&
run_step 200 gpurun_out/r5m_main.log python -u tools/probe/gemm_f16_bench.py &&
CFGS=6,11,12,6 run_step 200 gpurun_out/r5m_full.log python -u tools/probe/gemm_f16_bench.py &&
HX_GEMM_DIAG=2 CFGS=6,11,12 run_step 200 gpurun_out/r5m_noloop.log python -u tools/probe/gemm_f16_bench.py
echo done
run_step 300 gpurun_out/r5m_ner_graph.log python -u tools/bench_ner.py --steps 40 --graph-train-step --profile-phases --cprofile gpurun_out/r5m_ner_graph_cprof.txt &&
run_step 300 gpurun_out/r5m_ner_eager.log python -u tools/bench_ner.py --steps 40 --profile-phases --cprofile gpurun_out/r5m_ner_eager_cprof.txt
echo done2
