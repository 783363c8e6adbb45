# round 5 (t): the NER captured update's graph (dot dump, copied back); fused amax test
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5t_gemmtests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py &&
mkdir -p /tmp/dot && cd /tmp/dot && DEBUG_HIP_GRAPH_DOT_PRINT=1 run_step 300 $GRAFT_REPO_ROOT/gpurun_out/r5t_ner_dot.log python -u $GRAFT_REPO_ROOT/tools/bench_ner.py --steps 5 --graph-train-step && cd $GRAFT_REPO_ROOT &&
cp /tmp/dot/* gpurun_out/ && gzip -f gpurun_out/graph_*dot_print*
echo done
