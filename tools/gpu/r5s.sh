# round 5 (s): graph replay cost vs dirty bytes per node; NER graph dot dump; batch 32 with the new plan
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 120 gpurun_out/r5s_g_1k.log python -u tools/probe/graph_replay_probe.py --numel 1024 &&
run_step 120 gpurun_out/r5s_g_4m.log python -u tools/probe/graph_replay_probe.py --numel 4194304 --reps 20 &&
mkdir -p /tmp/dot && cd /tmp/dot && DEBUG_HIP_GRAPH_DOT_PRINT=1 run_step 300 $GRAFT_REPO_ROOT/gpurun_out/r5s_ner_dot.log python -u $GRAFT_REPO_ROOT/tools/bench_ner.py --steps 10 --graph-train-step && cd $GRAFT_REPO_ROOT &&
(ls -la /tmp/dot > gpurun_out/r5s_dot_ls.txt; for f in /tmp/dot/*.dot; do [ -f "$f" ] && grep -o 'label="[A-Za-z_]*' "$f" | sort | uniq -c | sort -rn | head -30 >> gpurun_out/r5s_dot_nodes.txt; done; true) &&
run_step 300 gpurun_out/r5s_b32.log python -u bench.py --batch 32
echo done
run_step 300 gpurun_out/r5s_gemmtests.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_f16_gpu.py &&
run_step 400 gpurun_out/r5s_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
echo done2
