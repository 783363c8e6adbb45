# round 5 (p): HIP graph replay cost per node under the runtime's graph settings; NER update with them
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 60 gpurun_out/r5p_mfma_shape.log ./tools/probe/mfma_shape_probe &&
run_step 120 gpurun_out/r5p_g_default.log python -u tools/probe/graph_replay_probe.py &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 run_step 120 gpurun_out/r5p_g_pc1.log python -u tools/probe/graph_replay_probe.py &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run_step 120 gpurun_out/r5p_g_pc0.log python -u tools/probe/graph_replay_probe.py &&
DEBUG_HIP_GRAPH_BATCH_SIZE=1000 run_step 120 gpurun_out/r5p_g_bs1000.log python -u tools/probe/graph_replay_probe.py &&
DEBUG_HIP_FORCE_GRAPH_QUEUES=1 run_step 120 gpurun_out/r5p_g_fq1.log python -u tools/probe/graph_replay_probe.py
echo done
run_step 300 gpurun_out/r5p_b32.log python -u bench.py --batch 32 &&
run_step 400 gpurun_out/r5p_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
echo done2
