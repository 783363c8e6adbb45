# round 4 (f): GEMM main-loop forms A/B (PF 0 / 1) + tests, NER profile, phase-2 trace
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4f_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
CFGS=plan/0,plan/1,0/0,0/1,1/0,1/1,2/0,2/1 run_step 240 gpurun_out/r4f_sweep.log python -u tools/probe/gemm_f16_bench.py
HX_GEMM_F16_PF=1 run_step 300 gpurun_out/r4f_bench_pf1.log python -u bench.py
run_step 300 gpurun_out/r4f_bench_pf0.log python -u bench.py
run_step 240 gpurun_out/r4f_ner_probe.log python -u tools/probe/ner_graph_probe.py
run_step 240 gpurun_out/r4f_ner_probe_noside.log python -u tools/probe/ner_graph_probe.py --no-overlap-wgrad
run_step 240 gpurun_out/r4f_ner_probe_bf16.log python -u tools/probe/ner_graph_probe.py --precision bf16
run_step 450 gpurun_out/r4f_prof_p2.log bash tools/prof_run.sh r4f_p2 --seq 512 --batch 32 --max-pred 80
echo done
