# round 4 (d): 128x192 two-per-CU tile tests + tile sweep, NER host profiles (eager / graph)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4d_tests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
CFGS=plan,0,1,2,4 run_step 240 gpurun_out/r4d_sweep.log python -u tools/probe/gemm_f16_bench.py
run_step 240 gpurun_out/r4d_ner_cprof.log python -u tools/bench_ner.py --steps 30 --cprofile gpurun_out/r4d_ner_cprof.txt
run_step 240 gpurun_out/r4d_ner_graph_cprof.log python -u tools/bench_ner.py --steps 30 --graph-train-step --cprofile gpurun_out/r4d_ner_graph_cprof.txt
echo done
