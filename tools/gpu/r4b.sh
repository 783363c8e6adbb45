# round 4 (b): bf16 determinism probe, the two failing GPU tests, fp16x3 across the BASELINE
# configs (now the default), bf16, NER graph + reducer, and the 300-update parity run
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 240 gpurun_out/r4b_probe.log python -u tools/probe/bf16_det_probe.py
run_step 400 gpurun_out/r4b_tests.log python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_train_graph_gpu.py tests/test_determinism_gpu.py tests/test_optim_mask_gpu.py
run_step 120 gpurun_out/r4b_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run_step 300 gpurun_out/r4b_bench.log python -u bench.py
run_step 300 gpurun_out/r4b_bench_b32.log python -u bench.py --batch 32
run_step 300 gpurun_out/r4b_bench_p2.log python -u bench.py --seq 512 --batch 32 --max-pred 80
run_step 300 gpurun_out/r4b_bench_bf16.log python -u bench.py --precision bf16
run_step 300 gpurun_out/r4b_ner.log python -u tools/bench_ner.py --steps 40
run_step 300 gpurun_out/r4b_ner_graph_reducer.log python -u tools/bench_ner.py --steps 40 --graph-train-step --force-reducer
run_step 900 gpurun_out/r4b_parity.log python -u tools/parity_run.py --updates 300 \
  --modes native,native#2,bf16x6,fp16x3 --out gpurun_out/r4b_parity
echo done
