# round 4 (g): split-K for few-tile GEMMs (fine-tuning sizes) + slab combine with beta / bias;
# NER-size tile sweep; two-register-stage weight gradient; bench; NER probe
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 200 gpurun_out/r4g_gemmtests.log python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gemm_f16_gpu.py
T=2048 CFGS=2:1,2:2,2:4,3:1,3:2,plan run_step 240 gpurun_out/r4g_sweep2048.log python -u tools/probe/gemm_f16_bench.py
T=4096 CFGS=2:1,3:1,plan run_step 240 gpurun_out/r4g_sweep4096.log python -u tools/probe/gemm_f16_bench.py
run_step 180 gpurun_out/r4g_gemm_bench.log python -u tools/probe/gemm_f16_bench.py
run_step 300 gpurun_out/r4g_bench.log python -u bench.py
run_step 300 gpurun_out/r4g_bench_nooverlap.log python -u bench.py --no-overlap-wgrad
run_step 300 gpurun_out/r4g_bench_graph.log python -u bench.py --graph-train-step
run_step 240 gpurun_out/r4g_ner_probe.log python -u tools/probe/ner_graph_probe.py --no-overlap-wgrad
run_step 240 gpurun_out/r4g_ner.log python -u tools/bench_ner.py --steps 40
run_step 300 gpurun_out/r4g_bench_b32.log python -u bench.py --batch 32
export TMPDIR=/tmp
run_step 60 gpurun_out/r4h_counters.txt rocprofv3 -L
ONLY=qkv run_step 90 gpurun_out/r4h_pmc1.log rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_r4h1 -o run -- python3 tools/probe/gemm_f16_bench.py
ONLY=qkv run_step 90 gpurun_out/r4h_pmc2.log rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_r4h2 -o run -- python3 tools/probe/gemm_f16_bench.py
echo done
