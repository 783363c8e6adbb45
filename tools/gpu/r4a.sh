# round 4, first call: the fp16x3 kernels' numerics, the fp16x3 bench + kernel trace, then the tree's state
mkdir -p gpurun_out
source tools/gpu/run_step.sh
run_step 400 gpurun_out/r4a_f16.log python -u -m pytest tests/test_gemm_f16_gpu.py -v -s --timeout 120 --timeout-method thread
run_step 300 gpurun_out/r4a_bench_f16.log python -u bench.py --fp32-gemm fp16x3
run_step 420 gpurun_out/r4a_prof.log bash tools/prof_run.sh r4a_f16 --fp32-gemm fp16x3
run_step 300 gpurun_out/r4a_bench.log python -u bench.py
run_step 300 gpurun_out/r4a_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
run_step 1000 gpurun_out/r4a_gputests.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
