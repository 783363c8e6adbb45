# q-kernel (cfg 7) check: its GEMM tests, then the probe switches ($QPROBE) and the cfg sweep
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_f16_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "every_tile or gelu_epilogues or row_ramp or presplit_a_bitwise" > gpurun_out/q1_tests.log 2>&1 || { tail -30 gpurun_out/q1_tests.log; exit 1; }
tail -2 gpurun_out/q1_tests.log
timeout -k 10 300 python -u tools/probe/gemm_q_probe.py > gpurun_out/q1_probe.log 2>&1 || { tail -30 gpurun_out/q1_probe.log; exit 1; }
cat gpurun_out/q1_probe.log
if [ -n "$CFGS" ]; then
  timeout -k 10 300 python -u tools/probe/gemm_f16_bench.py > gpurun_out/q1_sweep.log 2>&1 || { tail -30 gpurun_out/q1_sweep.log; exit 1; }
  cat gpurun_out/q1_sweep.log
fi
