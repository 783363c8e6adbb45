# quick GPU round: smoke, 1-GPU bench, GEMM layout / MFMA-shape probes -> gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench1.log 2>&1 &&
CFGS=0,1,7 timeout -k 10 300 python -u tools/probe/gemm_layout_probe.py > gpurun_out/layout_probe.log 2>&1
