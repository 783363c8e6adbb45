set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe/gemm_stagger_probe.py > gpurun_out/mf16_probe.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -k "every_cfg or gelu_epilogues or b16_layouts" -x -v --timeout 120 --timeout-method thread > gpurun_out/mf16_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -k rccl -x -v --timeout 300 --timeout-method thread > gpurun_out/rccl_tests.log 2>&1 &&
bash tools/probe/comm_contention_probe.sh 16 > gpurun_out/comm_contention.log 2>&1
