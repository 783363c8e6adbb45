set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -m gpu -x -v --timeout 60 --timeout-method thread -k "pingpong" > gpurun_out/pp_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_split_gemm_gpu.py -m gpu -x -q --timeout 60 --timeout-method thread -k "every_cfg or gelu_epilogues" > gpurun_out/pp_tests2.log 2>&1 &&
timeout -k 10 200 python -u tools/probe/gemm_pingpong_probe.py > gpurun_out/pp_probe.log 2>&1
