set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/n_b128.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch 32 > gpurun_out/n_b32.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch 64 > gpurun_out/n_b64_planes.log 2>&1 &&
HX_PIECE_MIN_ROWS=0 timeout -k 10 300 python -u bench.py --batch 64 > gpurun_out/n_b64_pieces.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_ner.py > gpurun_out/n_ner.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_n.log 2>&1
