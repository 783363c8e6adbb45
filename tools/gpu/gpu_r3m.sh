set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --seq 512 --max-pred 80 --batch 32 --steps 10 --warmup 3 > gpurun_out/m_p2_side.log 2>&1 &&
timeout -k 10 300 python -u bench.py --seq 512 --max-pred 80 --batch 32 --steps 10 --warmup 3 --no-overlap-wgrad > gpurun_out/m_p2_main.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch 32 > gpurun_out/m_b32_side.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch 32 --no-overlap-wgrad > gpurun_out/m_b32_main.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_ner.py > gpurun_out/m_ner_side.log 2>&1 &&
timeout -k 10 300 python -u tools/bench_ner.py --no-overlap-wgrad > gpurun_out/m_ner_main.log 2>&1
