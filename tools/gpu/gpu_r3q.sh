set -o pipefail
mkdir -p gpurun_out
A="--seq 512 --max-pred 80 --batch 32 --steps 12 --warmup 3"
timeout -k 10 300 python -u bench.py $A > gpurun_out/q_side0.log 2>&1 &&
timeout -k 10 300 python -u bench.py $A --no-overlap-wgrad > gpurun_out/q_main0.log 2>&1 &&
timeout -k 10 300 python -u bench.py $A > gpurun_out/q_side1.log 2>&1 &&
timeout -k 10 300 python -u bench.py $A --no-overlap-wgrad > gpurun_out/q_main1.log 2>&1
