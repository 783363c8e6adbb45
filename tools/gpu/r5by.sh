# round 5 (by): token-type gradient kernel vs the one-hot GEMM (standalone)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/probe/type_grad_probe.py > gpurun_out/r5by_type_grad.log 2>&1
echo done
