# round 5 (v): 300-update BERT-base parity of fp16x3 (per-row / per-column scales) vs native fp32
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 1100 gpurun_out/r5v_parity.log python -u tools/parity_run.py --updates 300 --out gpurun_out/r5v_parity
echo done
