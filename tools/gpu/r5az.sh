# round 5 (az): LayerNorm backward grid cap sweep (fp32 / bf16), alternated twice
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for c in 512 1024 2048; do
    HX_LN_BWD_CAP=$c timeout -k 10 120 python -u tools/probe/ln_probe.py >> gpurun_out/r5az_ln_cap.log 2>&1 || exit 1
  done
done
echo done
