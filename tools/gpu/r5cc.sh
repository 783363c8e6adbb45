# round 5 (cc): HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory) on the host-bound
# configurations: batch 32 and the eager NER update (alternated twice)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5cc_warm.log python -u tools/bench_ner.py --steps 10 &&
for i in 1 2; do
run_step 300 gpurun_out/r5cc_b32_def_$i.log python -u bench.py --batch 32 &&
HIP_FORCE_DEV_KERNARG=1 run_step 300 gpurun_out/r5cc_b32_dka_$i.log python -u bench.py --batch 32 &&
run_step 300 gpurun_out/r5cc_ner_def_$i.log python -u tools/bench_ner.py &&
HIP_FORCE_DEV_KERNARG=1 run_step 300 gpurun_out/r5cc_ner_dka_$i.log python -u tools/bench_ner.py || exit 1
done
echo done
