# round 5 (bw): bf16 bench with the shipped GEMM table vs the table + TunableOp-tuned bf16 keys
# (alternated twice; the box's tree is scratch, the table is swapped in place)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
cp hetseq_9cme_amd/tuning/gemm_gfx950.csv /tmp/shipped.csv
for i in 1 2; do
cp /tmp/shipped.csv hetseq_9cme_amd/tuning/gemm_gfx950.csv &&
run_step 300 gpurun_out/r5bw_shipped_$i.log python -u bench.py --precision bf16 &&
cp tools/gpu/data/r5bv_merged_table.csv hetseq_9cme_amd/tuning/gemm_gfx950.csv &&
run_step 300 gpurun_out/r5bw_merged_$i.log python -u bench.py --precision bf16 || exit 1
done
run_step 300 gpurun_out/r5bw_fp32_merged.log python -u bench.py
echo done
