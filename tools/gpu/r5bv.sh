# round 5 (bv): TunableOp tuning of the --precision bf16 library products (online), then a
# table A/B: bf16 bench with the tuned table vs library defaults
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 600 gpurun_out/r5bv_tune.log python -u bench.py --precision bf16 --gemm-tuning online --gemm-tuning-file $GRAFT_REPO_ROOT/gpurun_out/r5bv_bf16_tuned.csv --steps 5 --warmup 3 &&
ls gpurun_out/ > gpurun_out/r5bv_ls.txt &&
python -c "
import glob
from hetseq_9cme_amd.ops.gemm_tuning import merge_tables
fs = sorted(glob.glob('gpurun_out/r5bv_bf16_tuned*.csv'))
print(fs)
print(merge_tables(['hetseq_9cme_amd/tuning/gemm_gfx950.csv'] + fs, 'gpurun_out/r5bv_merged.csv'))
" > gpurun_out/r5bv_merge.log 2>&1 &&
cp gpurun_out/r5bv_merged.csv hetseq_9cme_amd/tuning/gemm_gfx950.csv &&
for i in 1 2; do
run_step 300 gpurun_out/r5bv_off_$i.log python -u bench.py --precision bf16 --gemm-tuning off &&
run_step 300 gpurun_out/r5bv_tab_$i.log python -u bench.py --precision bf16 --gemm-tuning table || exit 1
done
echo done
