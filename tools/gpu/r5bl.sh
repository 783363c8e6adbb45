# round 5 (bl): eager NER update after the host-side caches (adjacent views, encoder weight list)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5bl_warm.log python -u tools/bench_ner.py --steps 10 &&
for i in 1 2 3; do run_step 300 gpurun_out/r5bl_eager_$i.log python -u tools/bench_ner.py || exit 1; done
run_step 300 gpurun_out/r5bl_ner_cprof.log python -u tools/bench_ner.py --steps 20 --cprofile gpurun_out/r5bl_ner_cprofile.txt
echo done
