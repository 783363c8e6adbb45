# round 5 (bk): host profile of the eager NER update (cProfile, 20 updates)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5bk_ner_cprof.log python -u tools/bench_ner.py --steps 20 --cprofile gpurun_out/r5bk_ner_cprofile.txt
echo done
