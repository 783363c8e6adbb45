# round 5 (bj): NER eager update host cost of the pre-split / bias-epilogue paths (alternated)
set -o pipefail
mkdir -p gpurun_out
. tools/gpu/run_step.sh
run_step 300 gpurun_out/r5bj_warm.log python -u tools/bench_ner.py --steps 10 &&
for i in 1 2; do
HX_PRESPLIT=0 HX_QKV_BIAS_EPILOGUE=0 run_step 300 gpurun_out/r5bj_p0b0_$i.log python -u tools/bench_ner.py &&
HX_PRESPLIT=1 HX_QKV_BIAS_EPILOGUE=0 run_step 300 gpurun_out/r5bj_p1b0_$i.log python -u tools/bench_ner.py &&
HX_PRESPLIT=0 HX_QKV_BIAS_EPILOGUE=1 run_step 300 gpurun_out/r5bj_p0b1_$i.log python -u tools/bench_ner.py &&
HX_PRESPLIT=1 HX_QKV_BIAS_EPILOGUE=1 run_step 300 gpurun_out/r5bj_p1b1_$i.log python -u tools/bench_ner.py || exit 1
done
echo done
