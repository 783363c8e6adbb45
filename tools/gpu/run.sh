#!/bin/bash
# One parametrised GPU runner (replaces the per-round r4*/r5* one-off scripts, which remain in
# git history).  Usage on the GPU box, e.g.
#   gpurun -- 'bash tools/gpu/run.sh TAG tests bench "--batch 32" profile "" pmc "SQ_WAVES GRBM_GUI_ACTIVE"'
# RECIPE ARGS pairs, run in order; every GPU step is time-bounded and a fault / timeout / crash
# stops the call (run_step.sh).  Outputs: gpurun_out/TAG_<recipe><n>.{log,md}.
#   tests   ARGS  pytest -m gpu ARGS (e.g. "-k attention")
#   smoke   -     __graft_entry__.smoke()
#   bench   ARGS  python bench.py ARGS
#   ner     ARGS  python tools/bench_ner.py ARGS
#   profile ARGS  rocprofv3 --kernel-trace --stats of bench.py --steps 5 --warmup 3 ARGS + the
#                 per-step kernel table (tools/prof_summary.py)
#   pmc     CTRS  rocprofv3 --pmc CTRS of tools/probe/gemm_f16_bench.py (ONLY=$ONLY) + pmc_summary
#   parity  ARGS  python tools/parity_run.py ARGS
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
. tools/gpu/run_step.sh
TAG=$1; shift
n=0
while [ $# -gt 0 ]; do
  r=$1; a=$2; shift 2; n=$((n + 1)); out=gpurun_out/${TAG}_${r}${n}
  case $r in
    tests)   timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread $a \
               > $out.log 2>&1 || { echo "tests failed: $out.log"; tail -30 $out.log; exit 1; } ;;
    smoke)   run_step 300 $out.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench)   run_step 400 $out.log python -u bench.py $a || exit 1 ;;
    ner)     run_step 400 $out.log python -u tools/bench_ner.py $a || exit 1 ;;
    profile) run_step 400 $out.log rocprofv3 --kernel-trace --stats -d /tmp/prof$n -o run -- \
               python3 bench.py --steps 5 --warmup 3 $a || exit 1
             python tools/prof_summary.py /tmp/prof$n/run_results.db --steps 6 --marker adam_k --top 45 > $out.md
             python tools/step_sequence.py /tmp/prof$n/run_results.db > ${out}_sequence.md || true ;;
    pmc)     run_step 120 $out.log timeout -s KILL 100 rocprofv3 --pmc $a --output-format csv -d /tmp/pmc$n -o run -- \
               python3 tools/probe/gemm_f16_bench.py || exit 1
             python tools/pmc_summary.py /tmp/pmc$n/run_counter_collection.csv > $out.md 2>&1 || true ;;
    parity)  run_step 1000 $out.log python -u tools/parity_run.py $a || exit 1 ;;
    *) echo "unknown recipe $r"; exit 2 ;;
  esac
  echo "$r done: $out"
done
echo all done
