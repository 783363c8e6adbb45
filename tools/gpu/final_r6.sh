# Round-6 final validation on one MI355X: full GPU test suite, smoke, headline bench (x2), batch 32,
# phase 2, BERT-large (seq 128 b32 / seq 512 b8), NER (default path), and a rocprofv3 kernel trace
# of the headline step.  Outputs gpurun_out/${P}_* (P, default r6v).
set -o pipefail
mkdir -p gpurun_out
P=${P:-r6v}
export TMPDIR=/tmp
. tools/gpu/run_step.sh
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${P}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${P}_tests.log; exit 1; }
tail -1 gpurun_out/${P}_tests.log
run_step 300 gpurun_out/${P}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
for i in 1 2; do run_step 400 gpurun_out/${P}_bench$i.log python -u bench.py --steps 20 --warmup 5 || exit 1; done
run_step 400 gpurun_out/${P}_bench_b32.log python -u bench.py --steps 20 --warmup 5 --batch 32 || exit 1
run_step 400 gpurun_out/${P}_bench_p2.log python -u bench.py --steps 10 --warmup 3 --seq 512 --batch 32 --max-pred 80 || exit 1
run_step 400 gpurun_out/${P}_bench_large128.log python -u bench.py --steps 10 --warmup 3 --model large --batch 32 || exit 1
run_step 400 gpurun_out/${P}_bench_large512.log python -u bench.py --steps 10 --warmup 3 --model large --seq 512 --batch 8 --max-pred 80 || exit 1
run_step 400 gpurun_out/${P}_ner.log python -u tools/bench_ner.py --steps 40 --repeats 5 || exit 1
run_step 400 gpurun_out/${P}_prof.log rocprofv3 --kernel-trace --stats -d /tmp/${P}prof -o run -- python3 bench.py --steps 5 --warmup 3 || exit 1
python tools/prof_summary.py /tmp/${P}prof/run_results.db --steps 6 --marker adam_k --top 45 > gpurun_out/${P}_step_profile.md
python tools/step_sequence.py /tmp/${P}prof/run_results.db > gpurun_out/${P}_step_sequence.md || true
for f in gpurun_out/${P}_bench*.log gpurun_out/${P}_ner.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*\|"s_per_update_min_median_max": \[[0-9., ]*\]' $f | head -2 | tr '\n' ' ')"; done
echo all done
