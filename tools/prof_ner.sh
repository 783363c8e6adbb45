# usage: bash tools/prof_ner.sh NAME [bench_ner.py args...]
# rocprofv3 kernel trace of a short NER fine-tuning run -> gpurun_out/prof_NAME/summary.md
set -o pipefail
name=$1; shift
out=gpurun_out/prof_$name
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $out -o run -- python3 tools/bench_ner.py --steps 12 --warmup 4 "$@" > $out/bench.log 2>&1 &&
db=$(find $out -name '*results.db' | head -n 1) &&
python3 tools/prof_summary.py "$db" --steps 10 --top 25 > $out/summary.md &&
rm -f "$db"
