# usage: bash tools/prof_run.sh NAME [bench.py args...]
# rocprofv3 kernel trace of a short bench run -> gpurun_out/prof_NAME/ (+ markdown summary)
set -o pipefail
name=$1; shift
out=gpurun_out/prof_$name
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $out -o run -- python3 bench.py --steps 7 --warmup 3 "$@" > $out/bench.log 2>&1 &&
db=$(find $out -name '*results.db' | head -n 1) &&
python3 tools/prof_summary.py "$db" --steps 6 --gaps 25 --seq 10 > $out/summary.md &&
rm -f "$db"
