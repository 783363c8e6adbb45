# usage: bash tools/api_run.sh NAME [bench.py args...] -- HIP API + kernel trace, long host calls
set -o pipefail
name=$1; shift
out=gpurun_out/api_$name
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace -d $out -o run -- python3 bench.py --steps 7 --warmup 3 "$@" > $out/bench.log 2>&1 &&
db=$(find $out -name '*results.db' | head -n 1) &&
python3 tools/api_trace.py "$db" --steps 4 --min-us 150 > $out/api.txt &&
python3 tools/prof_summary.py "$db" --steps 4 --gaps 12 > $out/summary.md &&
rm -f "$db"
