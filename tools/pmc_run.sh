# usage: bash tools/pmc_run.sh NAME "COUNTERS" python3 script.py args...
# one rocprofv3 counter pass (<= 8 SQ counters) -> gpurun_out/pmc_NAME/ (csv)
set -o pipefail
name=$1; shift
ctr=$1; shift
out=gpurun_out/pmc_$name
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $out -o run -- "$@" > $out/log.txt 2>&1
