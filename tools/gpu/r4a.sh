# round 4, first call: state of the tree on a fresh box (smoke, headline bench, GPU suite)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r4a_bench.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a_gputests.log 2>&1
