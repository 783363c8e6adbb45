set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_f.log 2>&1 &&
timeout -k 10 300 python -u bench.py --seq 512 --max-pred 80 --batch 32 --steps 10 --warmup 3 > gpurun_out/bench_p2.log 2>&1 &&
timeout -k 10 200 python -u tools/probe/ffn_epilogue_probe.py > gpurun_out/ffn_epi2.log 2>&1 &&
bash tools/pmc_run.sh gemm "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_LDS_BANK_CONFLICT,SQ_INSTS_VALU_MFMA_MOPS_BF16,GRBM_GUI_ACTIVE,GRBM_COUNT" python3 tools/probe/gemm_pmc_probe.py
find gpurun_out/pmc_gemm -name '*.csv' > gpurun_out/pmc_gemm/files.txt
python3 tools/pmc_summary.py $(grep counter_collection gpurun_out/pmc_gemm/files.txt) --match gemm_piece > gpurun_out/pmc_gemm/summary.md
