# round 5 (bq): MLM decoder tiles at batch 32 / 128 masked-row counts
set -o pipefail
mkdir -p gpurun_out
M=640 timeout -k 10 200 python -u tools/probe/decoder_tiles.py > gpurun_out/r5bq_decoder_tiles.log 2>&1 &&
M=2560 timeout -k 10 200 python -u tools/probe/decoder_tiles.py >> gpurun_out/r5bq_decoder_tiles.log 2>&1
echo done
