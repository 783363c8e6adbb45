#!/bin/bash
# Heterogeneous launch (BASELINE config 3): a 5-GPU "node" (ranks 0-4) + a 3-GPU "node"
# (ranks 5-7) on one 8-GPU box, each launcher seeing only its own GPUs.
DATA=${DATA:-./data/phase1}; CFG=${CFG:-./configs/bert_base.json}; VOCAB=${VOCAB:-./configs/vocab.txt}
python tools/launch_hetero.py --nodes 5,3 -- --task bert --data $DATA --dict $VOCAB --config_file $CFG \
  --max-sentences 128 --fast-stat-sync --max-update 1000 --disable-validation --num-workers 4 \
  --warmup-updates 10000 --lr 0.0001 --weight-decay 0.01 --save-dir bert_hetero_5p3
