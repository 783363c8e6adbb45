#!/bin/bash
# BERT-base phase 1 (seq 128) on one MI355X; DATA holds *train*.hdf5 shards (NVIDIA schema).
# Synthetic shards: python -c "from hetseq_9cme_amd.data.synthetic import *; write_synthetic_bert_shards('DATA', 8, 8192)"
DATA=${DATA:-./data/phase1}; CFG=${CFG:-./configs/bert_base.json}; VOCAB=${VOCAB:-./configs/vocab.txt}
python -m hetseq_9cme_amd.train --task bert --data $DATA --dict $VOCAB --config_file $CFG \
  --max-sentences 128 --fast-stat-sync --max-update 450000 --update-freq 1 \
  --disable-validation --num-workers 4 --warmup-updates 10000 --total-num-update 1000000 \
  --lr 0.0001 --weight-decay 0.01 --save-dir bert_phase1_1gpu --distributed-world-size 1
