#!/bin/bash
# One node, all 8 GPUs, one process per GPU over RCCL/xGMI (reference mode (c)).
DATA=${DATA:-./data/phase1}; CFG=${CFG:-./configs/bert_base.json}; VOCAB=${VOCAB:-./configs/vocab.txt}
python -m hetseq_9cme_amd.train --task bert --data $DATA --dict $VOCAB --config_file $CFG \
  --max-sentences 128 --fast-stat-sync --max-update 450000 --disable-validation --num-workers 4 \
  --warmup-updates 10000 --total-num-update 1000000 --lr 0.0001 --weight-decay 0.01 \
  --distributed-world-size 8 --save-dir bert_phase1_node8
