#!/bin/bash
# Phase 2 (seq 512, 80 masked positions): global batch 256 on 8 GPUs (BASELINE config 4).
DATA=${DATA:-./data/phase2}; CFG=${CFG:-./configs/bert_base.json}; VOCAB=${VOCAB:-./configs/vocab.txt}
python -m hetseq_9cme_amd.train --task bert --data $DATA --dict $VOCAB --config_file $CFG \
  --max-sentences 32 --fast-stat-sync --max-update 10000 --disable-validation --num-workers 4 \
  --lr 0.00005 --weight-decay 0.01 --distributed-world-size 8 --save-dir bert_phase2_node8 \
  --restore-file bert_phase1_node8/checkpoint_last.pt --reset-optimizer --reset-lr-scheduler --reset-dataloader
