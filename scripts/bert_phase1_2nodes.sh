#!/bin/bash
# Two nodes x 8 GPUs (reference STORE_RUN_FILE/Train_bert/node2gpu4/*): run this on node 0 with
# RANK_BASE=0 and on node 1 with RANK_BASE=8; both reach node 0 at MASTER:PORT (or a shared file:// path).
MASTER=${MASTER:-10.0.0.1}; PORT=${PORT:-12345}; RANK_BASE=${RANK_BASE:-0}
DATA=${DATA:-./data/phase1}; CFG=${CFG:-./configs/bert_base.json}; VOCAB=${VOCAB:-./configs/vocab.txt}
python -m hetseq_9cme_amd.train --task bert --data $DATA --dict $VOCAB --config_file $CFG \
  --max-sentences 128 --fast-stat-sync --max-update 450000 --disable-validation --num-workers 4 \
  --warmup-updates 10000 --lr 0.0001 --weight-decay 0.01 --save-dir bert_2nodes \
  --distributed-init-method tcp://$MASTER:$PORT --distributed-world-size 16 \
  --distributed-gpus 8 --distributed-rank $RANK_BASE
