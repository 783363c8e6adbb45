#!/bin/bash
# MNIST (reference STORE_RUN_FILE/Train_mnist/*): CPU / gloo world 1 plumbing run (BASELINE config 1).
python -m hetseq_9cme_amd.train --task mnist --optimizer adadelta --lr-scheduler PolynomialDecayScheduler \
  --data ${DATA:-./data/mnist} --clip-norm 100 --max-sentences 64 --fast-stat-sync --max-epoch 20 \
  --update-freq 1 --valid-subset test --num-workers 4 --warmup-updates 0 --total-num-update 50000 \
  --lr 1.01 --save-dir mnist_cpu --cpu
python -m hetseq_9cme_amd.eval_mnist --mnist_dir ${DATA:-./data/mnist} --model_ckpt mnist_cpu/checkpoint_last.pt --cpu
