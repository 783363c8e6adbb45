#!/bin/bash
# CoNLL-2003 NER fine-tuning from a pre-training checkpoint (BASELINE config 5: 4 GPUs).
CK=${CK:-bert_phase1_node8/checkpoint_last.pt}; DIR=${DIR:-./data/conll2003}
python -m hetseq_9cme_amd.train --task BertForTokenClassification --optimizer adam \
  --lr-scheduler PolynomialDecayScheduler --fast-stat-sync --max-update 5000 --update-freq 1 \
  --valid-subset test --num-workers 4 --warmup-updates 0 --total-num-update 50000 --lr 0.0001 \
  --dict ${VOCAB:-./configs/vocab.txt} --config_file ${CFG:-./configs/bert_base.json} \
  --hetseq_state_dict $CK --train_file $DIR/train.txt --validation_file $DIR/valid.txt \
  --test_file $DIR/test.txt --extension_file conll --max-sentences 32 --load_state_dict_strict False \
  --find-unused-parameters --distributed-world-size 4 --save-dir bert_ner
python -m hetseq_9cme_amd.eval_ner --model_ckpt bert_ner/checkpoint_last.pt --config_file ${CFG:-./configs/bert_base.json} \
  --dict ${VOCAB:-./configs/vocab.txt} --test_file $DIR/test.txt --train_file $DIR/train.txt
