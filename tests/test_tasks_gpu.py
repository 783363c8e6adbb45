"""Non-pretraining tasks end-to-end on the GPU through the real CLI: MNIST
(Adadelta, fused optimizer kernel) and NER fine-tuning (variable sequence
lengths -> the any-length fused attention, token-classification head), each
followed by its evaluator on the GPU."""
import os

import pytest

from hetseq_9cme_amd.data.synthetic import (BERT_TINY, WORDS, write_bert_config, write_synthetic_conll,
                                            write_synthetic_mnist, write_vocab)
from test_engine_cpu import load, run_cli

pytestmark = pytest.mark.gpu


def test_mnist_gpu_cli_and_eval(tmp_path):
    write_synthetic_mnist(str(tmp_path / 'mnist'), n_train=640, n_test=64)
    save = str(tmp_path / 'ck')
    run_cli(['--task', 'mnist', '--optimizer', 'adadelta', '--data', str(tmp_path / 'mnist'), '--max-sentences',
             '64', '--fast-stat-sync', '--max-epoch', '3', '--valid-subset', 'test', '--num-workers', '1',
             '--lr', '1.01', '--clip-norm', '100', '--save-dir', save, '--log-format', 'json', '--log-interval', '9',
             '--distributed-world-size', '1'])
    ck = load(os.path.join(save, 'checkpoint_last.pt'))
    assert ck['optimizer_history'][-1]['num_updates'] == 30
    from hetseq_9cme_amd.eval_mnist import evaluate
    assert evaluate(os.path.join(save, 'checkpoint_last.pt'), str(tmp_path / 'mnist'), device='cuda') > 0.5


def test_ner_gpu_cli_and_eval(tmp_path):
    vocab = write_vocab(str(tmp_path / 'vocab.txt'), 1024, extra_words=WORDS)
    cfg = write_bert_config(str(tmp_path / 'tiny.json'), **BERT_TINY)
    tr = write_synthetic_conll(str(tmp_path / 'train.txt'), 96, seed=0, min_len=5, max_len=30)
    te = write_synthetic_conll(str(tmp_path / 'test.txt'), 32, seed=1, min_len=5, max_len=30)
    save = str(tmp_path / 'ner')
    r = run_cli(['--task', 'BertForTokenClassification', '--fast-stat-sync', '--max-update', '24',
                 '--valid-subset', 'test', '--num-workers', '1', '--lr', '2e-3', '--dict', vocab,
                 '--config_file', cfg, '--train_file', tr, '--test_file', te, '--extension_file', 'conll',
                 '--max-sentences', '8', '--save-dir', save, '--distributed-world-size', '1'])
    assert 'done training' in r.stdout
    from hetseq_9cme_amd.eval_ner import evaluate
    res = evaluate(os.path.join(save, 'checkpoint_last.pt'), cfg, vocab, te, train_file=tr, device='cuda')
    # the synthetic tags are a deterministic function of the word: learnable in a few updates
    assert res['f1'] > 0.9 and res['accuracy'] > 0.9, res
