"""End-to-end engine tests on CPU: CLI training, checkpoint format, exact resume,
multi-process (gloo) heterogeneous launch, DP gradient equivalence."""
import argparse
import os
import subprocess
import sys

import pytest
import torch

from hetseq_9cme_amd.data.synthetic import (BERT_TINY, write_bert_config, write_synthetic_bert_shards,
                                            write_synthetic_mnist, write_vocab)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_cli(argv, env=None, check=True):
    e = dict(os.environ)
    e['PYTHONPATH'] = ROOT + os.pathsep + e.get('PYTHONPATH', '')
    e.setdefault('OMP_NUM_THREADS', '2')
    if env:
        e.update(env)
    r = subprocess.run([sys.executable, '-m', 'hetseq_9cme_amd.train'] + argv, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, env=e, timeout=600)
    if check and r.returncode != 0:
        raise AssertionError(r.stdout[-4000:])
    return r


def load(path):
    with torch.serialization.safe_globals([argparse.Namespace]):
        return torch.load(path, map_location='cpu', weights_only=True)


@pytest.fixture(scope='module')
def bert_data(tmp_path_factory):
    d = tmp_path_factory.mktemp('bert')
    write_synthetic_bert_shards(str(d), n_files=2, samples_per_file=48, seq_len=32, max_pred=5, vocab_size=1024,
                                split='train', seed=1)
    write_synthetic_bert_shards(str(d), n_files=1, samples_per_file=16, seq_len=32, max_pred=5, vocab_size=1024,
                                split='test', seed=2)
    cfg = write_bert_config(str(d / 'tiny.json'), **BERT_TINY)
    vocab = write_vocab(str(d / 'vocab.txt'), 1024)
    return str(d), cfg, vocab


def bert_argv(data, cfg, vocab, save, extra=()):
    return ['--task', 'bert', '--data', data, '--dict', vocab, '--config_file', cfg, '--max-sentences', '4',
            '--fast-stat-sync', '--valid-subset', 'test', '--num-workers', '1', '--lr', '1e-3',
            '--warmup-updates', '2', '--weight-decay', '0.01', '--save-dir', save, '--cpu',
            '--log-interval', '1'] + list(extra)


def test_mnist_cli_learns_and_checkpoints(tmp_path):
    write_synthetic_mnist(str(tmp_path / 'mnist'), n_train=640, n_test=64)
    save = str(tmp_path / 'ck')
    r = run_cli(['--task', 'mnist', '--optimizer', 'adadelta', '--data', str(tmp_path / 'mnist'), '--max-sentences',
                 '64', '--fast-stat-sync', '--max-epoch', '3', '--valid-subset', 'test', '--num-workers', '1',
                 '--lr', '1.01', '--clip-norm', '100', '--save-dir', save, '--cpu', '--log-format', 'json',
                 '--log-interval', '9'])
    assert 'done training' in r.stdout
    ck = load(os.path.join(save, 'checkpoint_last.pt'))
    assert set(ck.keys()) >= {'args', 'model', 'optimizer_history', 'extra_state', 'last_optimizer_state'}
    assert ck['optimizer_history'][-1]['optimizer_name'] == '_Adadelta'
    assert ck['optimizer_history'][-1]['num_updates'] == 30
    assert ck['extra_state']['train_iterator']['epoch'] == 3
    st = ck['last_optimizer_state']['state'][0]
    assert set(st.keys()) == {'step', 'square_avg', 'acc_delta'}
    assert os.path.exists(os.path.join(save, 'checkpoint3.pt'))
    # MNIST evaluator on the checkpoint
    from hetseq_9cme_amd.eval_mnist import evaluate
    acc = evaluate(os.path.join(save, 'checkpoint_last.pt'), str(tmp_path / 'mnist'), device='cpu')
    assert acc > 0.5


def test_bert_exact_resume(tmp_path, bert_data):
    data, cfg, vocab = bert_data
    a = str(tmp_path / 'a')
    b = str(tmp_path / 'b')
    run_cli(bert_argv(data, cfg, vocab, a, ['--max-update', '8']))
    # first half with background (async) checkpoint writes: same bits on disk, no temp files left
    run_cli(bert_argv(data, cfg, vocab, b, ['--max-update', '4', '--async-save']))
    assert not [f for f in os.listdir(b) if f.endswith('.tmp')]
    ckb = load(os.path.join(b, 'checkpoint_last.pt'))
    assert ckb['extra_state']['train_iterator'] == {'epoch': 1, 'iterations_in_epoch': 4}
    run_cli(bert_argv(data, cfg, vocab, b, ['--max-update', '8']))
    ca = load(os.path.join(a, 'checkpoint_last.pt'))
    cb = load(os.path.join(b, 'checkpoint_last.pt'))
    assert ca['optimizer_history'][-1]['num_updates'] == cb['optimizer_history'][-1]['num_updates'] == 8
    for k in ca['model']:
        torch.testing.assert_close(ca['model'][k], cb['model'][k], rtol=0, atol=0, msg=k)
    sa = ca['last_optimizer_state']['state']
    sb = cb['last_optimizer_state']['state']
    for i in sa:
        assert sa[i]['step'] == sb[i]['step'] == 8
        torch.testing.assert_close(sa[i]['exp_avg'], sb[i]['exp_avg'], rtol=0, atol=0)


def test_fault_injection_then_resume(tmp_path, bert_data):
    data, cfg, vocab = bert_data
    save = str(tmp_path / 'f')
    r = run_cli(bert_argv(data, cfg, vocab, save, ['--max-update', '10', '--save-interval-updates', '3']),
                env={'HETSEQ_FAIL_AT_UPDATE': '7'}, check=False)
    assert r.returncode != 0 and 'fault injection' in r.stdout
    ck = load(os.path.join(save, 'checkpoint_last.pt'))
    assert ck['optimizer_history'][-1]['num_updates'] == 6
    r = run_cli(bert_argv(data, cfg, vocab, save, ['--max-update', '10', '--save-interval-updates', '3']))
    assert '@ 6 updates' in r.stdout
    ck = load(os.path.join(save, 'checkpoint_last.pt'))
    assert ck['optimizer_history'][-1]['num_updates'] == 10


@pytest.mark.slow
def test_heterogeneous_two_node_gloo(tmp_path, bert_data):
    """Two 'nodes' launched separately (node A: 1 proc, base rank 0; node B: spawns 2
    procs, base rank 1) meeting through a shared-file rendezvous; world = 3."""
    data, cfg, vocab = bert_data
    init = 'file://' + str(tmp_path / 'rdzv')
    save = str(tmp_path / 'ck')
    common = bert_argv(data, cfg, vocab, save, ['--max-update', '4', '--distributed-init-method', init,
                                                '--distributed-world-size', '3', '--check-params-every', '1'])
    e = dict(os.environ)
    e['PYTHONPATH'] = ROOT + os.pathsep + e.get('PYTHONPATH', '')
    e['OMP_NUM_THREADS'] = '1'
    procs = [subprocess.Popen([sys.executable, '-m', 'hetseq_9cme_amd.train'] + common +
                              ['--distributed-gpus', '1', '--distributed-rank', '0', '--distributed-no-spawn'],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e),
             subprocess.Popen([sys.executable, '-m', 'hetseq_9cme_amd.train'] + common +
                              ['--distributed-gpus', '2', '--distributed-rank', '1'],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e)]
    outs = [p.communicate(timeout=600)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs[0][-3000:] + outs[1][-3000:]
    assert 'done training' in outs[0]
    ck = load(os.path.join(save, 'checkpoint_last.pt'))
    assert ck['optimizer_history'][-1]['num_updates'] == 4


def test_data_parallel_gradient_equivalence(tmp_path, bert_data):
    """2 ranks x 1 micro-batch == 1 rank x 2 micro-batches (--update-freq 2): same update."""
    data, cfg, vocab = bert_data
    cfg0 = str(tmp_path / 'nodrop.json')
    write_bert_config(cfg0, **dict(BERT_TINY, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0))
    one = str(tmp_path / 'one')
    two = str(tmp_path / 'two')
    run_cli(bert_argv(data, cfg0, vocab, one, ['--max-update', '1', '--update-freq', '2']))
    # --allreduce-impl xgmi on CPU/gloo: not eligible -> warns and keeps the c10d transport
    run_cli(bert_argv(data, cfg0, vocab, two, ['--max-update', '1', '--distributed-world-size', '2',
                                               '--distributed-backend', 'gloo', '--allreduce-impl', 'xgmi']))
    c1 = load(os.path.join(one, 'checkpoint_last.pt'))
    c2 = load(os.path.join(two, 'checkpoint_last.pt'))
    for k in c1['model']:
        torch.testing.assert_close(c1['model'][k], c2['model'][k], rtol=1e-5, atol=1e-6, msg=k)
    s1 = c1['last_optimizer_state']['state']
    s2 = c2['last_optimizer_state']['state']
    for i in s1:
        torch.testing.assert_close(s1[i]['exp_avg'], s2[i]['exp_avg'], rtol=1e-4, atol=1e-9)


@pytest.mark.slow
def test_launch_hetero_tool_tcp(tmp_path):
    """tools/launch_hetero.py: two 'nodes' (2 + 1 ranks) meeting over a tcp://
    rendezvous, gloo on CPU; every rank ends with identical parameters."""
    write_synthetic_mnist(str(tmp_path / 'mnist'), n_train=384, n_test=64)
    save = str(tmp_path / 'ck')
    e = dict(os.environ)
    e['PYTHONPATH'] = ROOT + os.pathsep + e.get('PYTHONPATH', '')
    e['OMP_NUM_THREADS'] = '1'
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'launch_hetero.py'), '--cpu', '--nodes', '2,1',
                        '--', '--task', 'mnist', '--optimizer', 'adadelta', '--data', str(tmp_path / 'mnist'),
                        '--max-sentences', '32', '--max-update', '4', '--num-workers', '1', '--lr', '1.0',
                        '--save-dir', save, '--check-params-every', '1', '--fast-stat-sync'],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    ck = load(os.path.join(save, 'checkpoint_last.pt'))
    assert ck['optimizer_history'][-1]['num_updates'] == 4
    assert ck['args'].distributed_world_size == 3


def test_four_rank_gradient_equivalence_small_buckets(tmp_path, bert_data):
    """4 ranks (gloo) x 1 micro-batch with 1 MB gradient buckets == 1 rank x --update-freq 4:
    a rehearsal of the N > 2 reducer path (many buckets launched in order from the backward
    hooks, the last one after backward) on the CPU."""
    data, cfg, vocab = bert_data
    cfg0 = str(tmp_path / 'nodrop.json')
    write_bert_config(cfg0, **dict(BERT_TINY, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0))
    one = str(tmp_path / 'one')
    four = str(tmp_path / 'four')
    run_cli(bert_argv(data, cfg0, vocab, one, ['--max-update', '1', '--update-freq', '4']))
    run_cli(bert_argv(data, cfg0, vocab, four, ['--max-update', '1', '--distributed-world-size', '4',
                                                '--distributed-backend', 'gloo', '--bucket-cap-mb', '1']))
    c1 = load(os.path.join(one, 'checkpoint_last.pt'))
    c4 = load(os.path.join(four, 'checkpoint_last.pt'))
    for k in c1['model']:
        torch.testing.assert_close(c1['model'][k], c4['model'][k], rtol=1e-5, atol=1e-6, msg=k)


@pytest.mark.slow
def test_heterogeneous_5p3_replicas_match_update_freq(tmp_path):
    """The BASELINE 5+3 heterogeneous launch in miniature on the CPU: tools/launch_hetero.py
    starts two "nodes" (5 and 3 ranks, one tcp:// rendezvous, gloo), BERT-tiny, 3 updates.
    --check-params-every 1 asserts bit-identical replicas after every update on every rank, and
    the result equals ONE rank with --update-freq 8 (the 8 micro-batches of an update, summed
    locally instead of all-reduced: same math, different summation order)."""
    d = tmp_path / 'data'
    d.mkdir()
    write_synthetic_bert_shards(str(d), n_files=2, samples_per_file=64, seq_len=32, max_pred=5, vocab_size=1024,
                                split='train', seed=3)
    write_synthetic_bert_shards(str(d), n_files=1, samples_per_file=16, seq_len=32, max_pred=5, vocab_size=1024,
                                split='test', seed=4)
    cfg0 = write_bert_config(str(tmp_path / 'nodrop.json'),
                             **dict(BERT_TINY, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0))
    vocab = write_vocab(str(tmp_path / 'vocab.txt'), 1024)
    het, one = str(tmp_path / 'het'), str(tmp_path / 'one')
    common = ['--task', 'bert', '--data', str(d), '--dict', vocab, '--config_file', cfg0, '--max-sentences', '4',
              '--fast-stat-sync', '--valid-subset', 'test', '--num-workers', '0', '--lr', '1e-3',
              '--warmup-updates', '2', '--weight-decay', '0.01', '--log-interval', '1', '--max-update', '3',
              '--disable-validation']
    e = dict(os.environ)
    e['PYTHONPATH'] = ROOT + os.pathsep + e.get('PYTHONPATH', '')
    e['OMP_NUM_THREADS'] = '1'
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'launch_hetero.py'), '--cpu', '--nodes', '5,3',
                        '--'] + common + ['--save-dir', het, '--check-params-every', '1',
                                          '--distributed-backend', 'gloo'],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=e, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:]
    run_cli(common + ['--save-dir', one, '--cpu', '--update-freq', '8'])
    ch = load(os.path.join(het, 'checkpoint_last.pt'))
    c1 = load(os.path.join(one, 'checkpoint_last.pt'))
    assert ch['args'].distributed_world_size == 8
    assert ch['optimizer_history'][-1]['num_updates'] == c1['optimizer_history'][-1]['num_updates'] == 3
    for k in c1['model']:
        torch.testing.assert_close(ch['model'][k], c1['model'][k], rtol=1e-5, atol=1e-6, msg=k)
