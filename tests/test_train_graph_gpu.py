"""--graph-train-step: HIP-graph replayed updates == eager updates.

Two engines from the same seed train on the same batches, one eagerly and one with
captured-and-replayed updates (utils/train_graph.py).  Dropout is ON, so the replays must
read fresh per-update keys from the device seed tensor, the Adam kernels the current
bias-corrected step size / scheduled LR from the device hyper-parameter buffer, and the
grad scale / clip must stay live -- any of those baked into the graph shows up as a weight
mismatch after a few replays.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(argv):
    from hetseq_9cme_amd import options, tasks
    from hetseq_9cme_amd.controller import Controller
    args = options.parse_training_args(argv)
    args.device_id = 0
    args.distributed_rank = 0
    torch.manual_seed(args.seed)
    task = tasks.setup_task(args)
    model = task.build_model(args)
    ctrl = Controller(args, task, model)
    epoch_itr = ctrl.get_train_iterator(epoch=0, load_dataset=True)
    ctrl.lr_step(epoch_itr.epoch)
    return ctrl, epoch_itr


def _run(argv, n):
    from hetseq_9cme_amd.data import iterators
    ctrl, epoch_itr = _engine(argv)
    itr = iterators.GroupedIterator(epoch_itr.next_epoch_itr(shuffle=False), 1)
    losses = []
    for _ in range(n):
        out = ctrl.train_step(next(itr))
        losses.append(float(out['loss']))
    torch.cuda.synchronize()
    state = {k: v.detach().float().cpu().clone() for k, v in ctrl.get_model().state_dict().items()}
    return ctrl, losses, state


def _compare(eager, graph, tol):
    ce, le, se = eager
    cg, lg, sg = graph
    assert cg._graph_step.captures >= 1 and cg._graph_step.replays >= 1, \
        (cg._graph_step.captures, cg._graph_step.replays)
    for a, b in zip(le, lg):
        assert abs(a - b) <= tol * max(1.0, abs(a)), (le, lg)
    assert ce.get_num_updates() == cg.get_num_updates()
    assert ce.get_lr() == cg.get_lr()
    for k in se:
        d = (se[k] - sg[k]).abs().max().item()
        assert d <= tol * max(1.0, se[k].abs().max().item()), (k, d)
    assert ce.optimizer.steps == cg.optimizer.steps


@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
def test_graph_step_matches_eager_bert(dev, tmp_path, precision):
    from hetseq_9cme_amd.data.synthetic import BERT_TINY, write_bert_config, write_synthetic_bert_shards, write_vocab
    d = tmp_path / 'data'
    write_synthetic_bert_shards(str(d), n_files=1, samples_per_file=96, seq_len=128, max_pred=20, vocab_size=1024,
                                split='train')
    cfg = write_bert_config(str(tmp_path / 'c.json'), **BERT_TINY)    # dropout 0.1 on
    vocab = write_vocab(str(tmp_path / 'v.txt'), 1024)
    argv = ['--task', 'bert', '--data', str(d), '--dict', vocab, '--config_file', cfg, '--max-sentences', '8',
            '--fast-stat-sync', '--disable-validation', '--num-workers', '1', '--lr', '1e-3', '--weight-decay',
            '0.01', '--clip-norm', '0.5', '--distributed-world-size', '1', '--no-save', '--precision', precision,
            '--warmup-updates', '3', '--total-num-update', '20', '--lr-scheduler', 'PolynomialDecayScheduler']
    n = 8   # 2 eager warm-up, 1 capture, 5 replays
    eager = _run(argv, n)
    graph = _run(argv + ['--graph-train-step'], n)
    assert graph[0]._graph_step.captures == 1 and graph[0]._graph_step.replays == n - 3
    # identical kernels, keys and hyper-parameters: only the word-embedding scatter's float
    # atomics reorder (the eager engines differ from each other by as much)
    _compare(eager, graph, 1e-4 if precision == 'fp32' else 2e-3)


def test_graph_step_matches_eager_ner_shapes(dev, tmp_path):
    """Variable-length NER batches: padded to multiples of 4, several shapes, one graph
    each (sharing one memory pool), replays interleaved across shapes."""
    from hetseq_9cme_amd.data.synthetic import (BERT_TINY, WORDS, write_bert_config, write_synthetic_conll,
                                                write_vocab)
    vocab = write_vocab(str(tmp_path / 'vocab.txt'), 1024, extra_words=WORDS)
    cfg = write_bert_config(str(tmp_path / 'c.json'), **BERT_TINY)
    tr = write_synthetic_conll(str(tmp_path / 'train.txt'), 40 * 8, seed=0, min_len=4, max_len=40)
    argv = ['--task', 'BertForTokenClassification', '--optimizer', 'adam', '--fast-stat-sync', '--lr', '1e-4',
            '--dict', vocab, '--config_file', cfg, '--train_file', tr, '--extension_file', 'conll',
            '--max-sentences', '8', '--num-workers', '1', '--find-unused-parameters', '--disable-validation',
            '--no-save', '--pad-to-multiple-of', '4']
    n = 30
    eager = _run(argv + ['--no-graph-train-step'], n)
    assert eager[0]._graph_step is None
    graph = _run(argv, n)   # the default for token classification on a GPU: graph-captured updates
    gs = graph[0]._graph_step
    assert gs.captures >= 2, gs.captures
    _compare(eager, graph, 1e-4)


REDUCER_GRAPH_SCRIPT = r'''
import sys, torch, torch.distributed as dist
from hetseq_9cme_amd import options, tasks
from hetseq_9cme_amd.controller import Controller
from hetseq_9cme_amd.data import iterators
argv = sys.argv[2:]
torch.cuda.set_device(0)
dist.init_process_group('nccl', init_method=sys.argv[1], world_size=1, rank=0)
res = []
for extra in ([], ['--graph-train-step']):
    args = options.parse_training_args(argv + extra)
    args.device_id, args.distributed_rank = 0, 0
    torch.manual_seed(args.seed)
    task = tasks.setup_task(args)
    ctrl = Controller(args, task, task.build_model(args))
    assert ctrl.reducer.enabled
    ep = ctrl.get_train_iterator(epoch=0, load_dataset=True)
    ctrl.lr_step(ep.epoch)
    itr = iterators.GroupedIterator(ep.next_epoch_itr(shuffle=False), 1)
    losses = [float(ctrl.train_step(next(itr))['loss']) for _ in range(24)]
    torch.cuda.synchronize()
    st = {k: v.detach().float().cpu().clone() for k, v in ctrl.get_model().state_dict().items()}
    res.append((ctrl, losses, st))
gs = res[1][0]._graph_step
print('captures', gs.captures, 'replays', gs.replays)
assert gs.captures >= 1 and gs.replays >= 8, (gs.captures, gs.replays)
for a, b in zip(res[0][1], res[1][1]):
    assert abs(a - b) <= 1e-4 * max(1.0, abs(a)), (res[0][1], res[1][1])
for k, v in res[0][2].items():
    d = (v - res[1][2][k]).abs().max().item()
    assert d <= 1e-4 * max(1.0, v.abs().max().item()), (k, d)
dist.destroy_process_group()
print('GRAPH-REDUCER OK')
'''


def test_graph_step_with_rccl_reducer_ner(dev, tmp_path):
    """--graph-train-step with the gradient reducer on (a one-rank RCCL group, --force-reducer,
    --find-unused-parameters: the NER runs' DDP settings, run_bert_fine_tuning_ner.sh:36): the
    bucket collectives, the stats all-reduce and the used flags are captured into the update
    graph, and the replayed updates match eager reducer updates on the same batches (to the
    word-embedding scatter's atomics)."""
    import os
    import socket
    import subprocess
    import sys
    from hetseq_9cme_amd.data.synthetic import (BERT_TINY, WORDS, write_bert_config, write_synthetic_conll,
                                                write_vocab)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    vocab = write_vocab(str(tmp_path / 'vocab.txt'), 1024, extra_words=WORDS)
    cfg = write_bert_config(str(tmp_path / 'c.json'), **BERT_TINY)
    tr = write_synthetic_conll(str(tmp_path / 'train.txt'), 40 * 8, seed=0, min_len=4, max_len=40)
    argv = ['--task', 'BertForTokenClassification', '--optimizer', 'adam', '--fast-stat-sync', '--lr', '1e-4',
            '--dict', vocab, '--config_file', cfg, '--train_file', tr, '--extension_file', 'conll',
            '--max-sentences', '8', '--num-workers', '1', '--find-unused-parameters', '--disable-validation',
            '--no-save', '--pad-to-multiple-of', '16', '--force-reducer', '--distributed-world-size', '1',
            '--distributed-backend', 'nccl', '--bucket-cap-mb', '1']
    script = tmp_path / 'graph_reducer.py'
    script.write_text(REDUCER_GRAPH_SCRIPT)
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, str(script), 'tcp://127.0.0.1:{}'.format(port)] + argv,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       env=dict(os.environ, PYTHONPATH=root), timeout=300)
    assert r.returncode == 0 and 'GRAPH-REDUCER OK' in r.stdout, r.stdout[-4000:]
