"""Distributed engine with the GPU kernels: 2 ranks share the box's GPU over gloo
(a rehearsal of the RCCL path -- same reducer, buckets, hooks, stats sync) and must
match 1 rank with --update-freq 2 on the same batches."""
import argparse
import os
import subprocess
import sys

import pytest
import torch

from hetseq_9cme_amd.data.synthetic import BERT_TINY, write_bert_config, write_synthetic_bert_shards, write_vocab

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_gpu_equivalence(dev, tmp_path):
    d = tmp_path / 'data'
    write_synthetic_bert_shards(str(d), n_files=1, samples_per_file=64, seq_len=128, max_pred=20, vocab_size=1024,
                                split='train')
    cfg = write_bert_config(str(tmp_path / 'c.json'), **dict(BERT_TINY, hidden_dropout_prob=0.0,
                                                               attention_probs_dropout_prob=0.0))
    vocab = write_vocab(str(tmp_path / 'v.txt'), 1024)
    common = ['--task', 'bert', '--data', str(d), '--dict', vocab, '--config_file', cfg, '--max-sentences', '8',
              '--fast-stat-sync', '--max-update', '2', '--disable-validation', '--num-workers', '1', '--lr', '1e-3',
              '--bucket-cap-mb', '1']
    # 'one'/'two': 2 micro-batches per update either way; 'one4'/'two2': the same with
    # local accumulation under no_sync on top (first micro-batch claims the flat
    # slots, later ones accumulate through autograd)
    runs = {'one': ['--update-freq', '2', '--distributed-world-size', '1'],
            'two': ['--distributed-world-size', '2', '--distributed-backend', 'gloo'],
            'one4': ['--update-freq', '4', '--distributed-world-size', '1'],
            'two2': ['--update-freq', '2', '--distributed-world-size', '2', '--distributed-backend', 'gloo'],
            # gradient buckets through the hand-written two-shot kernel over IPC-mapped buffers
            # (both ranks on this box's one GPU; kernel waits bounded by the 60 s timeout)
            'twox': ['--distributed-world-size', '2', '--distributed-backend', 'gloo', '--allreduce-impl', 'xgmi',
                     '--distributed-timeout', '60'],
            # the default fp32 path (bf16x6 split GEMMs) forced onto these small GEMMs
            'one6': ['--update-freq', '2', '--distributed-world-size', '1', '--fp32-gemm', 'bf16x6'],
            'two6': ['--distributed-world-size', '2', '--distributed-backend', 'gloo', '--fp32-gemm', 'bf16x6']}
    ck = {}
    for name, extra in runs.items():
        save = str(tmp_path / name)
        env = dict(os.environ, PYTHONPATH=ROOT)
        if name.endswith('6'):
            env['HETSEQ_SPLIT_MIN_ROWS_X6'] = '0'
        r = subprocess.run([sys.executable, '-m', 'hetseq_9cme_amd.train'] + common + extra + ['--save-dir', save],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, timeout=400)
        assert r.returncode == 0, r.stdout[-3000:]
        with torch.serialization.safe_globals([argparse.Namespace]):
            ck[name] = torch.load(os.path.join(save, 'checkpoint_last.pt'), map_location='cpu', weights_only=True)
    for k, v in ck['one']['model'].items():
        torch.testing.assert_close(ck['two']['model'][k], v, rtol=1e-4, atol=1e-6, msg=k)
    for k, v in ck['one']['model'].items():
        torch.testing.assert_close(ck['twox']['model'][k], v, rtol=1e-4, atol=1e-6, msg=k)
    for k, v in ck['one4']['model'].items():
        torch.testing.assert_close(ck['two2']['model'][k], v, rtol=1e-4, atol=1e-6, msg=k)
    for k, v in ck['one6']['model'].items():
        torch.testing.assert_close(ck['two6']['model'][k], v, rtol=1e-4, atol=1e-6, msg=k)
    assert ck['two2']['optimizer_history'][-1]['num_updates'] == 2


def test_bench_two_ranks_contract(tmp_path):
    """bench.py under torch.distributed.run with 2 ranks (the driver's N > 1 launch; here both
    ranks share the box's GPU over gloo): one JSON line from rank 0 with the whole-job value,
    n_gpus = 2 and the global batch of both ranks."""
    import json
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=ROOT, TMPDIR=str(tmp_path))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(port), os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', '3',
           '--warmup', '1', '--model', 'tiny', '--batch', '8', '--backend', 'gloo', '--same-device',
           '--num-workers', '1']
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 2 and rec['steps'] == 3 and rec['warmup'] == 1
    assert rec['config']['global_batch'] == 16 and rec['config']['parallelism'] == 'dp2'
    assert rec['value'] > 0 and rec['ms_per_step'] > 0
    assert abs(rec['value'] - 16 * 1000.0 / rec['ms_per_step']) / rec['value'] < 1e-3


def test_bench_heterogeneous_nodes_contract(tmp_path):
    """bench.py --nodes 2,1 (the BASELINE config-3 5+3 launch in miniature): one launcher per
    "node" spawns its ranks like train.py mode (a), all meet over one tcp:// rendezvous; rank 0
    prints ONE JSON line for the whole 3-rank job with the per-node split (rehearsal: every
    rank on this box's GPU over gloo)."""
    import json
    env = dict(os.environ, PYTHONPATH=ROOT, TMPDIR=str(tmp_path))
    env.pop('RANK', None)
    env.pop('WORLD_SIZE', None)
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--nodes', '2,1', '--steps', '3', '--warmup', '1',
           '--model', 'tiny', '--batch', '8', '--backend', 'gloo', '--same-device', '--num-workers', '1']
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 3 and rec['config']['global_batch'] == 24
    assert rec['config']['nodes'] == [2, 1] and rec['config']['parallelism'] == 'dp3 (nodes 2+1)'
    assert abs(rec['value'] - 24 * 1000.0 / rec['ms_per_step']) / rec['value'] < 1e-3


def test_bench_ner_torchrun_contract(tmp_path):
    """tools/bench_ner.py under torch.distributed.run (BASELINE config 5, 4-GPU NER, here 2 ranks
    on the box's GPU over gloo, BERT-tiny): env:// rendezvous, LOCAL_RANK device, one JSON line
    from rank 0 with the max-over-ranks seconds per update."""
    import json
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=ROOT, TMPDIR=str(tmp_path))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2', '--master-addr',
           '127.0.0.1', '--master-port', str(port), os.path.join(ROOT, 'tools', 'bench_ner.py'), '--gpus', '2',
           '--steps', '3', '--warmup', '1', '--batch', '8', '--backend', 'gloo', '--same-device', '--model', 'tiny']
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == 2 and rec['global_batch'] == 16 and rec['value'] > 0
