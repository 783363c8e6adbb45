"""bench.py launch contract on the CPU (no GPU needed): a plain ``bench.py --gpus N`` spawns N
rank processes itself (RANK / WORLD_SIZE / MASTER_* like torch.distributed.run), a launch whose
world is not --gpus exits non-zero, and a failing rank makes the whole job fail."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, 'bench.py')


def _env(**kw):
    env = dict(os.environ, PYTHONPATH=ROOT, HIP_VISIBLE_DEVICES='', CUDA_VISIBLE_DEVICES='')
    for k in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env.update(kw)
    return env


@pytest.mark.skipif(__import__('torch').cuda.is_available(), reason='CPU-only launch check')
def test_plain_launch_spawns_n_ranks():
    r = subprocess.run([sys.executable, BENCH, '--gpus', '3', '--steps', '1', '--warmup', '0'], env=_env(),
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, cwd=ROOT)
    # each child reached run() with its own rank of a 3-rank env:// world, then stopped: no GPU here
    for rk in range(3):
        assert 'bench: rank {}/3 on device {} (env://)'.format(rk, rk) in r.stdout, r.stdout[-2000:]
    assert r.returncode == 4, r.stdout[-2000:]
    assert '{"metric"' not in r.stdout


def test_world_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, BENCH, '--gpus', '3', '--steps', '1', '--warmup', '0'],
                       env=_env(RANK='0', LOCAL_RANK='0', WORLD_SIZE='2', MASTER_ADDR='127.0.0.1',
                                MASTER_PORT='29999'),
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 2, r.stdout[-2000:]
    assert '--gpus 3 but the launch gives WORLD_SIZE 2' in r.stdout
    assert '{"metric"' not in r.stdout


def test_single_gpu_default_world_is_one():
    # no flags -> N = 1, no spawn; on a GPU-less host the rank stops before the GPU
    if __import__('torch').cuda.is_available():
        pytest.skip('CPU-only launch check')
    r = subprocess.run([sys.executable, BENCH, '--steps', '1', '--warmup', '0'], env=_env(),
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, cwd=ROOT)
    assert 'bench: rank 0/1 on device 0' in r.stdout and r.returncode == 4, r.stdout[-2000:]
