"""User-extension path: --user-module registering a task / optimizer / LR
scheduler (examples/toy_extension.py), trained through the real CLI."""
import os

import torch

from test_engine_cpu import ROOT, load, run_cli


def test_user_module_task_optimizer_scheduler(tmp_path):
    save = str(tmp_path / 'ck')
    run_cli(['--user-module', os.path.join(ROOT, 'examples', 'toy_extension.py'), '--task', 'toy_regression',
             '--optimizer', 'sgd', '--momentum', '0.9', '--lr-scheduler', 'constant', '--lr', '0.02',
             '--toy-dim', '6', '--max-sentences', '32', '--max-epoch', '15', '--data', 'unused',
             '--valid-subset', 'valid', '--num-workers', '1', '--clip-norm', '0', '--save-dir', save,
             '--cpu', '--log-format', 'json', '--log-interval', '1000', '--no-epoch-checkpoints'])
    ck = load(os.path.join(save, 'checkpoint_last.pt'))
    # the linear model recovered y = x . [1..6]
    assert torch.allclose(ck['model']['lin.weight'].flatten(), torch.arange(1., 7.), atol=1e-2)
    assert ck['last_optimizer_state']['param_groups'][0]['momentum'] == 0.9
    assert ck['optimizer_history'][-1]['optimizer_name'] == 'SGDMomentum'
    assert ck['args'].lr_scheduler == 'constant' and ck['args'].toy_dim == 6


def test_profile_phases_log(tmp_path):
    """--profile-phases adds per-phase host times (t_*) to the log line."""
    r = run_cli(['--user-module', os.path.join(ROOT, 'examples', 'toy_extension.py'), '--task', 'toy_regression',
                 '--optimizer', 'sgd', '--lr-scheduler', 'constant', '--lr', '0.01', '--max-sentences', '32',
                 '--max-update', '4', '--data', 'unused', '--num-workers', '1', '--save-dir', str(tmp_path / 'ck'),
                 '--no-save', '--cpu', '--log-format', 'json', '--log-interval', '2', '--profile-phases'])
    import json
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{')]
    assert lines, r.stdout[-2000:]
    for k in ('t_prep', 't_sample', 't_forward', 't_backward', 't_optimizer'):
        assert k in lines[-1], (k, lines[-1])
