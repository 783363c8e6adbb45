"""Flag parity with the reference and the poly-decay LR schedule."""
import argparse
import math

import pytest

from hetseq_9cme_amd import options
from hetseq_9cme_amd.optim.lr_scheduler import PolynomialDecayScheduler


def parse(extra):
    return options.parse_training_args(['--task', 'bert', '--config_file', 'x.json'] + extra)


def test_reference_defaults():
    a = parse([])
    assert a.seed == 19940802
    assert a.log_interval == 1 and a.log_format == 'simple'
    assert a.num_workers == -1 and a.required_batch_size_multiple == 1
    assert a.train_subset == 'train' and a.valid_subset == 'valid'
    assert a.max_pred_length == 512 and a.num_file == 0
    assert a.distributed_rank == 0 and a.distributed_gpus == 4 and a.distributed_backend == 'nccl'
    assert a.bucket_cap_mb == 25 and a.ddp_backend == 'c10d'
    assert a.max_epoch == 0 and a.max_update == 0 and a.clip_norm == 25
    assert a.update_freq == [1] and a.lr == [0.25] and a.min_lr == -1
    assert a.adam_betas == '(0.9, 0.999)' and a.adam_eps == 1e-8 and a.weight_decay == 0.0
    assert a.warmup_updates == 0 and a.end_learning_rate == 0.0 and a.power == 1.0
    assert a.total_num_update == 1000000
    assert a.save_dir == 'checkpoints' and a.restore_file == 'checkpoint_last.pt'
    assert a.save_interval == 1 and a.keep_interval_updates == -1 and a.keep_last_epochs == -1
    assert a.optimizer_overrides == '{}' and a.best_checkpoint_metric == 'loss'
    assert a.precision == 'fp32'


def test_aliases_and_lists():
    a = parse(['--batch-size', '32', '--mu', '7', '--me', '2', '--wd', '0.01', '--update-freq', '4,2',
               '--learning-rate', '0.1,0.05', '--local_rank', '3', '--fa', '5'])
    assert a.max_sentences == 32 and a.max_update == 7 and a.max_epoch == 2 and a.weight_decay == 0.01
    assert a.update_freq == [4, 2] and a.lr == [0.1, 0.05] and a.device_id == 3 and a.force_anneal == 5
    assert a.max_sentences_valid == 32


def test_task_specific_groups():
    a = options.parse_training_args(['--task', 'mnist', '--optimizer', 'adadelta', '--data', '/x'])
    assert a.task == 'mnist' and a.optimizer == 'adadelta' and a.adadelta_rho == 0.9 and a.adadelta_eps == 1e-6
    a = options.parse_training_args(['--task', 'BertForTokenClassification', '--config_file', 'c',
                                     '--load_state_dict_strict', 'True'])
    assert a.load_state_dict_strict is True and a.hetseq_state_dict is None
    with pytest.raises(SystemExit):
        options.parse_training_args(['--task', 'bert'])   # --config_file is required


class _Opt(object):
    def __init__(self):
        self.lr = None

    def set_lr(self, lr):
        self.lr = lr

    def get_lr(self):
        return self.lr


def _sched(**kw):
    args = argparse.Namespace(lr=[1e-4], warmup_updates=0, end_learning_rate=0.0, total_num_update=1000000,
                              power=1.0, force_anneal=None)
    for k, v in kw.items():
        setattr(args, k, v)
    return PolynomialDecayScheduler(args, _Opt())


def test_poly_decay_matches_reference_log():
    # shipped NER log: lr=0.0001, warmup 0, total 50000 -> lr at update 439 printed as 9.9122e-05
    s = _sched(total_num_update=50000)
    assert abs(s.step_update(439) - 9.9122e-05) < 5e-10
    assert abs(s.step_update(2) - 9.9996e-05) < 5e-10


def test_poly_decay_warmup_and_end():
    s = _sched(warmup_updates=100, total_num_update=1000, power=2.0, end_learning_rate=1e-6)
    assert s.step_update(0) == 0.0
    assert abs(s.step_update(50) - 0.5e-4) < 1e-12
    assert abs(s.step_update(100) - 1e-4) < 1e-12
    n = 550
    expect = (1e-4 - 1e-6) * (1 - (n - 100) / 900) ** 2 + 1e-6
    assert abs(s.step_update(n) - expect) < 1e-12
    assert s.step_update(1000) == 1e-6 and s.step_update(5000) == 1e-6


def test_epoch_step_lr_list():
    s = _sched(lr=[0.1, 0.05])
    assert s.step(0) == 0.1
    assert s.step(1) == 0.05 and s.step(7) == 0.05


def test_comm_cus_auto_plan():
    """--comm-cus defaults to 0 (no CU reservation, no RCCL channel cap) until a multi-GPU run
    measures the trade-off; 'auto' is opt-in: the channel cap + plan reservation (16 CUs) on GPU
    runs with world > 1 (profiles/r3_comm_contention.md: a one-GPU 16-CU comm load costs +15 %
    unplanned, +6 % planned), off for one rank, CPU / gloo rehearsals."""
    from hetseq_9cme_amd import options
    base = ['--task', 'mnist', '--data', '/tmp/x']
    a = options.parse_training_args(base)
    assert a.comm_cus == 0
    a.distributed_world_size = 8
    assert options.comm_cus(a) == 0
    a = options.parse_training_args(base + ['--comm-cus', 'auto'])
    a.distributed_world_size = 8
    assert options.comm_cus(a) == options.AUTO_COMM_CUS == 16
    a.distributed_world_size = 1
    assert options.comm_cus(a) == 0
    a.distributed_world_size = 8
    a.distributed_backend = 'gloo'
    assert options.comm_cus(a) == 0
    a = options.parse_training_args(base + ['--comm-cus', '8', '--cpu'])
    a.distributed_world_size = 8
    assert options.comm_cus(a) == 8
    a = options.parse_training_args(base + ['--comm-cus', '0'])
    a.distributed_world_size = 8
    assert options.comm_cus(a) == 0
    a = options.parse_training_args(base + ['--cpu'])
    a.distributed_world_size = 4
    assert options.comm_cus(a) == 0
