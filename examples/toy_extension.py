"""Extending the framework without editing it: a custom task, optimizer and LR
scheduler registered from a user module (reference docs/source/extending.rst
describes subclassing ``Task`` / ``_Optimizer`` / ``_LRScheduler``; here they
are also registered so the CLI accepts them).

    python -m hetseq_9cme_amd.train --user-module examples/toy_extension.py \
        --task toy_regression --optimizer sgd --momentum 0.9 --lr-scheduler constant \
        --lr 0.05 --max-sentences 32 --max-epoch 5 --data unused --cpu
"""
import numpy as np
import torch

from hetseq_9cme_amd.optim import _LRScheduler, _Optimizer, register_lr_scheduler, register_optimizer
from hetseq_9cme_amd.tasks import Task, register_task


class RegressionData(torch.utils.data.Dataset):
    """y = x . [1..d]  (+ nothing): a linear model can fit it exactly."""

    def __init__(self, n=512, d=8, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.x = torch.randn(n, d, generator=g)
        self.y = self.x @ torch.arange(1., d + 1)

    def __len__(self):
        return len(self.x)

    def __getitem__(self, i):
        return self.x[i], self.y[i]

    # protocol used by Task.get_batch_iterator / EpochBatchIterator
    def ordered_indices(self):
        return np.arange(len(self))

    def num_tokens(self, index):
        return 1

    def collater(self, samples):
        return torch.utils.data.default_collate(samples)

    def set_epoch(self, epoch):
        pass


class LinearRegressor(torch.nn.Module):
    def __init__(self, d):
        super().__init__()
        self.lin = torch.nn.Linear(d, 1)

    def forward(self, x, y):          # models return the loss (Task.train_step contract)
        return ((self.lin(x).squeeze(-1) - y) ** 2).mean()


@register_task('toy_regression')
class ToyRegressionTask(Task):
    @staticmethod
    def add_args(group):
        group.add_argument('--toy-dim', type=int, default=8)

    @classmethod
    def setup_task(cls, args, **kwargs):
        return cls(args)

    def build_model(self, args):
        return LinearRegressor(args.toy_dim)

    def load_dataset(self, split, **kwargs):
        self.datasets[split] = RegressionData(d=self.args.toy_dim, seed=0 if split == 'train' else 1)


@register_optimizer('sgd')
class SGDMomentum(_Optimizer):
    """Plain torch-op update over the flat buffers (no custom kernel needed)."""

    @staticmethod
    def add_args(group):
        group.add_argument('--momentum', type=float, default=0.0)

    def __init__(self, args, flat):
        self.args = args
        super().__init__(args, flat)
        self.buf = torch.zeros_like(flat.param_flat)

    @property
    def optimizer_config(self):
        return {'lr': float(self.args.lr[0]), 'momentum': float(self.args.momentum)}

    def step(self, closure=None):
        g = self.scaled_grad_flat()
        self.buf.mul_(self.param_groups[0]['momentum']).add_(g)
        self.flat.param_flat.add_(self.buf, alpha=-self._lr)

    def _param_state(self, i):
        s, e = self.flat.param_range(i)
        return {'momentum_buffer': self.buf[s:e].view(self.flat.params[i].shape)}

    def _load_param_state(self, i, st):
        s, e = self.flat.param_range(i)
        self.buf[s:e].copy_(st['momentum_buffer'].reshape(-1))


@register_lr_scheduler('constant')
class ConstantLR(_LRScheduler):
    def __init__(self, args, optimizer):
        super().__init__(args, optimizer)
        optimizer.set_lr(args.lr[0])
