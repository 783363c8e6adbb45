"""Small helpers shared across the engine (reference: hetseq/utils.py:12-37,
86-91, 167-171).  Only the helpers the training path actually uses are kept;
the reference's unused fairseq leftovers (``resolve_max_positions`` etc.,
SURVEY P25) are not carried over."""
import math

import torch


def apply_to_sample(f, sample):
    """Apply ``f`` to every tensor in a (possibly nested) sample."""
    if sample is None or (hasattr(sample, '__len__') and len(sample) == 0):
        return {}

    def _apply(x):
        if torch.is_tensor(x):
            return f(x)
        if isinstance(x, dict):
            return {k: _apply(v) for k, v in x.items()}
        if isinstance(x, list):
            return [_apply(v) for v in x]
        if isinstance(x, tuple):
            return tuple(_apply(v) for v in x)
        return x

    return _apply(sample)


def move_to_device(sample, device, non_blocking=True):
    """Move every tensor of a sample to ``device``.  Host tensors are copied
    asynchronously: pageable ones are first staged through the (cached) pinned
    host allocator, because a pageable ``.to(device)`` blocks the host until the
    GPU has drained its queue -- once per batch tensor, which made small-batch
    fine-tuning host-bound (the reference's ``.cuda()`` is synchronous and
    pageable, utils.py:32-37)."""
    def _move(t):
        if t.device == device:
            return t
        if non_blocking and device.type == 'cuda' and t.device.type == 'cpu':
            if not t.is_pinned():
                t = t.pin_memory()
            return t.to(device, non_blocking=True)
        return t.to(device, non_blocking=non_blocking and t.is_pinned())
    return apply_to_sample(_move, sample)


def move_to_cuda(sample):
    return move_to_device(sample, torch.device('cuda', torch.cuda.current_device()))


def item(tensor):
    if hasattr(tensor, 'item'):
        return tensor.item()
    if hasattr(tensor, '__getitem__'):
        return tensor[0]
    return tensor


def get_perplexity(loss):
    try:
        return float('{:.2f}'.format(math.pow(2, loss)))
    except OverflowError:
        return float('inf')


def count_parameters(model):
    return sum(p.numel() for p in model.parameters())


def ensure_train(model):
    """``model.train()`` only when the model is not already in training mode.

    The reference calls ``model.train()`` in both the controller and the task on every
    update (hetseq/controller.py:228, tasks/tasks.py:163); for BERT-base that walks ~220
    modules and performs ~440 ``__setattr__`` calls per step -- 1.6 ms of host time per
    update, which matters once the step is host-bound (fine-tuning at batch 32).  The root
    flag is kept in sync by ``train()`` / ``eval()``, so checking it is enough."""
    if not model.training:
        model.train()
    return model
