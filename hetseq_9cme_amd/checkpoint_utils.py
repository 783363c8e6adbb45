"""Checkpoint save / load / retention (reference hetseq/checkpoint_utils.py:14-222).

File format = the reference's ``torch.save`` dict so existing tools keep working:
  {'args', 'model', 'optimizer_history': [{optimizer_name, lr_scheduler_state,
   num_updates}], 'extra_state', 'last_optimizer_state'}
with ``last_optimizer_state`` in torch-optimizer layout (``state[i]['step' |
'exp_avg' | 'exp_avg_sq']``, ``param_groups``) and model keys per SURVEY App. C.
Names: checkpoint{E}.pt, checkpoint_{E}_{U}.pt, checkpoint_best.pt,
checkpoint_last.pt; only rank 0 writes; regex-based pruning.

Deliberate fixes: ``extra_state`` is persisted (reference writes ``{}`` --
App. A1 -- so resume was impossible); meters are stored as plain dicts; ``args``
is stored as a Namespace of plain values; loading uses ``weights_only=True``
(with argparse.Namespace allow-listed) so loading never executes code.
"""
import argparse
import collections
import logging
import os
import re
import shutil
import traceback
from collections import OrderedDict

import torch

from .parallel import distributed as dist_utils
from .utils import meters as meters_mod

_PRIMS = (int, float, str, bool, type(None))


def sanitize_args(args):
    """Namespace holding only plain values (tokenizers / datasets stashed on args
    by fine-tuning tasks are dropped)."""
    out = argparse.Namespace()
    for k, v in vars(args).items():
        if isinstance(v, _PRIMS):
            setattr(out, k, v)
        elif isinstance(v, (list, tuple)) and all(isinstance(x, _PRIMS) for x in v):
            setattr(out, k, list(v))
    return out


def meters_state(meters):
    out = OrderedDict()
    for k, m in meters.items():
        if isinstance(m, meters_mod.AverageMeter):
            out[k] = {'type': 'avg', 'val': m.val, 'sum': m.sum, 'count': m.count}
        elif isinstance(m, meters_mod.TimeMeter):
            out[k] = {'type': 'time', 'init': m.elapsed_time, 'n': m.n}
        elif isinstance(m, meters_mod.StopwatchMeter):
            out[k] = {'type': 'stopwatch', 'sum': m.sum, 'n': m.n}
    return out


def load_meters_state(meters, state):
    for k, s in state.items():
        if k not in meters:
            continue
        m = meters[k]
        if s.get('type') == 'avg':
            m._val, m._sum, m.count = s['val'], s['sum'], s['count']
        elif s.get('type') == 'time':
            m.reset(s['init'])
            m.n = s['n']
        elif s.get('type') == 'stopwatch':
            m.sum, m.n = s['sum'], s['n']


def save_checkpoint(args, controller, epoch_itr, val_loss):
    prev_best = getattr(save_checkpoint, 'best', val_loss)
    if val_loss is not None:
        best_function = max if args.maximize_best_checkpoint_metric else min
        save_checkpoint.best = best_function(val_loss, prev_best)
    if hasattr(controller, 'check_transport_all'):
        controller.check_transport_all()   # on EVERY rank: all raise together, before rank 0 writes
    if args.no_save or not dist_utils.is_master(args):
        return

    def is_better(a, b):
        return a >= b if args.maximize_best_checkpoint_metric else a <= b

    write_timer = meters_mod.StopwatchMeter()
    write_timer.start()
    epoch = epoch_itr.epoch
    end_of_epoch = epoch_itr.end_of_epoch()
    updates = controller.get_num_updates()

    conds = collections.OrderedDict()
    conds['checkpoint{}.pt'.format(epoch)] = (end_of_epoch and not args.no_epoch_checkpoints
                                              and epoch % args.save_interval == 0)
    conds['checkpoint_{}_{}.pt'.format(epoch, updates)] = (not end_of_epoch and args.save_interval_updates > 0
                                                           and updates % args.save_interval_updates == 0)
    conds['checkpoint_best.pt'] = (val_loss is not None and (not hasattr(save_checkpoint, 'best')
                                                             or is_better(val_loss, save_checkpoint.best)))
    conds['checkpoint_last.pt'] = not args.no_last_checkpoints

    extra_state = {'train_iterator': epoch_itr.state_dict(), 'val_loss': val_loss}
    if hasattr(save_checkpoint, 'best'):
        extra_state.update({'best': save_checkpoint.best})

    checkpoints = [os.path.join(args.save_dir, fn) for fn, cond in conds.items() if cond]
    if len(checkpoints) > 0:
        # with --async-save the write (and the copies) continue on a background thread
        controller.save_checkpoint(checkpoints[0], extra_state, copies=checkpoints[1:])
        write_timer.stop()
        print('| saved checkpoint {} (epoch {} @ {} updates) (writing took {} seconds)'.format(
            checkpoints[0], epoch, updates, write_timer.sum))

    if not end_of_epoch and args.keep_interval_updates > 0:
        for old in checkpoint_paths(args.save_dir, pattern=r'checkpoint_\d+_(\d+)\.pt')[args.keep_interval_updates:]:
            if os.path.lexists(old):
                os.remove(old)
    if args.keep_last_epochs > 0:
        for old in checkpoint_paths(args.save_dir, pattern=r'checkpoint(\d+)\.pt')[args.keep_last_epochs:]:
            if os.path.lexists(old):
                os.remove(old)


def load_checkpoint(args, controller):
    """Load a checkpoint (if present) and return (extra_state, epoch_itr)."""
    if args.distributed_rank == 0:
        os.makedirs(args.save_dir, exist_ok=True)
    if args.restore_file in ('checkpoint_last.pt', 'checkpoint_best.pt'):
        checkpoint_path = os.path.join(args.save_dir, args.restore_file)
    else:
        checkpoint_path = args.restore_file
    import ast
    overrides = ast.literal_eval(args.optimizer_overrides) if isinstance(args.optimizer_overrides, str) \
        else args.optimizer_overrides
    extra_state = controller.load_checkpoint(checkpoint_path, args.reset_optimizer, args.reset_lr_scheduler,
                                             overrides, reset_meters=args.reset_meters)
    if extra_state is not None and 'best' in extra_state and not args.reset_optimizer and not args.reset_meters:
        save_checkpoint.best = extra_state['best']
    if extra_state is not None and 'train_iterator' in extra_state and not args.reset_dataloader:
        itr_state = extra_state['train_iterator']
        epoch_itr = controller.get_train_iterator(epoch=itr_state['epoch'], load_dataset=True)
        epoch_itr.load_state_dict(itr_state)
    else:
        epoch_itr = controller.get_train_iterator(epoch=0, load_dataset=True)
    controller.lr_step(epoch_itr.epoch)
    return extra_state, epoch_itr


def load_checkpoint_to_cpu(path, arg_overrides=None):
    with torch.serialization.safe_globals([argparse.Namespace]):
        state = torch.load(path, map_location='cpu', weights_only=True)
    args = state.get('args')
    if arg_overrides is not None and args is not None:
        for k, v in arg_overrides.items():
            setattr(args, k, v)
    if state.get('extra_state') is None:
        state['extra_state'] = {}
    return state


def checkpoint_paths(path, pattern=r'checkpoint(\d+)\.pt'):
    pt_regexp = re.compile(pattern)
    entries = []
    for i, f in enumerate(os.listdir(path)):
        m = pt_regexp.fullmatch(f)
        if m is not None:
            idx = int(m.group(1)) if len(m.groups()) > 0 else i
            entries.append((idx, m.group(0)))
    return [os.path.join(path, x[1]) for x in sorted(entries, reverse=True)]


def torch_persistent_save(obj, filename, copies=()):
    """Atomic save: write ``filename.tmp`` then ``os.replace`` it, so a crash or
    preemption mid-write never leaves a truncated ``checkpoint_last.pt``
    (reference: plain ``torch.save`` with 3 retries, checkpoint_utils.py).
    ``copies`` (other checkpoint names for the same state) are produced the
    same way from the finished file."""
    tmp = filename + '.tmp'
    for i in range(3):
        try:
            torch.save(obj, tmp)
            os.replace(tmp, filename)
            break
        except Exception:
            if i == 2:
                logging.error(traceback.format_exc())
                return
    for cp in copies:
        ctmp = cp + '.tmp'
        shutil.copyfile(filename, ctmp)
        os.replace(ctmp, cp)


def convert_state_dict_type(state_dict, ttype=torch.float32):
    """Recursively copy tensors to CPU fp32 (de-duplicating shared storage views)."""
    memo = {}

    def conv(x):
        if isinstance(x, dict):
            return OrderedDict((k, conv(v)) for k, v in x.items())
        if isinstance(x, list):
            return [conv(v) for v in x]
        if torch.is_tensor(x):
            key = (x.data_ptr(), tuple(x.shape), x.dtype)
            if key not in memo:
                y = x.detach().to('cpu', dtype=ttype if x.is_floating_point() else x.dtype, copy=True)
                memo[key] = y.contiguous()
            return memo[key]
        return x
    return conv(state_dict)


def build_state(args, model_state_dict, optimizer, lr_scheduler, num_updates, optim_history=None,
                extra_state=None):
    optim_history = optim_history or []
    state = {
        'args': sanitize_args(args),
        'model': convert_state_dict_type(model_state_dict) if model_state_dict else {},
        'optimizer_history': optim_history + [{
            'optimizer_name': optimizer.__class__.__name__,
            'lr_scheduler_state': lr_scheduler.state_dict(),
            'num_updates': num_updates,
        }],
        'extra_state': extra_state if extra_state is not None else {},
    }
    if not getattr(args, 'no_save_optimizer_state', False):
        state['last_optimizer_state'] = convert_state_dict_type(optimizer.state_dict())
    return state


def save_state(filename, args, model_state_dict, criterion, optimizer, lr_scheduler, num_updates,
               optim_history=None, extra_state=None):
    torch_persistent_save(build_state(args, model_state_dict, optimizer, lr_scheduler, num_updates,
                                      optim_history, extra_state), filename)


def verify_checkpoint_directory(save_dir):
    os.makedirs(save_dir, exist_ok=True)
    temp_file_path = os.path.join(save_dir, 'dummy')
    try:
        with open(temp_file_path, 'w'):
            pass
    except OSError as e:
        print('| Unable to access checkpoint save directory: {}'.format(save_dir))
        raise e
    else:
        os.remove(temp_file_path)
