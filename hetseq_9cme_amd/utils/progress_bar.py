"""Progress / log-line output.

Same line format as the reference's ``simple`` bar (hetseq/progress_bar.py:114-139):
``| epoch 001:      1 / 439 loss=0.044, ppl=1.03, ...``.  The reference names a
``json`` and ``tqdm`` bar but never defines them (progress_bar.py:20-27, SURVEY
App. A11); here ``json`` is implemented (one JSON object per log line, machine
readable) and ``tqdm`` maps to ``simple`` when no TTY is attached.
"""
from collections import OrderedDict
import json
from numbers import Number
import sys

import torch

from .meters import AverageMeter, StopwatchMeter, TimeMeter


def build_progress_bar(args, iterator, epoch=None, prefix=None, default='simple',
                       no_progress_bar='none'):
    if getattr(args, 'log_format', None) is None:
        args.log_format = no_progress_bar if args.no_progress_bar else default
    fmt = args.log_format
    if fmt == 'tqdm' and not sys.stderr.isatty():
        fmt = 'simple'
    if fmt == 'json':
        return json_progress_bar(iterator, epoch, prefix, args.log_interval)
    if fmt == 'none':
        return noop_progress_bar(iterator, epoch, prefix)
    if fmt in ('simple', 'tqdm'):
        return simple_progress_bar(iterator, epoch, prefix, args.log_interval)
    raise ValueError('Unknown log format: {}'.format(fmt))


def format_stat(stat):
    if torch.is_tensor(stat):
        stat = stat.item()
    if isinstance(stat, Number):
        return '{:g}'.format(stat)
    if isinstance(stat, AverageMeter):
        return '{:.3f}'.format(stat.avg)
    if isinstance(stat, TimeMeter):
        return '{:g}'.format(round(stat.avg))
    if isinstance(stat, StopwatchMeter):
        return '{:.4f}'.format(stat.sum)
    return stat


def _json_stat(stat):
    if torch.is_tensor(stat):
        return stat.item()
    if isinstance(stat, AverageMeter):
        return round(stat.avg, 6)
    if isinstance(stat, TimeMeter):
        return round(stat.avg, 3)
    if isinstance(stat, StopwatchMeter):
        return round(stat.sum, 4)
    if isinstance(stat, (int, float, str, type(None))):
        return stat
    return str(stat)


class progress_bar(object):
    """Abstract progress bar."""

    def __init__(self, iterable, epoch=None, prefix=None):
        self.iterable = iterable
        self.offset = getattr(iterable, 'offset', 0)
        self.epoch = epoch
        self.prefix = ''
        if epoch is not None:
            self.prefix += '| epoch {:03d}'.format(epoch)
        if prefix is not None:
            self.prefix += ' | {}'.format(prefix)

    def __len__(self):
        return len(self.iterable)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def __iter__(self):
        raise NotImplementedError

    def log(self, stats, tag='', step=None):
        raise NotImplementedError

    def print(self, stats, tag='', step=None):
        raise NotImplementedError

    def _str_commas(self, stats):
        return ', '.join(key + '=' + stats[key].strip() for key in stats.keys())

    def _str_pipes(self, stats):
        return ' | '.join(key + ' ' + stats[key].strip() for key in stats.keys())

    def _format_stats(self, stats):
        postfix = OrderedDict(stats)
        for key in postfix.keys():
            postfix[key] = str(format_stat(postfix[key]))
        return postfix


class noop_progress_bar(progress_bar):
    def __iter__(self):
        for obj in self.iterable:
            yield obj

    def log(self, stats, tag='', step=None):
        pass

    def print(self, stats, tag='', step=None):
        pass


class simple_progress_bar(progress_bar):
    """Minimal logger for non-TTY environments (stats formatted lazily, only
    on the iterations that actually print, so device meters are not synced
    every step)."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix)
        self.log_interval = log_interval
        self.stats = None

    def __iter__(self):
        size = len(self.iterable)
        for i, obj in enumerate(self.iterable, start=self.offset):
            yield obj
            if self.stats is not None and i > 0 and \
                    self.log_interval is not None and i % self.log_interval == 0:
                postfix = self._str_commas(self._format_stats(self.stats))
                print('{}:  {:5d} / {:d} {}'.format(self.prefix, i, size, postfix), flush=True)

    def log(self, stats, tag='', step=None):
        self.stats = stats

    def print(self, stats, tag='', step=None):
        postfix = self._str_pipes(self._format_stats(stats))
        print('{} | {}'.format(self.prefix, postfix), flush=True)


class json_progress_bar(progress_bar):
    """One JSON object per logged iteration (machine-readable log)."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix)
        self.log_interval = log_interval
        self.stats = None

    def __iter__(self):
        size = float(len(self.iterable))
        for i, obj in enumerate(self.iterable, start=self.offset):
            yield obj
            if self.stats is not None and i > 0 and \
                    self.log_interval is not None and i % self.log_interval == 0:
                update = self.epoch - 1 + float(i / size) if self.epoch is not None else None
                rec = OrderedDict([('epoch', self.epoch), ('update', update)])
                for k, v in self.stats.items():
                    rec[k] = _json_stat(v)
                print(json.dumps(rec), flush=True)

    def log(self, stats, tag='', step=None):
        self.stats = stats

    def print(self, stats, tag='', step=None):
        rec = OrderedDict([('epoch', self.epoch), ('tag', tag)])
        for k, v in stats.items():
            rec[k] = _json_stat(v)
        print(json.dumps(rec), flush=True)
