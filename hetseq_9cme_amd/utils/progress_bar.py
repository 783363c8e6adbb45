"""Progress / log-line output.

Line formats are the reference's, because scripts parse them
(hetseq/progress_bar.py:114-139): every ``log_interval`` iterations the ``simple``
bar prints ``| epoch 001:      1 / 439 loss=0.044, ppl=1.03, ...`` and ``print``
writes ``| epoch 001 | loss 0.044 | ...``.  The reference names a ``json`` and a
``tqdm`` bar but never defines them (progress_bar.py:20-27); here
``json`` is implemented (one JSON object per log line) and ``tqdm`` maps to
``simple`` when no TTY is attached.

Design: one base class owns the iteration and the "is this a logging iteration"
decision; a bar only supplies how a stats mapping is rendered (``_render_interval``
/ ``_render_summary``).  Stats are rendered lazily -- only on iterations that print --
so lazily-read device meters are not synchronised every step.
"""
from collections import OrderedDict
import json
from numbers import Number
import sys

import torch

from .meters import AverageMeter, StopwatchMeter, TimeMeter


def build_progress_bar(args, iterator, epoch=None, prefix=None, default='simple', no_progress_bar='none'):
    """Bar for ``args.log_format`` (defaulting it from ``--no-progress-bar``)."""
    if getattr(args, 'log_format', None) is None:
        args.log_format = no_progress_bar if args.no_progress_bar else default
    fmt = args.log_format
    if fmt == 'tqdm' and not sys.stderr.isatty():
        fmt = 'simple'
    bars = {'json': json_progress_bar, 'none': noop_progress_bar, 'simple': simple_progress_bar,
            'tqdm': simple_progress_bar}
    if fmt not in bars:
        raise ValueError('Unknown log format: {}'.format(fmt))
    return bars[fmt](iterator, epoch, prefix, args.log_interval)


def format_stat(stat):
    """Text of one stat as the reference prints it."""
    if torch.is_tensor(stat):
        stat = stat.item()
    if isinstance(stat, Number):
        return '{:g}'.format(stat)
    kinds = ((AverageMeter, lambda m: '{:.3f}'.format(m.avg)),
             (TimeMeter, lambda m: '{:g}'.format(round(m.avg))),
             (StopwatchMeter, lambda m: '{:.4f}'.format(m.sum)))
    for kind, fmt in kinds:
        if isinstance(stat, kind):
            return fmt(stat)
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


def _text_items(stats):
    return [(k, str(format_stat(v)).strip()) for k, v in stats.items()]


class progress_bar(object):
    """Base bar: wraps an iterable, remembers the stats last passed to ``log`` and
    renders them on every ``log_interval``-th iteration (counted from the resume offset)."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=None):
        self.iterable = iterable
        self.offset = getattr(iterable, 'offset', 0)
        self.epoch = epoch
        self.log_interval = log_interval
        self.stats = None
        head = []
        if epoch is not None:
            head.append('| epoch {:03d}'.format(epoch))
        if prefix is not None:
            head.append(' | {}'.format(prefix))
        self.prefix = ''.join(head)

    def __len__(self):
        return len(self.iterable)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

    def __iter__(self):
        size = len(self.iterable)
        for i, obj in enumerate(self.iterable, start=self.offset):
            yield obj
            if self._due(i):
                line = self._render_interval(i, size, self.stats)
                if line is not None:
                    print(line, flush=True)

    def _due(self, i):
        return self.stats is not None and i > 0 and self.log_interval is not None and i % self.log_interval == 0

    def log(self, stats, tag='', step=None):
        """Stats to show at the next logging iteration (rendered then, not now)."""
        self.stats = stats

    def print(self, stats, tag='', step=None):
        """End-of-epoch / validation summary line."""
        line = self._render_summary(stats, tag)
        if line is not None:
            print(line, flush=True)

    def _render_interval(self, i, size, stats):
        return None

    def _render_summary(self, stats, tag):
        return None


class noop_progress_bar(progress_bar):
    """No output."""


class simple_progress_bar(progress_bar):
    """The reference's line format, for non-TTY environments."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix, log_interval)

    def _render_interval(self, i, size, stats):
        body = ', '.join('{}={}'.format(k, v) for k, v in _text_items(stats))
        return '{}:  {:5d} / {:d} {}'.format(self.prefix, i, size, body)

    def _render_summary(self, stats, tag):
        body = ' | '.join('{} {}'.format(k, v) for k, v in _text_items(stats))
        return '{} | {}'.format(self.prefix, body)


class json_progress_bar(progress_bar):
    """One JSON object per logged iteration (machine-readable log)."""

    def __init__(self, iterable, epoch=None, prefix=None, log_interval=1000):
        super().__init__(iterable, epoch, prefix, log_interval)

    def _record(self, head, stats):
        rec = OrderedDict(head)
        rec.update((k, _json_stat(v)) for k, v in stats.items())
        return json.dumps(rec)

    def _render_interval(self, i, size, stats):
        update = self.epoch - 1 + float(i / float(size)) if self.epoch is not None else None
        return self._record([('epoch', self.epoch), ('update', update)], stats)

    def _render_summary(self, stats, tag):
        return self._record([('epoch', self.epoch), ('tag', tag)], stats)
