"""Running-statistics meters used by the training engine and the log line.

Behavioural parity with the reference meters (hetseq/meters.py:4-66):
``AverageMeter`` (weighted running mean), ``TimeMeter`` (events per wall
second) and ``StopwatchMeter`` (accumulated stopwatch).

MI355X-first difference: ``AverageMeter`` accepts *device* tensors and keeps
them un-synchronised until ``avg``/``val``/``sum`` is read, so the training
loop never forces a host<->device round trip per step just to update a meter
(the reference calls ``.tolist()`` every update, controller.py:306).
"""
import time

import torch


def _host(x):
    if torch.is_tensor(x):
        return x.item() if x.numel() == 1 else x.tolist()
    return x


class AverageMeter(object):
    """Weighted running average. Values may be python numbers or 0-d tensors."""

    def __init__(self):
        self.reset()

    def reset(self):
        self._val = 0
        self._sum = 0
        self._count = 0

    def update(self, val, n=1):
        """``val`` and the weight ``n`` may be device tensors (summed lazily)."""
        self._val = val
        if torch.is_tensor(n):
            n = n.detach().reshape(())
        if torch.is_tensor(val):
            val = val.detach()
            if torch.is_tensor(self._sum):
                self._sum = self._sum + val * n
            else:
                self._sum = val * n + self._sum
        else:
            self._sum = (n * val + self._sum) if torch.is_tensor(n) else (self._sum + val * n)
        self._count = (n + self._count) if torch.is_tensor(n) else (self._count + n)

    @property
    def count(self):
        self._count = _host(self._count)
        return self._count

    @count.setter
    def count(self, v):
        self._count = v

    @property
    def val(self):
        self._val = _host(self._val)
        return self._val

    @property
    def sum(self):
        self._sum = _host(self._sum)
        return self._sum

    @property
    def avg(self):
        if self.count == 0:
            return 0
        return self.sum / self.count

    # checkpoint support (meters are pickled into extra_state)
    def __getstate__(self):
        return {'_val': _host(self._val), '_sum': _host(self._sum), 'count': self.count}

    def __setstate__(self, state):
        state = dict(state)
        self._count = state.pop('count', 0)
        self.__dict__.update(state)


class TimeMeter(object):
    """Average occurrence of some event per second (counts may be device tensors,
    summed lazily like ``AverageMeter``)."""

    def __init__(self, init=0):
        self.reset(init)

    def reset(self, init=0):
        self.init = init
        self.start = time.time()
        self._n = 0

    def update(self, val=1):
        if torch.is_tensor(val):
            val = val.detach()
        self._n = self._n + val

    @property
    def n(self):
        self._n = _host(self._n)
        return self._n

    @n.setter
    def n(self, v):
        self._n = v

    @property
    def avg(self):
        return self.n / max(self.elapsed_time, 1e-12)

    @property
    def elapsed_time(self):
        return self.init + (time.time() - self.start)

    def __getstate__(self):
        return {'init': self.init, 'start': self.start, '_n': _host(self._n)}

    def __setstate__(self, state):
        if 'n' in state:
            state['_n'] = state.pop('n')
        self.__dict__.update(state)


class StopwatchMeter(object):
    """Sum / average duration of some event in seconds."""

    def __init__(self):
        self.reset()

    def start(self):
        self.start_time = time.time()

    def stop(self, n=1):
        if self.start_time is not None:
            delta = time.time() - self.start_time
            self.sum += delta
            self.n += n
            self.start_time = None

    def reset(self):
        self.sum = 0
        self.n = 0
        self.start_time = None

    @property
    def avg(self):
        return self.sum / self.n if self.n > 0 else 0.0
