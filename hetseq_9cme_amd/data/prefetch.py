"""Host -> device staging on a dedicated HIP copy stream.

The reference moves every micro-batch with a synchronous, pageable ``.cuda()``
inside the training step (hetseq/utils.py:32-37).  Here loader
threads read the batch into PINNED host memory (native HDF5 reader), then
enqueue ``hipMemcpyAsync`` (``non_blocking`` copies) on a per-device copy stream
and record an event.  The training step only makes the compute stream wait on
that event, so the copy overlaps with the previous step's forward/backward and
the host never blocks on H2D.

``DevicePrefetcher`` is a standalone wrapper with the same behaviour for any
iterator of host batches (used by tools/benchmarks).
"""
import threading

import torch

from ..utils.misc import apply_to_sample


class DeviceBatch(object):
    """A batch already enqueued for the device on the copy stream."""
    __slots__ = ('sample', 'event')

    def __init__(self, sample, event):
        self.sample = sample
        self.event = event

    def __len__(self):
        return len(self.sample)

    def wait(self, stream=None):
        stream = stream or torch.cuda.current_stream()
        if self.event is not None:
            stream.wait_event(self.event)

        def _rec(t):
            t.record_stream(stream)
            return t
        apply_to_sample(_rec, self.sample)
        return self.sample


_streams = {}
_lock = threading.Lock()


def copy_stream(device):
    key = torch.device(device).index
    with _lock:
        if key not in _streams:
            with torch.cuda.device(device):
                _streams[key] = torch.cuda.Stream(device=device)
        return _streams[key]


def stage_to_device(sample, device):
    """Enqueue the H2D copy of ``sample`` on the copy stream; returns DeviceBatch."""
    if sample is None:
        return None
    device = torch.device(device)
    with torch.cuda.device(device):
        s = copy_stream(device)
        with torch.cuda.stream(s):
            dev = apply_to_sample(lambda t: t.to(device, non_blocking=True), sample)
            ev = torch.cuda.Event()
            ev.record(s)
    return DeviceBatch(dev, ev)


def unwrap(sample):
    """Make a (possibly staged) batch usable on the current stream."""
    if isinstance(sample, DeviceBatch):
        return sample.wait()
    return sample


class DevicePrefetcher(object):
    """Iterator wrapper that keeps ``depth`` batches in flight to ``device``."""

    def __init__(self, iterable, device, depth=2):
        self.iterable = iterable
        self.device = torch.device(device)
        self.depth = depth

    def __len__(self):
        return len(self.iterable)

    def __iter__(self):
        it = iter(self.iterable)
        q = []
        for x in it:
            q.append(stage_to_device(x, self.device) if self.device.type == 'cuda' else x)
            if len(q) > self.depth:
                yield unwrap(q.pop(0))
        while q:
            yield unwrap(q.pop(0))
