"""Per-phase timing of the training step (``--profile-phases``).

SURVEY §5.1: the reference has only wall-clock meters around the whole step and
one NVTX range.  Here each phase of ``Controller.train_step`` (prep, sample,
forward, backward, stats, optimizer, meters) is

* a **roctx range** (``torch.cuda.nvtx`` is routed to roctx on ROCm), so
  ``rocprofv3 --marker-trace`` / the trace viewer shows the phases around the
  kernels;
* a **host wall-time** interval (where the Python thread spends its time: with no
  host syncs in the step every phase is short, and a phase that blocks on the
  device shows up as long);
* a **device interval** between two HIP events recorded on the compute stream
  (how long the GPU spends on the work enqueued in that phase).  Events are
  resolved lazily -- only completed events are read during training, the rest
  when a report is requested -- so timing never adds a host sync to the step.
"""
import time
from collections import deque

import torch


class PhaseTimer(object):
    def __init__(self, enabled=False, cuda=False, use_roctx=True):
        self.enabled = bool(enabled)
        self.cuda = bool(cuda) and torch.cuda.is_available()
        self.use_roctx = use_roctx and self.cuda
        self.host = {}
        self.device = {}
        self.steps = 0
        self._cur = None
        self._t0 = 0.0
        self._ev0 = None
        self._pending = deque()
        self.lead_trace = None   # list -> also record (phase, host time, event) for host-lead analysis

    def begin(self, name):
        """Close the open phase (if any) and open ``name`` (None: just close)."""
        if not self.enabled:
            return
        now = time.perf_counter()
        ev = None
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        if self._cur is not None:
            self.host[self._cur] = self.host.get(self._cur, 0.0) + now - self._t0
            if ev is not None and self._ev0 is not None:
                self._pending.append((self._cur, self._ev0, ev))
            if self.use_roctx:
                torch.cuda.nvtx.range_pop()
        self._cur, self._t0, self._ev0 = name, now, ev
        if self.lead_trace is not None and ev is not None and name is not None:
            self.lead_trace.append((name, now, ev))
        if name is not None and self.use_roctx:
            torch.cuda.nvtx.range_push(name)
        self._drain(block=False)

    def end_step(self):
        self.begin(None)
        if self.enabled:
            self.steps += 1

    def _drain(self, block):
        while self._pending:
            name, a, b = self._pending[0]
            if not block and not b.query():
                break
            if block:
                b.synchronize()
            self.device[name] = self.device.get(name, 0.0) + a.elapsed_time(b) / 1e3
            self._pending.popleft()

    def host_lead(self, t0, ev0):
        """After a synchronize: per phase, how far the host ran ahead of the device when it
        opened the phase (ms; mean and min over the trace).  ~0 means the GPU was starved at
        that point (launch-bound); large values mean the host had work queued in advance."""
        out = {}
        for name, th, ev in self.lead_trace or []:
            lead = ev0.elapsed_time(ev) - (th - t0) * 1e3
            out.setdefault(name, []).append(lead)
        self.lead_trace = None
        return {k: (sum(v) / len(v), min(v)) for k, v in out.items()}

    def report(self, reset=True):
        """{'host': {phase: seconds}, 'device': {phase: seconds}, 'steps': n}."""
        self._drain(block=True)
        out = {'host': dict(self.host), 'device': dict(self.device), 'steps': self.steps}
        if reset:
            self.host, self.device, self.steps = {}, {}, 0
        return out
