"""Gradient reducer: bucketed, backward-overlapped all-reduce over RCCL/xGMI.

Replaces ``torch.nn.parallel.DistributedDataParallel`` as used by the
reference (hetseq/controller.py:75-90).  The per-parameter
and per-bucket machinery is native C++ (``csrc/native/reducer.cpp``, class
``_C.Reducer``); this module plans the buckets and wraps it:

* initial parameter broadcast from rank 0 (one collective over the flat
  parameter buffer instead of DDP's coalesced per-tensor broadcast);
* buckets are contiguous slices of the flat gradient buffer
  (``FlatParamSpace``), so RCCL all-reduces them in place -- no copy into
  bucket storage and back;
* a C++ post-accumulate-grad hook per parameter counts readiness; buckets are
  launched strictly in index order (identical collective sequence on every
  rank, even with unused parameters) as soon as they fill, overlapping the
  all-reduce with the rest of backward;
* an end-of-backward engine callback flushes buckets holding unused parameters
  (``--find-unused-parameters``) and makes the compute stream wait for the
  collectives (no host blocking);
* ``no_sync()`` accumulates locally for ``--update-freq`` > 1;
* the all-reduce is a plain SUM; the 1/W averaging that DDP applies is
  exposed as ``grad_prescale`` and folded into the single fused
  norm/clip/optimizer kernels (no separate scaling pass).

Bucket sizing for MI355X: RCCL's intra-node all-reduce drives the 7 xGMI
links of a fully connected 8-GPU node concurrently; a bucket only needs to be
large enough that each of the W ring/tree chunks amortises the per-step
latency (≈ a few MB per peer).  ``--bucket-cap-mb`` keeps the reference's
default of 25 MB.  Bucket boundaries fall on parameter starts, which the flat
layout places on 64-element (256 B) boundaries; the xGMI kernel rounds its
per-peer chunks up to 64 elements itself, so every chunk is 256 B aligned for
uneven worlds (W = 3, 5, ...) without padding the buckets.

Unused parameters (``--find-unused-parameters``): DDP gives a parameter that
this rank did not use, but another rank did, the reduced gradient on every
rank.  ``global_used`` therefore ORs the per-step used flags across ranks, and
the optimizer skips only parameters that NO rank used (the reference's
``grad is None`` skip), so replicas and per-parameter step counters agree.

``use_xgmi()`` swaps the per-bucket transport for the hand-written intra-node
two-shot xGMI kernel (``parallel/xgmi.py``): buckets are then reduced on a
dedicated high-priority HIP stream that waits for the producing stream(s), and
the end-of-backward callback makes the compute stream wait for it.
"""
import warnings
import contextlib

import torch
import torch.distributed as dist

from ..ops._ext import C


def bucket_cap_for(world, bucket_cap_mb, peer_mb=3.0):
    """Bucket size (MB) for a world of W ranks: each of the W chunks of a bucket (the two-shot
    kernel's per-peer share; RCCL's ring/tree pieces alike) about ``peer_mb``, bounded by the
    reference's ``--bucket-cap-mb`` (hetseq/options.py:215-216): W = 8 -> 24 MB (3 MB per peer
    over 7 concurrent xGMI links), W = 3 -> 9 MB, W = 5 -> 15 MB."""
    if not peer_mb or peer_mb <= 0 or world < 2:
        return bucket_cap_mb
    return min(float(bucket_cap_mb), peer_mb * max(2, world))


def plan_buckets(flat, bucket_cap_mb, world=1, peer_mb=0.0):
    """Contiguous buckets over the flat layout (params already reverse-ordered):
    [(start, end, [param idx])], ends extended to the next bucket's start.  Bucket starts fall
    on parameter starts (64-element = 256-B boundaries in the flat layout), and the transports
    cut a bucket into W chunks rounded up to 64 elements, so every per-peer chunk is 256-B
    aligned for any W (3, 5, ...)."""
    elem = flat.grad_flat.element_size()
    cap = max(1, int(bucket_cap_for(world, bucket_cap_mb, peer_mb) * 1024 * 1024 / elem))
    buckets = []
    cur, cur_start = [], 0
    for i in range(len(flat.params)):
        s, e = flat.param_range(i)
        if cur and (e - cur_start) > cap:
            end = flat.param_range(cur[-1])[1]
            buckets.append([cur_start, end, cur])
            cur, cur_start = [], s
        cur.append(i)
    if cur:
        buckets.append([cur_start, flat.numel, cur])
    # extend bucket ends to the next bucket start (covers alignment padding)
    for b in range(len(buckets) - 1):
        buckets[b][1] = buckets[b + 1][0]
    buckets[-1][1] = flat.numel
    return buckets


class GradReducer(object):
    def __init__(self, flat, bucket_cap_mb=25, process_group=None, find_unused_parameters=False,
                 broadcast_params=True, bucket_peer_mb=0.0, force=False):
        """``force``: reduce even in a one-rank group (``--force-reducer``): every bucket still
        goes through the transport's stream machinery (RCCL / xGMI), which a one-GPU box can
        then exercise; the sum over one rank leaves the gradients unchanged."""
        self.flat = flat
        self.force = bool(force) and dist.is_initialized()
        self.group = process_group
        self.world_size = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.find_unused = find_unused_parameters
        self.grad_prescale = 1.0 / self.world_size
        self.buckets = plan_buckets(flat, bucket_cap_mb, self.world_size, bucket_peer_mb)
        self.bucket_of = {}
        for b, (_, _, idxs) in enumerate(self.buckets):
            for i in idxs:
                self.bucket_of[i] = b
        self.xgmi = None
        # C++ post-accumulate hooks on every parameter: they record which parameters this
        # backward reached (and, multi-rank, launch buckets as they fill).  A single process used
        # to infer the used set from gradient version counters after backward, but every slot is
        # a view of ONE flat buffer and views share the version counter, so any write marked
        # every parameter with a defined gradient as used -- e.g. the NER pooler (never reached)
        # was stepped from its second update on, while the reference never steps it.
        pg = None
        if self.world_size > 1 or self.force:
            pg = process_group if process_group is not None else dist.group.WORLD
        bounds = [b[0] for b in self.buckets] + [flat.numel]
        self._native = C().Reducer(flat.grad_flat, list(flat.params), list(flat.offsets), bounds,
                                   [self.bucket_of[i] for i in range(len(flat.params))], pg, self.world_size,
                                   self.force)
        self._enabled = self.world_size > 1 or self.force
        if self.enabled and broadcast_params:
            dist.broadcast(flat.param_flat, src=0, group=self.group)

    # ------------------------------------------------------------------
    @property
    def enabled(self):
        return self._enabled

    @enabled.setter
    def enabled(self, flag):
        # e.g. --use-bmuf: keep the hooks (used flags / slot adoption), never reduce
        self._enabled = bool(flag) and (self.world_size > 1 or self.force)
        self._native.set_enabled(self._enabled)

    @property
    def used(self):
        return self._native.used()

    @property
    def _sync(self):
        return self._native.sync()

    def use_xgmi(self, blocks=64, timeout_s=1800.0, comm_cus=0):
        """Reduce gradient buckets with the intra-node xGMI kernel (collective call).
        Returns False (and keeps RCCL) when the group is not eligible."""
        from .xgmi import XgmiAllReduce, xgmi_eligible
        if not self.enabled or self.flat.grad_flat.dtype != torch.float32:
            return False
        ok, why = xgmi_eligible(self.group)
        if not ok:
            warnings.warn('--allreduce-impl xgmi unavailable ({}); using RCCL'.format(why))
            return False
        # buckets are slices of the flat gradient buffer: it is registered once and every bucket
        # is reduced in place over the peers' mappings of it (no staging copy)
        self.xgmi = XgmiAllReduce(self.flat.grad_flat, self.group, blocks=blocks, timeout_s=timeout_s,
                                  comm_cus=comm_cus)
        self._native.use_xgmi(self.xgmi.h, self.xgmi.stream.cuda_stream)
        return True

    def set_comm_cus(self, n):
        """--comm-cus: from the first bucket collective of a backward to its end, the GEMM /
        weight-gradient plans leave ``n`` CUs to the collectives (csrc/kernels/cu_reserve.hip)."""
        self._native.set_comm_cus(int(n))

    def check_transport(self):
        """Raise if the xGMI transport reported a timed-out wait (synchronising)."""
        if self.xgmi is not None:
            self.xgmi.check()

    def transport_error_async(self):
        """The xGMI error word as a 1-element float64 device tensor, copied on the
        current stream after every bucket of this step (no host sync), or None
        when buckets go over RCCL."""
        if self.xgmi is None:
            return None
        torch.cuda.current_stream().wait_stream(self.xgmi.stream)
        return self.xgmi.error_async().double()

    def global_used(self, step_used):
        """Per-parameter 'received a gradient this step' flags, OR-ed over ranks.

        Slow path (host-synchronising: a MAX all-reduce + ``.tolist()``), taken only with
        ``--find-unused-parameters`` WITHOUT ``--fast-stat-sync``; the fast path carries the flags
        in the stats all-reduce and the optimizer consumes them on device (controller.py).

        Without ``--find-unused-parameters`` every parameter takes part in every
        reduction (DDP's contract), so all are treated as used and no collective
        is needed.  With it, one small MAX all-reduce of the flags runs (the
        fine-tuning configurations, where a host read per step is cheap)."""
        if not self.enabled:
            return list(step_used)
        if not self.find_unused:
            return [True] * len(step_used)
        dev = self.flat.grad_flat.device
        t = torch.tensor([1 if u else 0 for u in step_used], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return [bool(v) for v in t.tolist()]

    # ------------------------------------------------------------------
    def prepare_for_backward(self):
        """Called before each micro-batch's forward; returns the previous micro-batch's
        used flags."""
        return self._native.prepare()

    def after_backward(self):
        """Called after each micro-batch's backward. When no gradient hook fired
        (the loss reached no parameter, or the task skipped backward), finalize
        here: unused slots are zeroed and this rank still joins every bucket
        collective the other ranks launch instead of leaving them waiting."""
        self._native.after_backward()

    @contextlib.contextmanager
    def no_sync(self):
        old = self._native.sync()
        self._native.set_sync(False)
        try:
            yield
        finally:
            self._native.set_sync(old)

    def all_reduce_now(self):
        """Synchronously reduce the whole gradient buffer (used when a rank ran
        no backward this step, e.g. a pure dummy update)."""
        if self.enabled:
            self._native.all_reduce_now()

    def remove(self):
        self._native.remove_hooks()
        if self.xgmi is not None:
            self._native.drop_xgmi()
            self.xgmi.close()
            self.xgmi = None


class TransportErrorMonitor(object):
    """Deferred, collective check of the xGMI transport's error word.

    The controller puts the error word into the per-step stats vector, so after
    the stats all-reduce every rank holds the SAME sum.  ``record`` copies that
    element to pinned host memory on the stream (no host sync); ``check`` reads
    the value recorded ``lag`` updates earlier -- long finished, because the host
    runs at most about one step ahead -- and raises on every rank at the same
    update when any rank's wait timed out.  Replaces a check that ran only when
    ``--check-params-every`` was set or on rank 0's checkpoint save.
    """

    def __init__(self, lag=2):
        self.lag = lag
        self._pending = []

    def record(self, update, err_reduced):
        e = err_reduced.detach().reshape(1)
        if e.is_cuda:
            host = torch.empty(1, dtype=e.dtype, pin_memory=True)
            host.copy_(e, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = e.clone(), None
        self._pending.append((update, host, ev))

    def check(self, force=False):
        while self._pending and (force or len(self._pending) > self.lag):
            update, host, ev = self._pending.pop(0)
            if ev is not None:
                ev.synchronize()
            if float(host[0]) != 0.0:
                self._pending = []
                raise RuntimeError('xGMI all-reduce: a peer did not arrive within the timeout during update {} '
                                   '(error bits summed over ranks: {:#x}); its gradients are invalid'
                                   .format(update, int(host[0])))
