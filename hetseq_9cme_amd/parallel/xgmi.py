"""Intra-node xGMI all-reduce transport for the gradient reducer.

``--allreduce-impl xgmi`` replaces RCCL for the per-bucket gradient all-reduce
 with the kernels of ``csrc/kernels/xgmi_allreduce.hip``:
every rank registers its flat gradient buffer and exports it ONCE through HIP IPC
together with an uncached signal page; the records are exchanged with
``all_gather_object`` over the existing process group (the role of the reference's
TCP/file store, hetseq/distributed_utils.py:20-25).  Each bucket -- a slice of that
buffer on every rank -- is then reduced IN PLACE:

* two-shot (large buckets): rank r pulls chunk r of every peer's bucket at once (all 7
  xGMI links busy), sums in rank order into its own chunk, then gathers the other W-1
  reduced chunks from their owners;
* one-shot (buckets up to ``oneshot_kb``, latency-bound): every rank sums the whole bucket
  over all peers in registers and stores it after one "done reading" hand-off.

Eligibility is decided by PCI bus id, not by process-local device ordinals: every rank
must sit on one host, on its own GPU (or share one, for tests), and see each peer's GPU
(by bus id) with peer access.  A launch that partitions ``HIP_VISIBLE_DEVICES`` per
"node" hides the peers and falls back to RCCL; ``tools/launch_hetero.py --device-offset``
keeps every GPU visible for exactly this reason.  RCCL keeps the one-off parameter
broadcast and the small stats all-reduce, and multi-node groups.

Waits inside the kernel are bounded by ``timeout_s``; a wait that expires sets
an error bit instead of hanging the GPU.  :meth:`error_async` copies that word
on the stream (no host sync); the controller folds it into the per-step stats
all-reduce and checks the reduced value two updates later, so every rank
raises at the same update (``TransportErrorMonitor`` in ``reducer.py``).
:meth:`check` is the synchronising local read.
"""
import socket

import torch
import torch.distributed as dist

from ..ops._ext import C

MAX_WORLD = 8


def _visible_bus_ids():
    return [C().device_pci_bus_id(d).lower() for d in range(torch.cuda.device_count())]


def eligibility(infos, rank, can_access):
    """Pure decision (unit-testable): ``infos[q]`` = (hostname, own bus id, tuple of the bus ids
    visible to rank q in ordinal order); ``can_access(a, b)`` = peer access between local
    ordinals a -> b of THIS rank.  Returns (ok, reason)."""
    world = len(infos)
    if world < 2 or world > MAX_WORLD:
        return False, 'world size {} outside 2..{}'.format(world, MAX_WORLD)
    if len({h for h, _, _ in infos}) != 1:
        return False, 'ranks span several hosts (xGMI is intra-node)'
    host, mine, visible = infos[rank]
    me = visible.index(mine)
    for q, (_, bus, _) in enumerate(infos):
        if q == rank or bus == mine:
            continue   # same GPU (tests share one device): plain device memory
        if bus not in visible:
            return False, ('rank {} runs on GPU {} which this process cannot see (HIP_VISIBLE_DEVICES '
                           'partitions the node; launch with all GPUs visible, e.g. '
                           'tools/launch_hetero.py --device-offset)').format(q, bus)
        if not can_access(me, visible.index(bus)):
            return False, 'no peer access from GPU {} to GPU {}'.format(mine, bus)
    return True, ''


def xgmi_eligible(group=None):
    """(ok, reason): can this process group use the xGMI transport?"""
    if not (dist.is_initialized() and torch.cuda.is_available()):
        return False, 'needs an initialised process group on GPUs'
    world = dist.get_world_size(group)
    if world < 2 or world > MAX_WORLD:
        return False, 'world size {} outside 2..{}'.format(world, MAX_WORLD)
    visible = tuple(_visible_bus_ids())
    info = (socket.gethostname(), visible[torch.cuda.current_device()], visible)
    infos = [None] * world
    dist.all_gather_object(infos, info, group=group)
    return eligibility(infos, dist.get_rank(group), torch.cuda.can_device_access_peer)


class XgmiAllReduce(object):
    """In-place SUM all-reduce of slices of ``buffer`` (this rank's flat fp32 gradients) over
    IPC-mapped peer buffers.

    Collective: every rank must construct it with an equally sized buffer and call
    :meth:`all_reduce_` with the same slices in the same order.
    """

    def __init__(self, buffer, group=None, blocks=64, timeout_s=300.0, oneshot_kb=512, comm_cus=0):
        """``comm_cus`` > 0 (--comm-cus): the kernel is confined to that many CUs -- its grid is
        capped at ``comm_cus`` workgroups and it runs on a CU-masked stream over the device's last
        ``comm_cus`` CUs -- the ones the GEMM plans leave free while buckets are in flight
        (csrc/kernels/cu_reserve.hip)."""
        self.group = group
        self._masked = 0
        if comm_cus > 0:
            blocks = max(1, min(blocks, int(comm_cus)))
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.buffer = buffer
        self.h = C().xar_create(self.rank, self.world, blocks, float(timeout_s), int(oneshot_kb) * 1024)
        C().xar_register(self.h, buffer)
        recs = [None] * self.world
        dist.all_gather_object(recs, C().xar_export(self.h), group=group)
        C().xar_open(self.h, b''.join(recs))
        # every rank has mapped every peer before any kernel may touch a peer page
        torch.cuda.synchronize()
        dist.barrier(group=group)
        if comm_cus > 0:
            ncu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
            self._masked = int(C().cu_masked_stream(max(0, ncu - int(comm_cus)), int(comm_cus)))
        if self._masked:
            self.stream = torch.cuda.ExternalStream(self._masked)
        else:
            self.stream = torch.cuda.Stream(priority=-1)

    @property
    def oneshot_max(self):
        """Largest bucket (floats) reduced by the one-shot kernel."""
        return C().xar_oneshot_max(self.h)

    def all_reduce_(self, t):
        """Reduce ``t`` (a contiguous slice of the registered buffer) on the CURRENT stream."""
        C().xar_allreduce(self.h, t)
        return t

    def error_async(self):
        """1-element int32 device tensor receiving the error word, written on the
        current stream (ordered after every all-reduce enqueued before it)."""
        out = torch.empty(1, dtype=torch.int32, device=torch.cuda.current_device())
        C().xar_error_async(self.h, out)
        return out

    def check(self):
        err = C().xar_error(self.h)
        if err:
            raise RuntimeError('xGMI all-reduce: a peer did not arrive within the timeout '
                               '(phase bits {:#x}); gradients of that step are invalid'.format(err))

    def close(self):
        if self.h:
            C().xar_destroy(self.h)
            self.h = 0
        if self._masked:
            C().destroy_stream(self._masked)
            self._masked = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def simulate_all_reduce(bufs, blocks=64, timeout_s=20.0, mute=-1, oneshot_kb=512):
    """Test helper: W simulated ranks in ONE grid on one GPU (no IPC); reduces the
    equal-size fp32 tensors ``bufs`` in place and returns the error word.
    ``mute`` = a simulated rank that never signals (the others' waits time out)."""
    W = len(bufs)
    hs = [C().xar_create(q, W, blocks, float(timeout_s), int(oneshot_kb) * 1024) for q in range(W)]
    try:
        C().xar_allreduce_sim(hs, list(bufs), int(mute))
        torch.cuda.synchronize()
        return max(C().xar_error(h) for h in hs)
    finally:
        for h in hs:
            C().xar_destroy(h)
