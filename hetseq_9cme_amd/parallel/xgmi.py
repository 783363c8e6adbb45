"""Intra-node xGMI all-reduce transport for the gradient reducer.

``--allreduce-impl xgmi`` replaces RCCL for the per-bucket gradient all-reduce
 with the two-shot kernel of
``csrc/kernels/xgmi_allreduce.hip``: every rank exports one staging buffer and
one uncached signal page through HIP IPC, maps its peers' (exchanged with
``all_gather_object`` over the existing process group, which plays the role of
the reference's TCP/file store, hetseq/distributed_utils.py:20-25), and each
bucket is reduced by pulling chunk r from all W peers at once (all 7 xGMI links
busy) and gathering the other W-1 reduced chunks.

It applies only when every rank of the group lives on one host and holds its
own GPU with peer access to the others (or, for tests, when ranks share one
GPU); otherwise the reducer stays on RCCL (multi-node, CPU/gloo).  RCCL also
keeps the one-off parameter broadcast and the small stats all-reduce.

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


def xgmi_eligible(group=None):
    """(ok, reason): can this process group use the xGMI transport?"""
    if not (dist.is_initialized() and torch.cuda.is_available()):
        return False, 'needs an initialised process group on GPUs'
    world = dist.get_world_size(group)
    if world < 2 or world > MAX_WORLD:
        return False, 'world size {} outside 2..{}'.format(world, MAX_WORLD)
    dev = torch.cuda.current_device()
    info = [None] * world
    dist.all_gather_object(info, (socket.gethostname(), dev), group=group)
    if len({h for h, _ in info}) != 1:
        return False, 'ranks span several hosts (xGMI is intra-node)'
    for _, d in info:
        if d != dev and not torch.cuda.can_device_access_peer(dev, d):
            return False, 'no peer access from GPU {} to GPU {}'.format(dev, d)
    return True, ''


class XgmiAllReduce(object):
    """In-place SUM all-reduce of fp32 buckets over IPC-mapped peer buffers.

    Collective: every rank must construct it and call :meth:`all_reduce_` with
    buckets of identical sizes in identical order.
    """

    def __init__(self, group=None, cap_mb=64, blocks=64, timeout_s=300.0):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        cap = int(cap_mb * 1024 * 1024 // 4)
        self.h = C().xar_create(self.rank, self.world, cap, blocks, float(timeout_s))
        handles = [None] * self.world
        dist.all_gather_object(handles, C().xar_export(self.h), group=group)
        C().xar_open(self.h, b''.join(handles))
        # every rank has mapped every peer before any kernel may touch a peer page
        torch.cuda.synchronize()
        dist.barrier(group=group)
        self.stream = torch.cuda.Stream(priority=-1)

    @property
    def capacity(self):
        return C().xar_capacity(self.h)

    def all_reduce_(self, t):
        """Reduce ``t`` (contiguous fp32 GPU tensor) on the CURRENT stream."""
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

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def simulate_all_reduce(bufs, blocks=64, timeout_s=20.0, mute=-1):
    """Test helper: W simulated ranks in ONE grid on one GPU (no IPC); reduces the
    equal-size fp32 tensors ``bufs`` in place and returns the error word.
    ``mute`` = a simulated rank that never signals (the others' waits time out)."""
    W = len(bufs)
    cap = max(64, bufs[0].numel())
    hs = [C().xar_create(q, W, cap, blocks, float(timeout_s)) for q in range(W)]
    try:
        C().xar_allreduce_sim(hs, list(bufs), int(mute))
        torch.cuda.synchronize()
        return max(C().xar_error(h) for h in hs)
    finally:
        for h in hs:
            C().xar_destroy(h)
