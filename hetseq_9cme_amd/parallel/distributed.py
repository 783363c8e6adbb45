"""Process-group bring-up and small collectives.

Reference behaviour (hetseq/distributed_utils.py:11-132):
  * ``distributed_init`` joins a ``tcp://host:port`` or ``file:///shared/path``
    rendezvous with the explicit global rank ``node_base_rank + local_gpu``,
    then forces communicator creation with a 1-element all-reduce, then
    silences ``print`` on non-master ranks (``force=True`` escape).
  * ``all_gather_list`` gathers picklable objects with a SUM all-reduce over a
    zeroed byte buffer, 2-byte base-255 length header per rank.

MI355X-native differences:
  * backend ``nccl`` is RCCL over xGMI on MI355X; ``gloo`` is accepted for CPU
    runs.  The backend is chosen per device automatically when the requested
    one cannot serve the device (the reference crashes with ``--cpu`` and
    NCCL).
  * the warm-up collective runs on the rank's own HIP device
    (``torch.cuda.set_device`` happens before init, so RCCL binds the right GPU).
  * ``all_gather_list`` works on CPU and GPU (the reference is CUDA-only).
  * ``--distributed-timeout`` bounds every collective (reference: c10d default).
"""
import builtins
import datetime
import pickle
import socket
import os
import warnings

import torch
import torch.distributed as dist

_BUILTIN_PRINT = builtins.print


def _device_for(args):
    if torch.cuda.is_available() and not getattr(args, 'cpu', False):
        return torch.device('cuda', torch.cuda.current_device())
    return torch.device('cpu')


def _resolve_backend(args):
    backend = args.distributed_backend
    if _device_for(args).type == 'cpu' and backend == 'nccl':
        return 'gloo'
    return backend


def distributed_init(args):
    if args.distributed_world_size == 1 and not getattr(args, 'force_reducer', False):
        # (--force-reducer: a one-rank group on purpose, to drive the collective stream path)
        raise ValueError('Cannot initialize distributed with distributed_world_size=1')
    from ..options import comm_cus
    if comm_cus(args) > 0 and args.distributed_backend == 'nccl':
        # --comm-cus: RCCL's collectives take at most that many CUs (one workgroup per channel);
        # read by RCCL when the communicator is created, so before the first collective
        os.environ.setdefault('NCCL_MAX_NCHANNELS', str(comm_cus(args)))
    if dist.is_initialized():
        warnings.warn('Distributed is already initialized, cannot initialize twice!')
    else:
        print('| distributed init (rank {}): {}'.format(
            args.distributed_rank, args.distributed_init_method), flush=True)
        timeout = datetime.timedelta(seconds=getattr(args, 'distributed_timeout', 1800))
        init_kwargs = dict(
            backend=_resolve_backend(args),
            init_method=args.distributed_init_method,
            world_size=args.distributed_world_size,
            rank=args.distributed_rank,
            timeout=timeout,
        )
        dev = _device_for(args)
        if dev.type == 'cuda':
            # binds the RCCL communicator to this GPU up front (eager init)
            init_kwargs['device_id'] = dev
        if init_kwargs['backend'] == 'nccl' and not getattr(args, 'rccl_normal_priority', False):
            # RCCL kernels on high-priority HIP streams: a bucket all-reduce launched from a
            # gradient hook is dispatched ahead of the backward kernels already queued, so it
            # overlaps with them instead of waiting behind them (the last buckets, produced at
            # the very end of backward, are the only exposed communication)
            try:
                opts = dist.ProcessGroupNCCL.Options()
                opts.is_high_priority_stream = True
                init_kwargs['pg_options'] = opts
            except AttributeError:
                pass
        try:
            dist.init_process_group(**init_kwargs)
        except TypeError:  # older torch without device_id
            init_kwargs.pop('device_id', None)
            dist.init_process_group(**init_kwargs)
        print('| initialized host {} as rank {}'.format(
            socket.gethostname(), args.distributed_rank), flush=True)
        # dummy all-reduce: creates the communicator before the first real bucket
        dist.all_reduce(torch.zeros(1, device=dev))
        suppress_output(is_master(args))
    args.distributed_rank = dist.get_rank()
    return args.distributed_rank


def is_master(args):
    return args.distributed_rank == 0


def suppress_output(is_master):
    """Suppress ``print`` on non-master ranks.  ``print(..., force=True)`` still prints."""
    def _print(*a, **kw):
        force = kw.pop('force', False)
        if is_master or force:
            _BUILTIN_PRINT(*a, **kw)
    builtins.print = _print


def restore_output():
    builtins.print = _BUILTIN_PRINT


def get_rank():
    return dist.get_rank() if dist.is_initialized() else 0


def get_world_size():
    return dist.get_world_size() if dist.is_initialized() else 1


def get_default_group():
    return dist.group.WORLD


def all_reduce(tensor, group=None, op=None):
    if group is None:
        group = get_default_group()
    kw = {} if op is None else {'op': op}
    return dist.all_reduce(tensor, group=group, **kw)


_GATHER_BUF = {}


def all_gather_list(data, group=None, max_size=16384):
    """Gather arbitrary picklable ``data`` from every rank (list indexed by rank).

    Same wire format as the reference: each rank owns a ``max_size`` slot of a
    zeroed byte buffer, writes ``[len//255, len%255, pickle...]`` and a SUM
    all-reduce assembles the slots.  The buffer lives on the collective's
    device (GPU for RCCL, CPU for gloo)."""
    rank = get_rank()
    world_size = get_world_size()
    backend = dist.get_backend(group) if dist.is_initialized() else 'gloo'
    dev = (torch.device('cuda', torch.cuda.current_device())
           if backend == 'nccl' else torch.device('cpu'))
    buffer_size = max_size * world_size
    key = (dev.type, buffer_size)
    if key not in _GATHER_BUF:
        _GATHER_BUF[key] = torch.zeros(buffer_size, dtype=torch.uint8, device=dev)
    buffer = _GATHER_BUF[key]
    buffer.zero_()
    enc = pickle.dumps(data)
    enc_size = len(enc)
    if enc_size + 2 > max_size:
        raise ValueError('encoded data exceeds max_size: {}'.format(enc_size + 2))
    assert max_size < 255 * 256
    header = bytes([enc_size // 255, enc_size % 255])
    payload = torch.frombuffer(bytearray(header + enc), dtype=torch.uint8)
    start = rank * max_size
    buffer[start:start + enc_size + 2].copy_(payload)
    if world_size > 1:
        all_reduce(buffer, group=group)
    host = buffer.cpu().numpy().tobytes()
    try:
        result = []
        for i in range(world_size):
            out = host[i * max_size:(i + 1) * max_size]
            size = 255 * out[0] + out[1]
            if size > 0:
                result.append(pickle.loads(out[2:size + 2]))
        return result
    except pickle.UnpicklingError:
        raise Exception(
            'Unable to unpickle data from other workers. all_gather_list requires all '
            'workers to enter the function together, so this error usually indicates '
            'that the workers have fallen out of sync somehow (OOM on one rank, or one '
            'worker finishing an epoch while the others are still iterating).')


def barrier():
    if dist.is_initialized():
        dist.barrier()
