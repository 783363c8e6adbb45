"""Hand-written in-place all-reduce (csrc/kernels/xgmi_allreduce.hip).

* simulation: W ranks as ONE grid on one GPU (rank = blockIdx.y): one-shot (small buckets)
  and two-shot kernels, chunking for uneven W (3, 5, 7), tails that are not float4
  multiples, buckets smaller than W float4s, repeated calls (monotonic epochs), bitwise
  equality with the rank-order fp32 sum;
* IPC: two or three processes (uneven W) on the box's GPU register their "flat gradient"
  buffers, exchange IPC records over a gloo group and reduce slices of them in place through
  the mapped peer memory (the multi-GPU protocol minus the xGMI links themselves).
Every kernel wait is bounded (timeouts -> error bits, never a spinning GPU).
"""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize('W,n,oneshot_kb', [(2, 4096, 512), (3, 1000003, 512), (5, 77, 512), (7, 5, 512),
                                            (8, 3 * 2 ** 20 + 12, 512), (5, 300001, 512), (7, 131071, 512),
                                            (3, 4099, 0), (8, 40000, 0), (2, 200000, 1024)])
def test_xgmi_allreduce_simulated(dev, W, n, oneshot_kb):
    """oneshot_kb 0 forces the two-shot kernel on small buckets; 16 blocks x 256 threads x 16
    floats = 64K floats is the one-shot limit of these grids."""
    from hetseq_9cme_amd.parallel.xgmi import simulate_all_reduce
    g = torch.Generator(device='cpu').manual_seed(W * 1000 + n % 997)
    for it in range(2):
        src = [torch.randn(n, generator=g).to(dev) for _ in range(W)]
        ref = src[0].clone()
        for q in range(1, W):
            ref += src[q]
        bufs = [s.clone() for s in src]
        err = simulate_all_reduce(bufs, blocks=16, timeout_s=20.0, oneshot_kb=oneshot_kb)
        assert err == 0, 'kernel wait timed out (phase bits {:#x})'.format(err)
        for q in range(W):
            assert torch.equal(bufs[q], ref), (it, q, (bufs[q] - ref).abs().max().item())


def test_xgmi_timeout_sets_error_and_the_step_check_raises(dev):
    """A simulated rank that never signals: the others' bounded waits expire, the kernel
    drains, the error word is set, and the stream-ordered copy of it (what the controller
    folds into the stats all-reduce) makes TransportErrorMonitor raise two updates later."""
    from hetseq_9cme_amd.ops._ext import C
    from hetseq_9cme_amd.parallel.reducer import TransportErrorMonitor
    W, n = 3, 4096
    hs = [C().xar_create(q, W, 4, 0.05, 0) for q in range(W)]
    try:
        bufs = [torch.ones(n, device=dev) for _ in range(W)]
        C().xar_allreduce_sim(hs, bufs, 1)           # rank 1 muted
        torch.cuda.synchronize()
        words = [C().xar_error(h) for h in hs]
        assert words[0] != 0 and words[2] != 0, words
        out = torch.zeros(1, dtype=torch.int32, device=dev)
        C().xar_error_async(hs[0], out)
        mon = TransportErrorMonitor(lag=2)
        mon.record(1, out.double())
        mon.record(2, torch.zeros(1, dtype=torch.float64, device=dev))
        mon.check()                                    # update 1 not yet due
        mon.record(3, torch.zeros(1, dtype=torch.float64, device=dev))
        with pytest.raises(RuntimeError, match='update 1'):
            mon.check()
    finally:
        for h in hs:
            C().xar_destroy(h)


WORKER = textwrap.dedent('''
    import os, sys, time, torch, torch.distributed as dist
    sys.path.insert(0, os.environ['ROOT'])
    from hetseq_9cme_amd.parallel.xgmi import XgmiAllReduce, xgmi_eligible
    rank, W = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=W)
    ok, why = xgmi_eligible()
    assert ok, why
    sizes = [7, 4096, 1000003, 3 * 2 ** 20 + 5, 25 * 2 ** 18]
    offs, o = [], 0
    for n in sizes:              # the buckets: 16-B aligned slices of one registered buffer
        offs.append(o)
        o += (n + 63) // 64 * 64
    flat = torch.zeros(o, device='cuda')
    xar = XgmiAllReduce(flat, blocks=32, timeout_s=30.0)
    for it, (n, o) in enumerate(zip(sizes[:4], offs[:4])):
        data = [torch.randn(n, generator=torch.Generator().manual_seed(100 * it + q)).cuda() for q in range(W)]
        ref = data[0].clone()
        for q in range(1, W):
            ref += data[q]          # the kernel's rank-order sum
        buf = flat[o:o + n]
        buf.copy_(data[rank])
        xar.all_reduce_(buf)
        torch.cuda.synchronize()
        xar.check()
        assert torch.equal(buf, ref), (n, (buf - ref).abs().max().item())
    big = flat[offs[4]:offs[4] + sizes[4]]       # one 25 MB bucket, in place
    big.fill_(1.0)
    for _ in range(3):
        xar.all_reduce_(big)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(10):
        xar.all_reduce_(big)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    xar.check()
    assert torch.equal(big, torch.full_like(big, float(W) ** 13)), big[:4]
    if rank == 0:
        print('XAR_OK 25MB bucket {:.1f} us ({} ranks on one GPU)'.format(dt * 1e6, W), flush=True)
    xar.close()
    dist.destroy_process_group()
''')


@pytest.mark.parametrize('W', [2, 3])
def test_xgmi_allreduce_multi_process_ipc(dev, tmp_path, W):
    script = tmp_path / 'xar_worker.py'
    script.write_text(WORKER)
    env = dict(os.environ, ROOT=ROOT, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(29500 + W + os.getpid() % 2000),
               WORLD_SIZE=str(W))
    procs = [subprocess.Popen([sys.executable, '-u', str(script)], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(W)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), '\n----\n'.join(o[-3000:] for o in outs)
    assert 'XAR_OK' in outs[0]
    print([l for l in outs[0].splitlines() if 'XAR_OK' in l][0])
