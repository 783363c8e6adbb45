"""Probe: token-split count of the split-piece weight-gradient kernel (tile config 1,
256 x 128) at BERT-base shapes, T = 16384, bf16x6.  The shipped plan fills ONE round of
workgroup slots (nsplit = 256 // tiles), which leaves 40 of 256 CUs idle for the FFN and QKV
shapes; this sweep times other split counts, interleaved, median of 30 per point."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hetseq_9cme_amd import ops  # noqa: E402
from hetseq_9cme_amd.ops import split_gemm as sg  # noqa: E402
from hetseq_9cme_amd.ops._ext import C  # noqa: E402


def timeit(fn, iters=30, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


ops.set_fp32_gemm('bf16x6')
T = 16384
for (n_out, n_in) in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
    dy = torch.randn(T, n_out, device='cuda')
    x = torch.randn(T, n_in, device='cuda')
    dys, xs = sg.grad_planes(dy), sg.planes(x, sg.ORDER_P[6])
    slot = torch.empty(n_out, n_in, device='cuda')
    po, px = sg._piece_offsets(sg.ORDER_Q[6], n_out), sg._piece_offsets(sg.ORDER_P[6], n_in)
    fl = 2.0 * T * n_out * n_in * 6
    res = {}
    for rnd in range(2):
        for ns in (0, 3, 4, 5, 6, 7, 8, 9, 10, 12, 14, 16, 20, 28):
            if ns:
                os.environ['HX_WGRAD_SPLIT_CFG'] = '1:{}'.format(ns)
            else:
                os.environ.pop('HX_WGRAD_SPLIT_CFG', None)
            us = timeit(lambda: C().wgrad_split(dys, po, xs, px, 6, n_out, n_in, slot))
            res[ns] = min(res.get(ns, 1e9), us)
    os.environ.pop('HX_WGRAD_SPLIT_CFG', None)
    best = min(res, key=res.get)
    print('[{}x{}] '.format(n_out, n_in) + ' '.join('{}:{:.0f}'.format(k or 'plan', v) for k, v in res.items()) +
          '  best {} ({:.0f} TF/s vs plan {:.0f})'.format(best or 'plan', fl / res[best] / 1e6, fl / res[0] / 1e6),
          flush=True)
