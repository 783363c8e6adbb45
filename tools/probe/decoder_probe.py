"""Probe: MLM-decoder GEMMs under --fp32-gemm bf16x6 (2560 masked rows, V = 30522, H = 768).

forward  logits = h' [M, 6H] . W'^T  with W' [V, 6H] (V unpadded) vs W' padded to 30528 rows
         (16-B aligned output rows);
wgrad    dW = dl'^T . h' over 6M plane rows: library (current) vs the split-piece kernel with
         the vocabulary padded to a multiple of 256."""
import time

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from hetseq_9cme_amd import ops
from hetseq_9cme_amd.ops import split_gemm as sg
from hetseq_9cme_amd.ops._ext import C


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        for _ in range(it):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / it * 1e6)
    return best


ops.set_fp32_gemm('bf16x6')
M, V, H = 2560, 30522, 768
h = torch.randn(M, H, device='cuda')
W = torch.randn(V, H, device='cuda') * 0.02
dl = torch.randn(M, V, device='cuda') * 1e-3
hs = sg.planes(h, sg.ORDER_P[6])
wq = sg.planes(W, sg.ORDER_Q[6])
Wp = torch.zeros(30528, H, device='cuda')
Wp[:V] = W
wqp = sg.planes(Wp, sg.ORDER_Q[6])
fl = 2.0 * M * V * H * 6
t0 = timeit(lambda: torch.mm(hs, wq.t(), out_dtype=torch.float32))
t1 = timeit(lambda: torch.mm(hs, wqp.t(), out_dtype=torch.float32))
print('fwd V=30522 {:.1f} us ({:.2f} PF)  padded 30528 {:.1f} us ({:.2f} PF)'.format(
    t0, fl / t0 / 1e9, t1, fl / t1 / 1e9), flush=True)
# wgrad, current library form
Vp = 30528
dls = sg.grad_planes(dl, dpad=Vp)
a = dls.view(-1, Vp)[:, :V]
b = hs.view(-1, H)
t2 = timeit(lambda: torch.mm(a.t(), b, out_dtype=torch.float32))
# split-piece kernel over a 256-multiple vocabulary
V2 = 30720
dls2 = sg.grad_planes(dl, dpad=V2)
slot = torch.empty(V2, H, device='cuda')
po, px = sg._piece_offsets(sg.ORDER_Q[6], V2), sg._piece_offsets(sg.ORDER_P[6], H)
ok = C().wgrad_split_ok(dls2, hs, V2, H)
t3 = timeit(lambda: C().wgrad_split(dls2, po, hs, px, 6, V2, H, slot)) if ok else float('nan')
ref = torch.mm(a.t(), b, out_dtype=torch.float32)
err = (slot[:V] - ref).abs().max().item() if ok else float('nan')
print('wgrad library {:.1f} us ({:.2f} PF)  split-piece (V->30720) {:.1f} us ({:.2f} PF) ok={} maxdiff {:.2e}'.format(
    t2, fl / t2 / 1e9, t3, fl / t3 / 1e9, ok, err), flush=True)
