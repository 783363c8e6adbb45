"""Attention kernels (backward, and forward timings) side by side at the BERT-base shapes: the fp16x3
kernel (attention_f16.hip) and the fp32-MFMA kernel (attention.hip) -- time per
call (HIP events over back-to-back launches) and the worst-row error of dQ / dK / dV against an
fp64 reference on a small slice.  ``python tools/probe/attn_bwd_probe.py``."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    nh, d = 12, 64
    H = nh * d
    seed = torch.tensor([1234], dtype=torch.int64, device=dev)
    for B, S in ((128, 128), (32, 512), (32, 128)):
        qkv = torch.randn(B, S, 3 * H, device=dev)
        bias = 0.1 * torch.randn(3 * H, device=dev)
        mb = torch.zeros(B, S, device=dev)
        keep = 0.9
        out, lse, dm = C().attn_fwd(qkv, mb, nh, keep, seed, 3, bias)
        dout = torch.randn(B, S, H, device=dev)
        slots = [torch.empty(H, device=dev) for _ in range(3)]
        res = {}
        for name, f in (('f16', C().attn_bwd_f16), ('fp32', C().attn_bwd)):
            res[name] = timed(lambda: f(dout, qkv, mb, out, lse, dm, nh, keep, bias, *slots))
        fw = {}
        for name, f in (('f16', C().attn_fwd_f16), ('fp32', C().attn_fwd)):
            fw[name] = timed(lambda: f(qkv, mb, nh, keep, seed, 3, bias))
        print('B={} S={} forward: '.format(B, S) + ', '.join('{} {:.1f} us'.format(k, v) for k, v in fw.items()),
              flush=True)
        flops = 5 * 2 * B * nh * S * S * d
        print('B={} S={}: '.format(B, S) + ', '.join(
            '{} {:.1f} us ({:.0f} TF/s fp32-equiv)'.format(k, v, flops / v * 1e-6) for k, v in res.items()),
            flush=True)
    # accuracy on a slice: worst row of each gradient vs fp64
    B, S = 2, 512
    qkv = torch.randn(B, S, 3 * H, device=dev)
    mb = torch.zeros(B, S, device=dev)
    out, lse, dm = C().attn_fwd(qkv, mb, nh, 1.0, seed, 3, None)
    dout = torch.randn(B, S, H, device=dev)
    x = qkv.double().requires_grad_(True)
    q = x.view(B, S, 3, nh, d).permute(2, 0, 3, 1, 4)
    p = torch.softmax(q[0] @ q[1].transpose(-1, -2) / 8.0, -1)
    (p @ q[2]).permute(0, 2, 1, 3).reshape(B, S, H).backward(dout.double())
    gref = x.grad.view(B, S, 3, nh, d)
    for name, f in (('f16', C().attn_bwd_f16), ('fp32', C().attn_bwd)):
        g = f(dout, qkv, mb, out, lse, dm, nh, 1.0, None, None, None, None)[0].double().view(B, S, 3, nh, d)
        e = ((g - gref).abs().amax(-1) / gref.abs().amax(-1)).amax((0, 1, 3))
        print('{:5s} worst-row rel err dQ {:.2e} dK {:.2e} dV {:.2e}'.format(name, *e.tolist()), flush=True)


if __name__ == '__main__':
    main()
