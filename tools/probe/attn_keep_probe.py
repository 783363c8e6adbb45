"""Where the fp16x3 attention kernels spend their time: forward and backward at BERT-base phase-1 /
phase-2 shapes with dropout (keep 0.9: Philox in the forward, the stored bitmask in the backward)
and without (keep 1.0), HIP-event timed over back-to-back launches.
``python tools/probe/attn_keep_probe.py``"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, n=30):
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
    for B, S in ((128, 128), (32, 512)):
        qkv = torch.randn(B, S, 3 * H, device=dev)
        bias = 0.1 * torch.randn(3 * H, device=dev)
        mb = torch.zeros(B, S, device=dev)
        dout = torch.randn(B, S, H, device=dev)
        slots = [torch.empty(H, device=dev) for _ in range(3)]
        for keep in (0.9, 1.0):
            am = torch.empty(B * S, nh, device=dev)
            cm = torch.empty(B * ((S + 127) // 128), H, device=dev)
            fw = timed(lambda: C().attn_fwd_f16(qkv, mb, nh, keep, seed, 3, bias, am, cm))
            out, lse, dm = C().attn_fwd_f16(qkv, mb, nh, keep, seed, 3, bias, am, cm)[:3]
            bw = timed(lambda: C().attn_bwd_f16(dout, qkv, mb, out, lse, dm, nh, keep, bias, *slots))
            print('B={} S={} keep={}: forward {:.1f} us, backward {:.1f} us'.format(B, S, keep, fw, bw), flush=True)


if __name__ == '__main__':
    main()
