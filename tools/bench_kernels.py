"""Micro-benchmarks of the hand-written kernels at BERT-base phase-1 shapes.

``python tools/bench_kernels.py [--batch 128] [--seq 128] [--only attn,ln,...]``
Prints one line per kernel: time per call (HIP events, median of N) and the
achieved FLOP/s or HBM bytes/s against the MI355X peaks (157 TF/s fp32 MFMA,
~8 TB/s HBM3E).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hetseq_9cme_amd.ops._ext import C  # noqa: E402


SEED = None   # dropout key tensor (set in main: kernels read it from device memory)


def timeit(fn, iters=50, warmup=5):
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
    return ts[len(ts) // 2] * 1e3  # us


def report(name, us, flops=None, bytes_=None, peak=157.3):
    extra = []
    if flops:
        extra.append('{:.1f} TF/s ({:.0f}% of {:.0f})'.format(flops / us / 1e6, 100 * flops / us / 1e6 / peak, peak))
    if bytes_:
        extra.append('{:.2f} TB/s'.format(bytes_ / us / 1e6))
    print('{:<28s} {:9.1f} us   {}'.format(name, us, '  '.join(extra)), flush=True)


def _report_peak(peak, tag):
    return lambda name, us, flops=None, bytes_=None: report(tag + name, us, flops, bytes_, peak)


def bench_attn(B, S, nh=12, keep=0.9, dtype=torch.float32):
    d = 64
    peak = 157.3 if dtype == torch.float32 else 2500.0
    qkv = torch.randn(B, S, 3 * nh * d, device='cuda').to(dtype)
    mb = torch.zeros(B, S, device='cuda')
    out, lse, dm = C().attn_fwd(qkv, mb, nh, keep, SEED, 0, None)
    dout = torch.randn_like(out)
    f_fwd = 2 * 2 * B * nh * S * S * d
    report = _report_peak(peak, '' if dtype == torch.float32 else '[bf16] ')
    report('attn_fwd', timeit(lambda: C().attn_fwd(qkv, mb, nh, keep, SEED, 0, None)), flops=f_fwd)
    report('attn_fwd (no dropout)', timeit(lambda: C().attn_fwd(qkv, mb, nh, 1.0, SEED, 0, None)), flops=f_fwd)
    report('attn_bwd', timeit(lambda: C().attn_bwd(dout, qkv, mb, out, lse, dm, nh, keep, None, None, None, None)[0]), flops=2.5 * f_fwd)
    out1, lse1, dm1 = C().attn_fwd(qkv, mb, nh, 1.0, SEED, 0, None)
    report('attn_bwd (no dropout)', timeit(lambda: C().attn_bwd(dout, qkv, mb, out1, lse1, dm1, nh, 1.0, None, None, None, None)[0]),
           flops=2.5 * f_fwd)
    if dtype == torch.float32:   # fp32 on the fp16 matrix cores (fp16x3 pieces, attention_f16.hip)
        report('attn_fwd_f16', timeit(lambda: C().attn_fwd_f16(qkv, mb, nh, keep, SEED, 0, None)), flops=f_fwd)
        report('attn_fwd_f16 (no dropout)', timeit(lambda: C().attn_fwd_f16(qkv, mb, nh, 1.0, SEED, 0, None)),
               flops=f_fwd)
        # with the GEMM scale producers on (row max per (row, head), column max per query block)
        H = qkv.shape[-1] // 3
        am = torch.empty(B * S, nh, device=qkv.device)
        cm = torch.empty(B * ((S + 127) // 128), H, device=qkv.device)
        report('attn_fwd_f16 (+ row / col max)', timeit(lambda: C().attn_fwd_f16(qkv, mb, nh, keep, SEED, 0, None,
                                                                                   am, cm)), flops=f_fwd)
        bias = 0.1 * torch.randn(3 * H, device=qkv.device)
        report('attn_fwd_f16 (+ max, + QKV bias: the step)', timeit(lambda: C().attn_fwd_f16(
            qkv, mb, nh, keep, SEED, 0, bias, am, cm)), flops=f_fwd)
        slots = [torch.empty(H, device=qkv.device) for _ in range(3)]
        report('attn_bwd_f16 (+ QKV bias grad)', timeit(lambda: C().attn_bwd_f16(
            dout, qkv, mb, out, lse, dm, nh, keep, bias, *slots)[0]), flops=2.5 * f_fwd)
        if S <= 128:
            bam = torch.empty(B * S, nh, device=qkv.device)
            bcm = torch.empty(B, 3 * H, device=qkv.device)
            report('attn_bwd_f16 (+ bias grad, + max: the step)', timeit(lambda: C().attn_bwd_f16(
                dout, qkv, mb, out, lse, dm, nh, keep, bias, *slots, bam, bcm)[0]), flops=2.5 * f_fwd)
        report('attn_bwd_f16', timeit(lambda: C().attn_bwd_f16(dout, qkv, mb, out, lse, dm, nh, keep, None, None, None,
                                                                None)[0]), flops=2.5 * f_fwd)


def bench_ln(B, S, H=768):
    n = B * S
    x = torch.randn(n, H, device='cuda')
    res = torch.randn(n, H, device='cuda')
    g = torch.ones(H, device='cuda')
    bt = torch.zeros(H, device='cuda')
    bias = torch.zeros(H, device='cuda')
    report('ln_fwd(bias+drop+res)', timeit(lambda: C().ln_fwd(x, bias, res, g, bt, 1e-12, 0.9, SEED, 0, False, True)),
           bytes_=4 * n * H * 4)
    out, z, mean, rstd = C().ln_fwd(x, bias, res, g, bt, 1e-12, 0.9, SEED, 0, False, True)[:4]
    dout = torch.randn_like(out)
    report('ln_bwd(+dy,+dbias)', timeit(lambda: C().ln_bwd(dout, z, mean, rstd, g, 0.9, SEED, 0, False, True, True,
                                                           None, None, None)), bytes_=4 * n * H * 4)


def bench_ffn_act(B, S, F=3072):
    n = B * S
    y = torch.randn(n, F, device='cuda')
    b = torch.zeros(F, device='cuda')
    report('bias_gelu_fwd', timeit(lambda: C().bias_act_fwd(y, b, 0)), bytes_=2 * n * F * 4)
    dout = torch.randn_like(y)
    report('bias_gelu_bwd(+dbias)', timeit(lambda: C().bias_act_bwd(dout, y, b, None, 0, True, None)),
           bytes_=3 * n * F * 4)
    qkv = torch.randn(n, 2304, device='cuda')
    report('colsum(dqkv bias grad)', timeit(lambda: C().colsum(qkv, None, None)), bytes_=n * 2304 * 4)


def bench_adam(n=110_000_000):
    p = torch.randn(n, device='cuda')
    g = torch.randn(n, device='cuda')
    m = torch.zeros(n, device='cuda')
    v = torch.zeros(n, device='cuda')
    gs = torch.ones(1, device='cuda')
    report('adam(110M params)', timeit(lambda: C().adam(p, g, m, v, None, gs, 0, n, 0.9, 0.999, 1e-8, 1e-4, 1e-6, None)),
           bytes_=7 * n * 4)


def bench_xent(rows=2560, V=30522):
    """MLM decoder bias + softmax-xent + gradient, in place (rows = 128 x 20 masked positions)."""
    src = torch.randn(rows, V, device='cuda') * 3
    z = src.clone()
    bias = torch.randn(V, device='cuda') * 0.1
    lab = torch.randint(0, V, (rows,), device='cuda')
    copy = timeit(lambda: z.copy_(src))
    both = timeit(lambda: (z.copy_(src), C().softmax_xent_(z, bias, lab, -1)))
    report('softmax_xent({}x{})'.format(rows, V), both - copy, bytes_=2 * rows * V * 4)


def main():
    global SEED
    SEED = torch.ones(1, dtype=torch.int64, device='cuda')
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--seq', type=int, default=128)
    ap.add_argument('--only', default='attn,ln,ffn,adam,xent')
    a = ap.parse_args()
    torch.manual_seed(0)
    which = a.only.split(',')
    if 'attn' in which:
        bench_attn(a.batch, a.seq)
    if 'attn_bf16' in which:
        bench_attn(a.batch, a.seq, dtype=torch.bfloat16)
    if 'ln' in which:
        bench_ln(a.batch, a.seq)
    if 'ffn' in which:
        bench_ffn_act(a.batch, a.seq)
    if 'adam' in which:
        bench_adam()
    if 'xent' in which:
        bench_xent(a.batch * 20)


if __name__ == '__main__':
    main()
