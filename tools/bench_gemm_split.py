"""Forward / data-gradient GEMMs of --fp32-gemm bf16x3/x6: hand-written piece GEMM
(csrc/kernels/gemm_split.hip) vs the library on pass-stacked planes, BERT-base shapes,
checked against fp64.   python tools/bench_gemm_split.py [--tokens 16384]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tokens', type=int, default=16384)
    a = ap.parse_args()
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    T = a.tokens
    g = torch.Generator(device='cpu').manual_seed(0)
    for passes in (3, 6):
        ops.set_fp32_gemm('bf16x{}'.format(passes))
        # (name, n_in, n_out): forward y[T, n_out] = x W^T; dgrad dx[T, n_in] = dy W
        for name, n_in, n_out in (('qkv', 768, 2304), ('ao', 768, 768), ('up', 768, 3072), ('down', 3072, 768)):
            x = torch.randn(T, n_in, generator=g).cuda()
            W = (torch.randn(n_out, n_in, generator=g) * 0.05).cuda()
            dy = torch.randn(T, n_out, generator=g).cuda()
            xs, dys = sg.pieces(x), sg.pieces(dy)
            wf, wt = sg.weight_pieces(W)
            fl = 2.0 * T * n_in * n_out * passes
            t_f = timeit(lambda: sg.gemm(xs, wf))
            t_d = timeit(lambda: sg.gemm(dys, wt))
            xp, _ = sg.forward(x, W)
            t_lf = timeit(lambda: sg.forward(x, W))
            y = sg.gemm(xs, wf)
            ref = x.double() @ W.double().t()
            e_f = ((y.double() - ref).abs() / (x.double().abs() @ W.double().abs().t())).max().item()
            dx = sg.gemm(dys, wt)
            ref = dy.double() @ W.double()
            e_d = ((dx.double() - ref).abs() / (dy.double().abs() @ W.double().abs())).max().item()
            print('x{} {:5s} fwd {:7.1f} us ({:6.0f} TF/s bf16) dgrad {:7.1f} us ({:6.0f}) | lib stacked fwd incl. '
                  'split {:7.1f} us | err fwd {:.2e} dgrad {:.2e}'.format(
                      passes, name, t_f, fl / t_f / 1e6, t_d, fl / t_d / 1e6, t_lf, e_f, e_d), flush=True)
            del x, W, dy, xs, dys, wf, wt, xp
            torch.cuda.empty_cache()
    ops.set_fp32_gemm('native')


if __name__ == '__main__':
    main()
