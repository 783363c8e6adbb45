"""Can the split-piece weight-gradient kernel (wgrad_split.hip: reduction over the ROW index of
both operands, each distinct bf16 piece staged once) run the forward / data-gradient products
too?  Y[T][N] = X[T][K] W[N][K]^T is out[M=T][N] = sum_k X^T[k][T] . W^T[k][N], i.e. the kernel
over transposed pieces (reduction K = 768 / 3072).  Times it at the BERT-base shapes against
torch.mm over the pass-stacked planes (what the step runs).  ``python tools/probe/wgrad_as_fwd_probe.py``"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    T = 16384
    for name, N, K in [('qkv fwd', 2304, 768), ('ao fwd', 768, 768), ('up fwd', 3072, 768), ('down fwd', 768, 3072)]:
        x = torch.randn(T, K, device='cuda')
        w = torch.randn(N, K, device='cuda')
        fl = 2.0 * T * N * K * 6
        xs = sg.planes(x, sg.ORDER_P[6])
        wq = sg.planes(w, sg.ORDER_Q[6])
        t_lib = timeit(lambda: torch.mm(xs, wq.t(), out_dtype=torch.float32))
        # transposed distinct pieces: [K, 3 * T] and [K, 3 * N] (piece p at column p * T / p * N)
        xt = sg.planes(x.t().contiguous(), [0, 1, 2])
        wt = sg.planes(w.t().contiguous(), [0, 1, 2])
        out = torch.empty(T, N, device='cuda')
        po, pw = [0, T, 2 * T], [0, N, 2 * N]
        t_k = timeit(lambda: C().wgrad_split(xt, po, wt, pw, 6, T, N, out))
        ref = x.double() @ w.double().t()
        scale = x.double().abs() @ w.double().abs().t()
        err = ((out.double() - ref).abs() / scale).max().item()
        print('{:<9s} T{} N{} K{}: library over planes {:7.1f} us ({:5.0f} TF/s) | wgrad kernel on transposed pieces '
              '{:7.1f} us ({:5.0f} TF/s) err {:.1e}'.format(name, T, N, K, t_lib, fl / t_lib / 1e6, t_k, fl / t_k / 1e6,
                                                            err), flush=True)


if __name__ == '__main__':
    main()
