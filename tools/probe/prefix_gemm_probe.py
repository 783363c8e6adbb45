"""Probe: x6 forward GEMM as ONE product over 6 stacked activation planes vs THREE products
over prefixes of 3 distinct planes ([x0 x1 x2] . [w0 w0 w0], [x0 x1] . [w1 w1],
[x0] . [w2], accumulated with beta = 1).  The prefix form lets the producer write 3 planes
instead of 6 (half the plane bytes) at the cost of two extra passes over the fp32 output.

``python tools/probe/prefix_gemm_probe.py`` (one MI355X)."""
import time

import torch


def timeit(fn, iters=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    dev = 'cuda'
    for (T, K, N) in [(16384, 3072, 768), (16384, 768, 768), (16384, 768, 3072), (16384, 768, 2304)]:
        x = [torch.randn(T, K, device=dev).to(torch.bfloat16) for _ in range(3)]
        w = [torch.randn(N, K, device=dev).to(torch.bfloat16) for _ in range(3)]
        A6 = torch.cat([x[0], x[1], x[0], x[2], x[1], x[0]], 1)
        W6 = torch.cat([w[0], w[0], w[1], w[0], w[1], w[2]], 1)
        A3 = torch.cat([x[0], x[1], x[2]], 1)
        B1 = torch.cat([w[0], w[0], w[0]], 1)
        B2 = torch.cat([w[1], w[1]], 1)
        B3 = w[2].contiguous()
        C = torch.empty(T, N, device=dev)

        def one():
            return torch.mm(A6, W6.t(), out_dtype=torch.float32)

        def three():
            torch.mm(A3, B1.t(), out_dtype=torch.float32, out=C)
            torch.addmm(C, A3[:, :2 * K], B2.t(), out_dtype=torch.float32, out=C)
            torch.addmm(C, A3[:, :K], B3.t(), out_dtype=torch.float32, out=C)
            return C

        ref = one()
        got = three().clone()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        t1, t3 = timeit(one), timeit(three)
        plane_bytes = 3 * T * K * 2   # planes the producer no longer writes (and the GEMM no longer reads)
        print(f'T={T} K={K} N={N}: one GEMM (6 planes) {t1:7.1f} us | three prefix GEMMs {t3:7.1f} us '
              f'| saved plane bytes {plane_bytes / 1e6:.0f} MB (~{plane_bytes / 5.5e12 * 1e6:.0f} us at 5.5 TB/s) '
              f'| rel diff {err:.1e}', flush=True)


if __name__ == '__main__':
    main()
