"""Feasibility / accuracy probe for fp32 GEMMs emulated on bf16 matrix cores.

An fp32 operand x is split into bf16 planes (x = x0 + x1 [+ x2] + tiny); the
product A.B is a sum of plane products, each exact in the MFMA's fp32
accumulator.  Stacking the planes along the reduction dimension turns the sum
into ONE bf16 GEMM with K' = passes x K (see ops/split_gemm.py).

    python tools/bench_split_gemm.py            # BERT-base phase-1 shapes, T = 16384
"""
import argparse
import json
import time

import torch


def split_planes(x, n):
    planes, r = [], x
    for _ in range(n):
        p = r.to(torch.bfloat16)
        planes.append(p)
        r = r - p.float()
    return planes


PAIRS = {3: [(0, 0), (1, 0), (0, 1)],
         6: [(0, 0), (1, 0), (0, 1), (2, 0), (1, 1), (0, 2)]}


def emulated_nt(a, b, passes):
    """a [M,K] fp32, b [N,K] fp32 -> a @ b.T via one bf16 GEMM with K' = passes*K."""
    nsplit = 2 if passes == 3 else 3
    pa, pb = split_planes(a, nsplit), split_planes(b, nsplit)
    A = torch.cat([pa[i] for i, _ in PAIRS[passes]], dim=1)
    B = torch.cat([pb[j] for _, j in PAIRS[passes]], dim=1)
    return torch.mm(A, B.t(), out_dtype=torch.float32), (A, B)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tokens', type=int, default=16384)
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    dev = torch.device('cuda')
    T = args.tokens
    # (name, M, N, K, layout) with C[M,N] = A[M,K] B^T / A B / A^T B
    shapes = [
        ('qkv_fwd', T, 2304, 768), ('ao_fwd', T, 768, 768), ('up_fwd', T, 3072, 768), ('down_fwd', T, 768, 3072),
        ('qkv_dgrad', T, 768, 2304), ('up_dgrad', T, 768, 3072), ('down_dgrad', T, 3072, 768),
        ('qkv_wgrad', 2304, 768, T), ('ao_wgrad', 768, 768, T), ('up_wgrad', 3072, 768, T), ('down_wgrad', 768, 3072, T),
    ]
    g = torch.Generator(device='cpu').manual_seed(0)
    rows = []
    for name, M, N, K in shapes:
        a = torch.randn(M, K, generator=g).to(dev)
        b = torch.randn(N, K, generator=g).to(dev)
        flop = 2.0 * M * N * K
        t32 = timeit(lambda: torch.mm(a, b.t()))
        ref = (a.double() @ b.double().t())
        scale = (a.abs().double() @ b.abs().double().t())
        e32 = ((torch.mm(a, b.t()).double() - ref).abs() / scale).max().item()
        row = {'shape': name, 'M': M, 'N': N, 'K': K, 'fp32_us': t32 * 1e6, 'fp32_tflops': flop / t32 / 1e12,
               'fp32_err': e32}
        for passes in (3, 6):
            c, (A, B) = emulated_nt(a, b, passes)
            err = ((c.double() - ref).abs() / scale).max().item()
            tg = timeit(lambda: torch.mm(A, B.t(), out_dtype=torch.float32))
            row['x%d_us' % passes] = tg * 1e6
            row['x%d_eff_tflops' % passes] = flop / tg / 1e12
            row['x%d_bf16_tflops' % passes] = passes * flop / tg / 1e12
            row['x%d_err' % passes] = err
            # NN form (B' stacked along K rows) and TN form (A' stacked along rows) for dgrad/wgrad
            Bn = B.t().contiguous()
            row['x%d_nn_us' % passes] = timeit(lambda: torch.mm(A, Bn, out_dtype=torch.float32)) * 1e6
            At = A.t().contiguous()
            row['x%d_tn_us' % passes] = timeit(lambda: torch.mm(At.t(), Bn, out_dtype=torch.float32)) * 1e6
        rows.append(row)
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) and v > 1e-3 else v) for k, v in row.items()}),
              flush=True)
        del a, b, A, B, Bn, At, c, ref, scale
        torch.cuda.empty_cache()
    tot = {k: sum(r[k] for r in rows) for k in ('fp32_us', 'x3_us', 'x6_us')}
    print(json.dumps({'per_layer_total_us': tot}))
    if args.out:
        with open(args.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
