"""Weight-gradient GEMM variants at BERT shapes (bf16 activations, fp32 gradient slots).

``python tools/bench_wgrad.py [--tokens 16384]`` -- dW[out, in] = dY^T X with
dY [T, out], X [T, in] bf16, T = tokens per GPU.  Compares the library paths
(bf16 x bf16 -> fp32 output, bf16 output + cast, the transposed product) and
the hand-written split-K MFMA kernel (``_C.wgrad_bf16``) when present.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tokens', type=int, default=16384)
    ap.add_argument('--sweep', action='store_true',
                    help='time every (tile config, token split) of the hand-written kernel via HX_WGRAD_CFG')
    a = ap.parse_args()
    if a.sweep:
        return sweep(a.tokens)
    T = a.tokens
    try:
        from hetseq_9cme_amd.ops._ext import C
        ext = C() if hasattr(C(), 'wgrad_bf16') else None
    except Exception:  # noqa: BLE001
        ext = None
    for (n_out, n_in) in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
        dy = torch.randn(T, n_out, device='cuda').to(torch.bfloat16)
        x = torch.randn(T, n_in, device='cuda').to(torch.bfloat16)
        slot = torch.empty(n_out, n_in, device='cuda')
        fl = 2.0 * T * n_out * n_in
        res = {}
        res['mm out_dtype=f32'] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=slot))
        res['mm bf16 + cast'] = timeit(lambda: slot.copy_(torch.mm(dy.t(), x)))
        res['mm (x^T dy)^T f32'] = timeit(lambda: torch.mm(x.t(), dy, out_dtype=torch.float32))
        for sk in (4, 8, 16):   # library split-K as a batched GEMM over token chunks + a sum
            dyb = dy.view(sk, T // sk, n_out).transpose(1, 2)
            xb = x.view(sk, T // sk, n_in)
            res['bmm split{} bf16->f32+sum'.format(sk)] = timeit(
                lambda: torch.sum(torch.bmm(dyb, xb, out_dtype=torch.float32), 0, out=slot))
            res['bmm split{} bf16+sum'.format(sk)] = timeit(
                lambda: torch.sum(torch.bmm(dyb, xb), 0, dtype=torch.float32, out=slot))
        if ext is not None:
            res['hx wgrad_bf16'] = timeit(lambda: ext.wgrad_bf16(dy, x, slot))
            ref = torch.mm(dy.t().float(), x.float())
            got = slot.clone()
            ext.wgrad_bf16(dy, x, got)
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            res['hx wgrad_bf16'] = (res['hx wgrad_bf16'], err)
        for k, v in res.items():
            us, err = (v if isinstance(v, tuple) else (v, None))
            print('[{}x{} T={}] {:<22s} {:8.1f} us  {:7.1f} TF/s{}'.format(
                n_out, n_in, T, k, us, fl / us / 1e6, '' if err is None else '  rel.err {:.2e}'.format(err)),
                flush=True)


def sweep(T):
    from hetseq_9cme_amd.ops._ext import C
    tiles = {0: (128, 128), 1: (256, 128), 2: (256, 128), 3: (128, 128)}
    if os.environ.get("HX_SWEEP_CFGS"):
        tiles = {int(c): tiles[int(c)] for c in os.environ["HX_SWEEP_CFGS"].split(",")}
    for (n_out, n_in) in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
        dy = torch.randn(T, n_out, device='cuda').to(torch.bfloat16)
        x = torch.randn(T, n_in, device='cuda').to(torch.bfloat16)
        slot = torch.empty(n_out, n_in, device='cuda')
        ref = torch.mm(dy.t().float(), x.float())
        fl = 2.0 * T * n_out * n_in
        os.environ.pop('HX_WGRAD_CFG', None)
        base = timeit(lambda: C().wgrad_bf16(dy, x, slot))
        best = (base, 'plan')
        for cfg, (bm, bn) in tiles.items():
            if n_out % bm or n_in % bn:
                continue
            for ns in (1, 2, 3, 4, 6, 8, 12, 16):
                os.environ['HX_WGRAD_CFG'] = '{}:{}'.format(cfg, ns)
                us = timeit(lambda: C().wgrad_bf16(dy, x, slot))
                err = ((slot - ref).abs().max() / ref.abs().max()).item()
                assert err < 1e-3, (cfg, ns, err)
                if us < best[0]:
                    best = (us, '{}:{}'.format(cfg, ns))
                print('[{}x{} T={}] cfg {} nsplit {:2d} {:8.1f} us {:7.1f} TF/s'.format(
                    n_out, n_in, T, cfg, ns, us, fl / us / 1e6), flush=True)
        os.environ.pop('HX_WGRAD_CFG', None)
        print('[{}x{} T={}] plan {:.1f} us; best {} {:.1f} us ({:.1f} TF/s)'.format(
            n_out, n_in, T, base, best[1], best[0], fl / best[0] / 1e6), flush=True)




if __name__ == '__main__':
    main()
