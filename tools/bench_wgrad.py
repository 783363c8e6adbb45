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
    ap.add_argument('--split', type=int, default=0, help='time the split-piece kernel (3 or 6 passes) vs stacked')
    ap.add_argument('--variants', action='store_true',
                    help='with --split: time the pipeline variants (HX_WGRAD_SPLIT_VAR) at the planned split')
    ap.add_argument('--sweep', action='store_true',
                    help='time every (tile config, token split) of the hand-written kernel via HX_WGRAD_CFG')
    a = ap.parse_args()
    if a.split and a.variants:
        return split_variants(a.tokens, a.split)
    if a.split:
        return split_bench(a.tokens, a.split)
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


def split_bench(T, passes):
    """--fp32-gemm bf16x3/x6 weight gradients: split-piece kernel (all token splits) vs the
    stacked-rows kernel, checked against an fp64 product of the fp32 operands."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x{}'.format(passes))
    for (n_out, n_in) in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
        dy = torch.randn(T, n_out, device='cuda')
        x = torch.randn(T, n_in, device='cuda')
        dys, xs = sg.grad_planes(dy), sg.planes(x, sg.ORDER_P[passes])
        slot = torch.empty(n_out, n_in, device='cuda')
        ref = dy.double().t() @ x.double()
        scale = dy.double().abs().t() @ x.double().abs()
        fl = 2.0 * T * n_out * n_in * passes
        stacked = timeit(lambda: C().wgrad_bf16(dys.view(-1, n_out), xs.view(-1, n_in), slot))
        print('[{}x{} T={} x{}] stacked {:8.1f} us {:7.1f} TF/s'.format(n_out, n_in, T, passes, stacked,
                                                                       fl / stacked / 1e6), flush=True)
        po, px = sg._piece_offsets(sg.ORDER_Q[passes], n_out), sg._piece_offsets(sg.ORDER_P[passes], n_in)
        cfgs = [int(c) for c in os.environ.get('HX_SWEEP_CFGS', '0,1,2').split(',')]
        runs = [(None, 0)] + [(cfg, ns) for cfg in cfgs for ns in (1, 2, 3, 4, 6, 7, 8, 9, 12, 14, 16)
                              if not (n_out % (256 if cfg else 128) or (cfg >= 2 and passes != 6)
                                      or (cfg == 2 and n_in % 256))]
        for cfg, ns in runs:
            if ns:
                os.environ['HX_WGRAD_SPLIT_CFG'] = '{}:{}'.format(cfg, ns)
            else:
                os.environ.pop('HX_WGRAD_SPLIT_CFG', None)
            us = timeit(lambda: C().wgrad_split(dys, po, xs, px, passes, n_out, n_in, slot))
            err = ((slot.double() - ref).abs() / scale).max().item()
            print('[{}x{} T={} x{}] split cfg {} nsplit {} {:8.1f} us {:7.1f} TF/s err {:.2e}'.format(
                n_out, n_in, T, passes, 'plan' if cfg is None else cfg, ns or 'plan', us, fl / us / 1e6, err),
                flush=True)
        os.environ.pop('HX_WGRAD_SPLIT_CFG', None)


def split_variants(T, passes, rounds=3):
    """Pipeline variants of the split-piece kernel (register stages ahead x work order),
    interleaved over several rounds in one process (median per round, min over rounds)."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x{}'.format(passes))
    variants = ['2,0', '2,1', '1,0', '1,1', '0,0', '0,1']
    for (n_out, n_in) in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
        dy = torch.randn(T, n_out, device='cuda')
        x = torch.randn(T, n_in, device='cuda')
        dys, xs = sg.grad_planes(dy), sg.planes(x, sg.ORDER_P[passes])
        slot = torch.empty(n_out, n_in, device='cuda')
        ref = dy.double().t() @ x.double()
        scale = dy.double().abs().t() @ x.double().abs()
        fl = 2.0 * T * n_out * n_in * passes
        po, px = sg._piece_offsets(sg.ORDER_Q[passes], n_out), sg._piece_offsets(sg.ORDER_P[passes], n_in)
        best = {v: float('inf') for v in variants}
        for _ in range(rounds):
            for v in variants:
                os.environ['HX_WGRAD_SPLIT_VAR'] = v
                best[v] = min(best[v], timeit(lambda: C().wgrad_split(dys, po, xs, px, passes, n_out, n_in, slot)))
                err = ((slot.double() - ref).abs() / scale).max().item()
                assert err < 1e-5, (v, err)
        os.environ.pop('HX_WGRAD_SPLIT_VAR', None)
        print('[{}x{} T={} x{}] '.format(n_out, n_in, T, passes) + '  '.join(
            'var {} {:7.1f} us {:6.0f} TF/s'.format(v, best[v], fl / best[v] / 1e6) for v in variants), flush=True)


if __name__ == '__main__':
    main()
