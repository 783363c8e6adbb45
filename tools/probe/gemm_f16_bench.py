"""Standalone speed of the fp16x3 and bf16 GEMM kernels (csrc/kernels/gemm_f16.hip) at the
BERT-base phase-1 shapes (T = 16384 token rows), against hipBLASLt bf16 (torch.mm) on the same
shapes: median of 20 event-timed calls each.  ``eff`` = fp16 MFMA rate achieved counting all three
passes (the dense f16 peak is ~2.5 PF/s); ``fp32eq`` = the fp32 product rate it delivers."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, n=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[n // 2] * 1e3


def sweep(C, dev, cfgs):
    """fwd / dgrad (fp16x3 and bf16) of every shape under each forced tile configuration."""
    T = int(os.environ.get('T', '16384'))
    g = torch.Generator(device=dev).manual_seed(0)
    for (name, N, K) in [('qkv', 2304, 768), ('attn_out', 768, 768), ('ffn_up', 3072, 768), ('ffn_down', 768, 3072)]:
        x = torch.randn(T, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.03
        b = torch.randn(N, device=dev, generator=g)
        xp = C().amax_rows(x)
        wf, wt, wp, wc = C().split_weight_f16([W])[0]
        dy = torch.randn(T, N, device=dev, generator=g)
        dp = C().amax_rows(dy)
        acc = torch.randn(T, K, device=dev, generator=g)
        d = torch.randn(T, K, device=dev, generator=g)
        db = torch.zeros(K, device=dev)
        xb, Wb = x.bfloat16(), W.bfloat16()
        fl = 2.0 * T * N * K
        for c in cfgs:
            # 'cfg' or 'cfg:ks' (ks: split-K slabs of the plain / beta GEMMs; default = the plan)
            cfg, _, ks = c.partition(':')
            ks = int(ks) if ks else 0
            if cfg == 'plan':
                os.environ.pop('HX_GEMM_F16_CFG', None)
            else:
                os.environ['HX_GEMM_F16_CFG'] = cfg
            try:
                if name == 'ffn_up':
                    f = timed(lambda: C().gemm_f16_gelu(x, xp, wf, wp, b, 1))
                else:
                    f = timed(lambda: C().gemm_f16(x, xp, wf, wp, bias=b, ks=ks))
                if name == 'ffn_down':
                    dg = timed(lambda: C().gemm_f16_dgelu(dy, dp, wt, wc, d, None, db, 1))
                else:
                    dg = timed(lambda: C().gemm_f16(dy, dp, wt, wc, out=acc, beta=True, ks=ks))
                bf = timed(lambda: C().gemm_bf16(xb, Wb, bias=b))
            except RuntimeError as e:
                print('{:10s} cfg {}: {}'.format(name, c, str(e).splitlines()[0]), flush=True)
                continue
            print('{:10s} cfg {:4s} fwd {:7.1f} us ({:4.2f} PF/s)  dgrad {:7.1f} us ({:4.2f})  bf16 fwd {:6.1f} us '
                  '({:4.2f})'.format(name, c, f, 3 * fl / f / 1e9, dg, 3 * fl / dg / 1e9, bf, fl / bf / 1e9), flush=True)
    os.environ.pop('HX_GEMM_F16_CFG', None)


def wgrad_sweep(C, dev, plans):
    """weight gradients of every shape under forced (tile config : token splits) plans
    (HX_WGRAD_F16, 'plan' = the kernel's own)."""
    T = int(os.environ.get('T', '16384'))
    g = torch.Generator(device=dev).manual_seed(0)
    only = os.environ.get('ONLY')   # one shape name
    for (name, N, K) in [('qkv', 2304, 768), ('attn_out', 768, 768), ('ffn_up', 3072, 768), ('ffn_down', 768, 3072)]:
        if only and name != only:
            continue
        x = torch.randn(T, K, device=dev, generator=g)
        dy = torch.randn(T, N, device=dev, generator=g)
        out = torch.empty(N, K, device=dev)
        dc, xc = C().amax_cols(dy), C().amax_cols(x)
        fl = 2.0 * T * N * K
        for c in plans:
            if c == 'plan':
                os.environ.pop('HX_WGRAD_F16', None)
            else:
                os.environ['HX_WGRAD_F16'] = c
            us = timed(lambda: C().wgrad_f16(dy, dc, x, xc, out))
            print('{:10s} wgrad {:6s} {:7.1f} us ({:4.2f} PF/s)'.format(name, c, us, 3 * fl / us / 1e9), flush=True)
    os.environ.pop('HX_WGRAD_F16', None)


def pieces_ab(C, dev, reps):
    """A read as fp32 and split in the k loop vs A pre-split into P2 pieces (split_rows_f16), on the
    four products whose A operand a LayerNorm produces; alternated `reps` times on one box, and the
    outputs compared bit for bit (the split is the same rounding either way)."""
    T = int(os.environ.get('T', '16384'))
    g = torch.Generator(device=dev).manual_seed(0)
    for (name, N, K) in [('qkv fwd', 2304, 768), ('ffn_up fwd', 3072, 768), ('ffn_down dgrad', 3072, 768),
                         ('attn_out dgrad', 768, 768)]:
        x = torch.randn(T, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.03
        b = torch.randn(N, device=dev, generator=g)
        xp = C().amax_rows(x)
        xs = C().split_rows_f16(x, xp)
        wf, wt, wp, wc = C().split_weight_f16([W])[0]
        if name == 'ffn_up fwd':
            def run(a):
                return C().gemm_f16_gelu(a, xp, wf, wp, b, 1)
        elif name == 'ffn_down dgrad':
            u = torch.randn(T, N, device=dev, generator=g)
            db = torch.zeros(N, device=dev)

            def run(a):
                return C().gemm_f16_dgelu(a, xp, wf, wp, u, None, db, 1)
        elif name == 'attn_out dgrad':
            acc = torch.randn(T, N, device=dev, generator=g)

            def run(a):
                return [C().gemm_f16(a, xp, wf, wp, out=acc.clone(), beta=True)]
        else:
            def run(a):
                return [C().gemm_f16(a, xp, wf, wp, bias=b)]
        r0, r1 = run(x), run(xs)
        same = all(torch.equal(p, q) for p, q in zip(r0, r1) if p.dtype == torch.float32)
        t0, t1 = [], []
        for _ in range(reps):
            t0.append(timed(lambda: run(x)))
            t1.append(timed(lambda: run(xs)))
        t0.sort()
        t1.sort()
        print('{:16s} fp32 A {:7.1f} us  pieces A {:7.1f} us  ({:+.1f} %)  bitwise equal: {}  [{}] [{}]'.format(
            name, t0[reps // 2], t1[reps // 2], 100 * (t1[reps // 2] / t0[reps // 2] - 1), same,
            ' '.join('%.0f' % v for v in t0), ' '.join('%.0f' % v for v in t1)), flush=True)
        x16 = C().split_rows_f16(x, xp)
        us = timed(lambda: C().split_rows_f16(x, xp))
        print('{:16s} split_rows_f16 (standalone) {:6.1f} us'.format(name, us), flush=True)
        del x16


def main():
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda', 0)
    if os.environ.get('PIECES_AB'):
        return pieces_ab(C, dev, int(os.environ['PIECES_AB']))
    if os.environ.get('WGRAD_PLANS'):
        return wgrad_sweep(C, dev, os.environ['WGRAD_PLANS'].split(','))
    if os.environ.get('CFGS'):
        return sweep(C, dev, os.environ['CFGS'].split(','))
    T = int(os.environ.get('T', '16384'))
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*s):
        return torch.randn(*s, device=dev, generator=g)
    rows = []
    only = os.environ.get('ONLY')   # one shape name (PMC passes)
    for (name, N, K) in [('qkv', 2304, 768), ('attn_out', 768, 768), ('ffn_up', 3072, 768), ('ffn_down', 768, 3072)]:
        if only and name != only:
            continue
        x = rnd(T, K)
        W = rnd(N, K) * 0.03
        b = rnd(N)
        xp = C().amax_rows(x)
        wf, wt, wp, wc = C().split_weight_f16([W])[0]
        fl = 2.0 * T * N * K
        if name == 'ffn_up':
            us = timed(lambda: C().gemm_f16_gelu(x, xp, wf, wp, b, 1))
        else:
            us = timed(lambda: C().gemm_f16(x, xp, wf, wp, bias=b))
        rows.append(('fwd ' + name, T, N, K, us, fl))
        dy = rnd(T, N)
        dp = C().amax_rows(dy)
        acc = rnd(T, K)
        if name == 'ffn_down':
            d = rnd(T, K)
            db = torch.zeros(K, device=dev)
            us = timed(lambda: C().gemm_f16_dgelu(dy, dp, wt, wc, d, None, db, 1))
        else:
            us = timed(lambda: C().gemm_f16(dy, dp, wt, wc, out=acc, beta=True))
        rows.append(('dgrad ' + name, T, K, N, us, fl))
        out = torch.empty(N, K, device=dev)
        dc, xc = C().amax_cols(dy), C().amax_cols(x)
        us = timed(lambda: C().wgrad_f16(dy, dc, x, xc, out))
        rows.append(('wgrad ' + name, N, K, T, us, fl))
        xb, Wb, dyb = x.bfloat16(), W.bfloat16(), dy.bfloat16()
        us = timed(lambda: C().gemm_bf16(xb, Wb, bias=b))
        rows.append(('bf16 fwd ' + name, T, N, K, us, fl / 3))
        us = timed(lambda: torch.mm(xb, Wb.t()))
        rows.append(('blas bf16 fwd ' + name, T, N, K, us, fl / 3))
        us = timed(lambda: torch.mm(dyb.t(), xb))
        rows.append(('blas bf16 wgrad ' + name, N, K, T, us, fl / 3))
    tot = 0.0
    for (name, M, N, K, us, f16flops) in rows:
        # f16flops: three passes' worth for the fp16x3 kernels (fl), one pass for bf16 ones (fl / 3)
        passes = 3 if f16flops == 2.0 * M * N * K else 1
        eff = passes * 2.0 * M * N * K / (us * 1e-6) / 1e15
        print('{:24s} M{:6d} N{:5d} K{:6d} {:8.1f} us  eff {:5.2f} PF/s  fp32eq {:5.2f} PF/s'.format(
            name, M, N, K, us, eff, 2.0 * M * N * K / (us * 1e-6) / 1e15), flush=True)
        if not name.startswith(('bf16', 'blas')):
            tot += us
    print('fp16x3 total per layer (fwd + dgrad + wgrad): {:.1f} us'.format(tot))


if __name__ == '__main__':
    main()
