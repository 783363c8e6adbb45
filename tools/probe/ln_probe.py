"""LayerNorm forward / backward kernel times at BERT-base phase 1 (16384 x 768), fp32 and bf16,
with the arguments the training step passes (bias + dropout + residual; backward with dy, the bias
gradient and, fp32, the row / column maxima).  KEEP: the dropout keep probability (1 = none);
HX_EXT_SO: time an explicit build of the extension (ext_ab.py) instead of the in-tree one."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, n=30):
    for _ in range(5):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[n // 2] * 1e3


def main():
    if os.environ.get('HX_EXT_SO'):   # an explicit build (A/B of two builds, one process each)
        from ext_ab import load
        load(os.environ['HX_EXT_SO'])
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda', 0)
    n, H = 16384, 768
    seed = torch.full((1,), 5, dtype=torch.int64, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    tag = os.path.basename(os.environ.get('HX_EXT_SO', 'in-tree'))
    keep = float(os.environ.get('KEEP', '0.9'))
    tag += ' keep %g fwd cap %s bwd cap %s' % (keep, os.environ.get('HX_LN_FWD_CAP', '-'),
                                              os.environ.get('HX_LN_BWD_CAP', '-'))
    for dt in (torch.float32, torch.bfloat16):
        y = torch.randn(n, H, device=dev, generator=g).to(dt)
        res = torch.randn(n, H, device=dev, generator=g).to(dt)
        bias = torch.randn(H, device=dev, generator=g)
        gamma = torch.randn(H, device=dev, generator=g)
        beta = torch.randn(H, device=dev, generator=g)
        f32 = dt == torch.float32
        am = torch.empty(n, 1, device=dev) if f32 else None
        pc = torch.empty(n, 2 * H, dtype=torch.float16, device=dev) if f32 else None   # training's pieces
        out, z, mean, rstd = C().ln_fwd(y, bias, res, gamma, beta, 1e-12, keep, seed, 1, False, True, am, pc)
        tf = timed(lambda: C().ln_fwd(y, bias, res, gamma, beta, 1e-12, keep, seed, 1, False, True, am, pc))
        dout = torch.randn(n, H, device=dev, generator=g).to(dt)
        dg, db, dbb = (torch.zeros(H, device=dev) for _ in range(3))
        bm = torch.empty(n, 1, device=dev) if f32 else None
        cm = torch.empty(1, H, device=dev) if f32 else None
        tb = timed(lambda: C().ln_bwd(dout, z, mean, rstd, gamma, keep, seed, 1, False, True, True, dg, db, dbb,
                                      bm, cm))
        print('{} {:8s} ln_fwd {:6.1f} us  ln_bwd (+fold) {:6.1f} us'.format(tag, str(dt).split('.')[-1], tf, tb),
              flush=True)


if __name__ == '__main__':
    main()
