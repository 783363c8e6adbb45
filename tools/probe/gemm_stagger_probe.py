"""Piece GEMM pipelines A/B (gemm_split.hip, bf16x6, T = 16384 BERT-base forward shapes):
HX_GEMM_PIPE=3 (interleaved DMA) by default; PIPES=... adds other pipelines.  Records: 6 (3 on
16x16x32 MFMAs, profiles/r3_gemm_mfma16_probe.log) and 5 (3 with the SIMD partners staggered by
one pass, profiles/r3_gemm_stagger_probe.log) were measured slower and removed.  Both
piece layouts (lay2: weights B16; lay3: both operands B16), cfgs 0 and 1, interleaved rounds in
one process; every variant checked against fp64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_gemm_split import timeit, relerr  # noqa: E402
from tools.probe.gemm_layout_probe import blocked  # noqa: E402


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    T = 16384
    for name, n_in, n_out in (('qkv', 768, 2304), ('ao', 768, 768), ('up', 768, 3072), ('down', 3072, 768)):
        x = torch.rand(T, n_in, device='cuda') * 2 - 1
        W = (torch.rand(n_out, n_in, device='cuda') * 2 - 1) * 0.05
        xs = sg.pieces(x)
        wb, _ = C().split_weight(W, 3, True)
        xb = blocked(xs)
        ref = x.double() @ W.double().t()
        sc = x.double().abs() @ W.double().abs().t()
        fl = 2.0 * T * n_in * n_out * 6
        for cfg in (0, 1):
            if n_out % {0: 192, 1: 256}[cfg]:
                continue
            os.environ['HX_GEMM_CFG'] = str(cfg)
            res = {}
            for rnd in range(3):
                for lay, a_ in ((2, xs), (3, xb)):
                    for pipe in os.environ.get('PIPES', '3').split(','):
                        os.environ['HX_GEMM_PIPE'] = pipe
                        t = timeit(lambda: C().gemm_split(a_, wb, 6, None, False, lay))
                        k = (lay, pipe)
                        res[k] = min(res.get(k, 1e9), t)
                        if rnd == 0:
                            e = relerr(C().gemm_split(a_, wb, 6, None, False, lay), ref, sc)
                            assert e < 1e-6, (name, cfg, lay, pipe, e)
            line = '{:5s} cfg {}'.format(name, cfg)
            for (lay, pipe), t in sorted(res.items()):
                line += ' | lay{} pipe{} {:6.1f} us {:5.0f} TF/s'.format(lay, pipe, t, fl / t / 1e6)
            print(line, flush=True)
        os.environ.pop('HX_GEMM_CFG', None)
        os.environ.pop('HX_GEMM_PIPE', None)


if __name__ == '__main__':
    main()
