"""Piece layout probe for the LDS-DMA piece GEMM (gemm_split.hip), bf16x6, BERT-base forward
shapes at T = 16384: natural pieces [rows][3][K] vs the B16 layout [rows][K/16][3][16] for the
B operand only (weights: written by split_weight, read by nothing else) or for both operands."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_gemm_split import timeit, relerr  # noqa: E402


def blocked(p, npc=3, kb=16):
    R = p.shape[0]
    K = p.shape[1] // npc
    return p.view(R, npc, K // kb, kb).permute(0, 2, 1, 3).contiguous().view(R, -1)


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
        wf, _ = C().split_weight(W, 3)
        wb, _ = C().split_weight(W, 3, True)
        assert torch.equal(wb, blocked(wf))
        xb = blocked(xs)
        ref = x.double() @ W.double().t()
        sc = x.double().abs() @ W.double().abs().t()
        fl = 2.0 * T * n_in * n_out * 6
        for cfg in [int(c) for c in os.environ.get('CFGS', '0,1,2,7').split(',')]:
            if n_out % {0: 192, 1: 256, 2: 128, 7: 128}[cfg]:
                continue
            os.environ['HX_GEMM_CFG'] = str(cfg)
            line = '{:5s} cfg {}'.format(name, cfg)
            for lay, a_, b_ in ((0, xs, wf), (2, xs, wb), (3, xb, wb)):
                if lay and cfg == 2:
                    continue
                t = timeit(lambda: C().gemm_split(a_, b_, 6, None, False, lay))
                e = relerr(C().gemm_split(a_, b_, 6, None, False, lay), ref, sc)
                line += ' | lay{} {:6.1f} us {:5.0f} TF/s {:.1e}'.format(lay, t, fl / t / 1e6, e)
            print(line, flush=True)
        os.environ.pop('HX_GEMM_CFG', None)


if __name__ == '__main__':
    main()
