"""Piece layout probe for the LDS-DMA piece GEMM (gemm_split.hip): natural pieces
[rows][npc][K] vs k-blocked [rows][K/BK][npc][BK] (one BK-deep k step of a row contiguous
over all pieces), bf16x6, BERT-base forward shapes at T = 16384, every tile config."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_gemm_split import timeit, relerr  # noqa: E402


def blocked(p, npc, kb):
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
        wf, _ = sg.weight_pieces(W)
        ref = x.double() @ W.double().t()
        sc = x.double().abs() @ W.double().abs().t()
        fl = 2.0 * T * n_in * n_out * 6
        for cfg, kb in ((0, 16), (1, 16), (2, 32), (3, 16), (4, 16), (5, 16), (6, 16)):
            if n_out % {0: 192, 1: 256, 2: 128, 3: 192, 4: 128, 5: 256, 6: 128}[cfg]:
                continue
            os.environ['HX_GEMM_CFG'] = str(cfg)
            xb, wb = blocked(xs, 3, kb), blocked(wf, 3, kb)
            t_n = timeit(lambda: C().gemm_split(xs, wf, 6))
            t_b = timeit(lambda: C().gemm_split(xb, wb, 6, None, False, kb))
            e_b = relerr(C().gemm_split(xb, wb, 6, None, False, kb), ref, sc)
            print('{:5s} cfg {} natural {:7.1f} us {:5.0f} TF/s | blocked{} {:7.1f} us {:5.0f} TF/s err {:.2e}'.format(
                name, cfg, t_n, fl / t_n / 1e6, kb, t_b, fl / t_b / 1e6, e_b), flush=True)


if __name__ == '__main__':
    main()
