"""FFN epilogue GEMMs at BERT-base phase-1 size (T = 16384, bf16x6): FFN-up forward with the
bias + GELU epilogue (u or gelu'(u) stored) and the FFN-down data gradient with the dGELU
epilogue (from u or from gelu'(u)), on each tile configuration that takes N = 3072:
256 x 192 (cfg 0), 256 x 256 (cfg 1), 256 x 128 at two workgroups per CU (cfg 7) -- the last
overlaps one workgroup's epilogue with the other's main loop.  Interleaved rounds, one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_gemm_split import timeit  # noqa: E402


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    ops.set_fp32_gemm('bf16x6')
    T, H, I = 16384, 768, 3072
    x = torch.rand(T, H, device='cuda') * 2 - 1
    W1 = (torch.rand(I, H, device='cuda') * 2 - 1) * 0.05
    b1 = (torch.rand(I, device='cuda') * 2 - 1) * 0.1
    W2 = (torch.rand(H, I, device='cuda') * 2 - 1) * 0.05
    dy = torch.rand(T, H, device='cuda') * 2 - 1
    xs, dys = sg.pieces(x), sg.pieces(dy)
    w1f, _ = sg.weight_pieces(W1)
    _, w2t = sg.weight_pieces(W2)
    u, _ = sg.gemm_gelu(xs, w1f, b1)
    gd, _ = sg.gemm_gelu(xs, w1f, b1, deriv=True)
    hs = sg.pieces(torch.rand(T, I, device='cuda') * 2 - 1)
    w2f, _ = sg.weight_pieces(W2)
    fl = 2.0 * T * H * I * 6
    res = {}
    for rnd in range(3):
        for cfg in ('0', '1', '7'):
            os.environ['HX_GEMM_CFG'] = cfg
            for name, fn in (('plain C', lambda: sg.gemm(xs, w1f)),
                             ('down N768', lambda: sg.gemm(hs, w2f)),
                             ('gelu(u)', lambda: sg.gemm_gelu(xs, w1f, b1)),
                             ("gelu+gelu'", lambda: sg.gemm_gelu(xs, w1f, b1, deriv=True)),
                             ('dgelu(u)', lambda: sg.gemm_dgelu(dys, w2t, u, None, None)),
                             ("dgelu(gelu')", lambda: sg.gemm_dgelu(dys, w2t, gd, None, None, deriv=True))):
                k = (name, cfg)
                res[k] = min(res.get(k, 1e9), timeit(fn))
    os.environ.pop('HX_GEMM_CFG', None)
    for name in ('plain C', 'down N768', 'gelu(u)', "gelu+gelu'", 'dgelu(u)', "dgelu(gelu')"):
        print('{:13s} '.format(name) + ' | '.join('cfg {} {:6.1f} us {:5.0f} TF/s'.format(c, res[(name, c)],
                                                                                      fl / res[(name, c)] / 1e6)
                                                 for c in ('0', '1', '7')), flush=True)


if __name__ == '__main__':
    main()
