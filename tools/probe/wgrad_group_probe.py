"""Grouped weight-gradient launches (wgrad_split.hip, bf16x6, T = 16384): the attention block's
QKV dW (2304 x 768) + attention-output dW (768 x 768), and the FFN's W1 dW (3072 x 768) + W2 dW
(768 x 3072), each pair as two separate launches (their own split plans) vs ONE grouped launch;
results compared bit for bit (same token-split sums?) and against fp64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_gemm_split import timeit  # noqa: E402


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    T = 16384
    pairs = {'attn (qkv + ao)': ((2304, 768), (768, 768)), 'ffn (w1 + w2)': ((3072, 768), (768, 3072))}
    for name, shapes in pairs.items():
        ops_ = []
        for (M, N) in shapes:
            dy = torch.rand(T, M, device='cuda') * 2 - 1
            x = torch.rand(T, N, device='cuda') * 2 - 1
            ops_.append((sg.pieces(dy), sg.pieces(x), M, N, torch.empty(M, N, device='cuda'),
                         torch.empty(M, N, device='cuda'), dy, x))

        def separate():
            for dys, xs, M, N, o, _, _, _ in ops_:
                C().wgrad_split(dys, [0, M, 2 * M], xs, [0, N, 2 * N], 6, M, N, o)

        def grouped():
            assert C().wgrad_split_group([(dys, [0, M, 2 * M], xs, [0, N, 2 * N], M, N, o2)
                                          for dys, xs, M, N, _, o2, _, _ in ops_])
        res = {'separate': 1e9, 'grouped': 1e9}
        for _ in range(3):
            res['separate'] = min(res['separate'], timeit(separate))
            res['grouped'] = min(res['grouped'], timeit(grouped))
        errs = []
        for dys, xs, M, N, o, o2, dy, x in ops_:
            ref = dy.double().t() @ x.double()
            sc = dy.double().abs().t() @ x.double().abs()
            errs.append((((o2.double() - ref).abs() / sc).max().item(), ((o.double() - ref).abs() / sc).max().item()))
        fl = sum(2.0 * T * M * N * 6 for (M, N) in shapes)
        print('{:16s} separate {:6.1f} us ({:5.0f} TF/s) | grouped {:6.1f} us ({:5.0f} TF/s) | rel err grouped / '
              'separate {}'.format(name, res['separate'], fl / res['separate'] / 1e6, res['grouped'],
                                   fl / res['grouped'] / 1e6, ['{:.1e}/{:.1e}'.format(*e) for e in errs]), flush=True)


if __name__ == '__main__':
    main()
