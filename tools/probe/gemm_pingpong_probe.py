"""Default (PIPE 3) vs ping-pong (PIPE 8) piece GEMM on the BERT-base phase-1 shapes
(T = 16384 tokens, bf16x6, B16 weights, planned tile), plus the two FFN epilogues;
interleaved rounds in one process, best of 3.  Record of profiles/r3_gemm_pingpong_probe.log: PIPE 8
was removed after this measurement (gemm_split.hip, pipe_mode comment), so both columns now run
PIPE 3."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_gemm_split import timeit  # noqa: E402


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    ops.set_fp32_gemm('bf16x6')
    T = 16384
    cases = []
    for n_out, n_in in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        xs = sg.pieces(torch.rand(T, n_in, device='cuda') * 2 - 1)
        wf, _ = sg.weight_pieces((torch.rand(n_out, n_in, device='cuda') * 2 - 1) * 0.05)
        cases.append(('N%d K%d' % (n_out, n_in), 2.0 * T * n_out * n_in * 6, (lambda xs=xs, wf=wf: sg.gemm(xs, wf))))
    H, I = 768, 3072
    xs = sg.pieces(torch.rand(T, H, device='cuda') * 2 - 1)
    w1f, _ = sg.weight_pieces((torch.rand(I, H, device='cuda') * 2 - 1) * 0.05)
    b1 = (torch.rand(I, device='cuda') * 2 - 1) * 0.1
    _, w2t = sg.weight_pieces((torch.rand(H, I, device='cuda') * 2 - 1) * 0.05)
    dys = sg.pieces(torch.rand(T, H, device='cuda') * 2 - 1)
    gd, _ = sg.gemm_gelu(xs, w1f, b1, deriv=True)
    fl = 2.0 * T * H * I * 6
    cases.append(("gelu+gelu'", fl, lambda: sg.gemm_gelu(xs, w1f, b1, deriv=True)))
    cases.append(("dgelu(gelu')", fl, lambda: sg.gemm_dgelu(dys, w2t, gd, None, None, deriv=True)))
    res = {}
    for rnd in range(3):
        for pipe in ('3', '8'):
            os.environ['HX_GEMM_PIPE'] = pipe
            for name, _, fn in cases:
                res[(name, pipe)] = min(res.get((name, pipe), 1e9), timeit(fn))
    os.environ.pop('HX_GEMM_PIPE', None)
    for name, f, _ in cases:
        a, b = res[(name, '3')], res[(name, '8')]
        print('{:13s} pipe 3 {:6.1f} us {:5.0f} TF/s | pipe 8 {:6.1f} us {:5.0f} TF/s | {:+.1f} %'.format(
            name, a, f / a / 1e6, b, f / b / 1e6, 100 * (a - b) / a), flush=True)


if __name__ == '__main__':
    main()
