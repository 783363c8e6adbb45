"""QKV forward (T = 16384, 768 -> 2304, bf16x6) on the piece GEMM: 256 x 128 tile over natural
weight pieces (cfg 2, the plan so far) vs 256 x 192 / 256 x 256 over B16 weight pieces (cfg 0 / 1,
lay 2), interleaved rounds in one process, checked against fp64."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools.bench_gemm_split import timeit, relerr  # noqa: E402


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    T = 16384
    for n_in, n_out in ((768, 2304), (768, 768), (3072, 768)):
        x = torch.rand(T, n_in, device='cuda') * 2 - 1
        W = (torch.rand(n_out, n_in, device='cuda') * 2 - 1) * 0.05
        xs = sg.pieces(x)
        wf, _ = C().split_weight(W, 3, 0)
        wb, _ = C().split_weight(W, 3, 1)
        ref = x.double() @ W.double().t()
        sc = x.double().abs() @ W.double().abs().t()
        fl = 2.0 * T * n_in * n_out * 6
        arms = [('cfg2 lay0', '2', wf, 0), ('cfg0 lay0', '0', wf, 0), ('cfg0 lay2', '0', wb, 2), ('cfg1 lay2', '1', wb, 2)]
        res = {}
        for rnd in range(3):
            for name, cfg, w, lay in arms:
                if n_out % {'0': 192, '1': 256, '2': 128}[cfg]:
                    continue
                os.environ['HX_GEMM_CFG'] = cfg
                t = timeit(lambda: C().gemm_split(xs, w, 6, None, False, lay))
                res[name] = min(res.get(name, 1e9), t)
                if rnd == 0:
                    assert relerr(C().gemm_split(xs, w, 6, None, False, lay), ref, sc) < 1e-6
        os.environ.pop('HX_GEMM_CFG', None)
        print('{}x{}: '.format(n_in, n_out) + ' | '.join('{} {:6.1f} us {:5.0f} TF/s'.format(k, v, fl / v / 1e6)
                                                       for k, v in res.items()), flush=True)


if __name__ == '__main__':
    main()
