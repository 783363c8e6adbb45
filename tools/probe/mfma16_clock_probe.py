"""DVFS probe: the piece GEMM (cfg 0, natural layout, interleaved DMA) with its 32x32x16 MFMAs vs
the same kernel issuing two 16x16x32 MFMAs per 32x32x16 (equal pipe cycles; results are wrong,
timing only).  MI355X_MICROARCH.md 'DVFS give-back' item 7: the chip may hold a higher clock on
16x16x32.  Interleaved rounds in one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    os.environ['HX_GEMM_CFG'] = '0'
    T = 16384
    for name, n_in, n_out in (('ao', 768, 768), ('down', 3072, 768)):
        x = torch.rand(T, n_in, device='cuda') * 2 - 1
        W = (torch.rand(n_out, n_in, device='cuda') * 2 - 1) * 0.05
        xs, wf = sg.pieces(x), sg.weight_pieces(W)[0]
        fns = {'32x32x16': lambda: C().gemm_split(xs, wf, 6), '16x16x32': lambda: C().gemm_split_mfma16_timing(xs, wf)}
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, fn in fns.items():
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(20):
                    fn()
                b.record()
                b.synchronize()
                res[k].append(a.elapsed_time(b) / 20 * 1e3)
        print(name, {k: '{:.1f} us'.format(min(v)) for k, v in res.items()}, flush=True)


if __name__ == '__main__':
    main()
