"""A short fixed workload for counter passes over the LDS-DMA piece GEMM (gemm_split.hip):
BERT-base forward / dgrad shapes at T = 16384 tokens, bf16x6, 10 calls each
(``bash tools/pmc_run.sh NAME "<counters>" python3 tools/probe/gemm_pmc_probe.py [cfg]``)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    if len(sys.argv) > 1:
        os.environ['HX_GEMM_CFG'] = sys.argv[1]
    ops.set_fp32_gemm('bf16x6')
    T = 16384
    shapes = [(768, 3072)] if os.environ.get('ONLY_DOWN') else [(768, 768), (3072, 768)]
    for (n_out, n_in) in shapes:
        x = torch.rand(T, n_in, device='cuda') * 2 - 1
        W = (torch.rand(n_out, n_in, device='cuda') * 2 - 1) * 0.05
        xs = sg.pieces(x)
        wf, _ = sg.weight_pieces(W)   # in the layout the plan reads (B16 where sg.b16(n_out))
        from hetseq_9cme_amd.ops._ext import C
        for _ in range(10):
            sg.gemm(xs, wf)
        torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()
