"""A short fixed workload for counter passes over the split-piece weight-gradient kernel:
the four BERT-base dW shapes at T = 16384 tokens, bf16x6, 10 calls each with the default
plan (``bash tools/pmc_run.sh NAME "<counters>" python3 tools/probe/wgrad_pmc_probe.py``)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    T = 16384
    for (n_out, n_in) in [(3072, 768), (768, 3072), (2304, 768), (768, 768)]:
        dy = torch.randn(T, n_out, device='cuda')
        x = torch.randn(T, n_in, device='cuda')
        dys, xs = sg.grad_planes(dy), sg.planes(x, sg.ORDER_P[6])
        po, px = sg._piece_offsets(sg.ORDER_Q[6], n_out), sg._piece_offsets(sg.ORDER_P[6], n_in)
        slot = torch.empty(n_out, n_in, device='cuda')
        for _ in range(10):
            C().wgrad_split(dys, po, xs, px, 6, n_out, n_in, slot)
        torch.cuda.synchronize()
    print('done')


if __name__ == '__main__':
    main()
