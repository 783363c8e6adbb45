"""Per-phase cycle breakdown of the piece GEMM main loop (diagnostic stamp build, cfg 0):
DMA issue, MFMA issue, DMA wait (counted vmcnt), barrier -- mean cycles per k step per wave."""
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
    for name, n_in, n_out in (('ao', 768, 768), ('down', 3072, 768), ('qkv', 768, 2304)):
        x = torch.rand(T, n_in, device='cuda') * 2 - 1
        W = (torch.rand(n_out, n_in, device='cuda') * 2 - 1) * 0.05
        xs, wf = sg.pieces(x), sg.weight_pieces(W)[0]
        lay = int(os.environ.get('LAY', '0'))
        if lay:
            def blk(p):
                return p.view(p.shape[0], 3, -1, 16).permute(0, 2, 1, 3).contiguous().view(p.shape[0], -1)
            xs, wf = blk(xs), blk(wf)
        for _ in range(5):
            st = C().gemm_split_stamps(xs, wf, lay)
        torch.cuda.synchronize()
        st = st.double()
        live = st[:, 4] > 0
        st = st[live]
        nit = n_in // 16
        m = st.mean(0) / nit
        tot = st[:, 4].mean() / nit
        print('{:5s} cycles per k step per wave: dma issue {:6.0f} | mfma {:6.0f} | dma wait {:6.0f} | barrier {:6.0f} '
              '| loop total {:6.0f} (ideal MFMA 2304 per SIMD pair) | wave spread of barrier: p10 {:.0f} p90 {:.0f}'
              .format(name, m[0], m[1], m[2], m[3], tot, (st[:, 3] / nit).quantile(0.1), (st[:, 3] / nit).quantile(0.9)),
              flush=True)


if __name__ == '__main__':
    main()
