"""MLM decoder products at batch 32 (640 masked rows x 30528-padded vocab x 768): forward and data
gradient under forced tile configurations (HX_GEMM_F16_CFG), median of repeated event timings."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gemm_f16_bench import timed  # noqa: E402


def main():
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, V, H = int(os.environ.get('M', '640')), 30528, 768
    x = torch.randn(M, H, device=dev, generator=g)
    W = torch.randn(V, H, device=dev, generator=g) * 0.02
    dl = torch.randn(M, V, device=dev, generator=g) * 1e-3
    xp, dp = C().amax_rows(x), C().amax_rows(dl)
    wf, wt, wr, wc = C().split_weight_f16([W])[0]
    for rep in range(2):
        for cfg in os.environ.get('CFGS', 'plan,3,2,1').split(','):
            if cfg == 'plan':
                os.environ.pop('HX_GEMM_F16_CFG', None)
            else:
                os.environ['HX_GEMM_F16_CFG'] = cfg
            f = timed(lambda: C().gemm_f16(x, xp, wf, wr))
            d = timed(lambda: C().gemm_f16(dl, dp, wt, wc, ks=0))
            print('M {} cfg {:4s} decoder fwd {:7.1f} us  dgrad {:7.1f} us'.format(M, cfg, f, d), flush=True)
    os.environ.pop('HX_GEMM_F16_CFG', None)


if __name__ == '__main__':
    main()
