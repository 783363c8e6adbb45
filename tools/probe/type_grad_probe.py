"""Token-type embedding gradient at BERT-base phase 1 (16384 x 768, 2 types): the per-type column-sum
kernel vs the one-hot GEMM it replaced, fp32 and bf16 (median of event-timed calls)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gemm_f16_bench import timed  # noqa: E402


def main():
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rows, H, nt = 16384, 768, 2
    tt = torch.randint(0, nt, (rows,), device=dev, generator=g)
    out = torch.empty(nt, H, device=dev)
    for dt in (torch.float32, torch.bfloat16):
        dz = torch.randn(rows, H, device=dev, generator=g).to(dt)
        k = timed(lambda: C().embed_type_grad(dz, tt, out))

        def gemm():
            oh = torch.nn.functional.one_hot(tt, nt).to(dt)
            return torch.mm(oh.t(), dz)
        m = timed(gemm)
        print('{:9s} type-grad kernel {:6.1f} us   one-hot + GEMM {:6.1f} us'.format(str(dt).split('.')[-1], k, m),
              flush=True)


if __name__ == '__main__':
    main()
