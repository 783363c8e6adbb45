"""The 128 x 96 GEMM tile (cfg 2, two workgroups per CU) with a four- vs five-stage DMA ring at
fine-tuning-sized M (HX_GEMM_NS5, read per call), forward of the BERT-base products, warmed up and
alternated.  ``T=2048 python tools/probe/small_m_ring_probe.py``.  The switch lived in a measurement
build (removed: the five-stage ring was 3-20 % slower, profiles/r6o_small_m_ring_probe.log)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    from hetseq_9cme_amd.ops._ext import C
    os.environ['HX_GEMM_F16_CFG'] = '2'
    g = torch.Generator(device='cuda').manual_seed(0)
    for T in [int(t) for t in os.environ.get('T', '2048,4096').split(',')]:
        for (name, N, K) in [('qkv', 2304, 768), ('attn_out', 768, 768), ('ffn_down', 768, 3072)]:
            x = torch.randn(T, K, device='cuda', generator=g)
            W = torch.randn(N, K, device='cuda', generator=g) * 0.03
            xp = C().amax_rows(x)
            wf, wt, wp, wc = C().split_weight_f16([W])[0]
            f = lambda: C().gemm_f16(x, xp, wf, wp, ks=1)
            os.environ['HX_GEMM_NS5'] = '0'
            timed(f, 100)
            r = {'0': [], '1': []}
            for _ in range(3):
                for v in ('0', '1'):
                    os.environ['HX_GEMM_NS5'] = v
                    r[v].append(timed(f))
            print('T{} {} N{} K{}: 4-stage {} us | 5-stage {} us'.format(
                T, name, N, K, ' '.join('%.1f' % v for v in r['0']), ' '.join('%.1f' % v for v in r['1'])), flush=True)
    os.environ.pop('HX_GEMM_NS5', None)


if __name__ == '__main__':
    main()
