"""Where the k loop of the 16x16x32 fp16x3 GEMM (gemm_f16q_k, cfg 7) spends its time: the
timing-only switches HX_GEMM_Q_PROBE (results WRONG by construction) -- 1 no k-loop DMA, 2 no
k-loop fragment reads, 4 no k-loop waits / barrier, 8 no MFMAs, and their sums -- on pre-split A
(AT 2, plain epilogue) at T = 16384 token rows; HIP events, median of 20 calls, variants
interleaved twice after a warm-up.  Also cfg 1 (32x32x16) on the same operands."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, n=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[n // 2] * 1e3


def main():
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda', 0)
    T = int(os.environ.get('T', '16384'))
    g = torch.Generator(device=dev).manual_seed(0)
    variants = os.environ.get('QPROBE', 'c1,0,1,2,4,8,3,7,15').split(',')
    for (name, N, K) in [('qkv', 2304, 768), ('ffn_down', 768, 3072)]:
        x = torch.randn(T, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.03
        xp = C().amax_rows(x)
        xs = C().split_rows_f16(x, xp)
        wf, wt, wp, wc = C().split_weight_f16([W])[0]
        fl = 3 * 2.0 * T * N * K
        for _ in range(50):
            C().gemm_f16(xs, xp, wf, wp)
        res = {v: [] for v in variants}
        for _ in range(2):
            for v in variants:
                if v == 'c1':
                    os.environ['HX_GEMM_F16_CFG'] = '1'
                    os.environ.pop('HX_GEMM_Q_PROBE', None)
                else:
                    os.environ['HX_GEMM_F16_CFG'] = '7'
                    os.environ['HX_GEMM_Q_PROBE'] = v
                res[v].append(timed(lambda: C().gemm_f16(xs, xp, wf, wp)))
        for v in variants:
            us = min(res[v])
            print('{:9s} probe {:3s} {:7.1f} us ({:4.2f} PF/s pieces)  [{}]'.format(
                name, v, us, fl / us / 1e9, ' '.join('%.1f' % t for t in res[v])), flush=True)
    os.environ.pop('HX_GEMM_Q_PROBE', None)
    os.environ.pop('HX_GEMM_F16_CFG', None)


if __name__ == '__main__':
    main()
