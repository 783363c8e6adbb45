"""Timing-only probe of the fp16x3 weight gradient (wgrad_f16_k, 256 x 256 tile): what the k loop's
parts cost (profiles/r6g_gemm_wgrad_split_probe.md).  The switches lived in a measurement build of
gemm_f16.hip (a PRB template parameter read from the env at launch) that was removed after
measuring; the production kernels ignore these variables.  HX_WGRAD_PROBE (results WRONG for 1-7): 0 normal,
1 every stage re-reads the first 32 tokens (cache-resident loads), 2 no split (raw bits as pieces),
6 no split and no piece stores (stale LDS), 7 all three.  ``python tools/probe/wgrad_f16_probe.py``"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def timed(fn, n=20):
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
    T = 16384
    g = torch.Generator(device='cuda').manual_seed(0)
    for (M, N) in [(2304, 768), (3072, 768), (768, 3072), (768, 768)]:
        os.environ.pop('HX_WGRAD_PROBE', None)
        dy = torch.randn(T, M, device='cuda', generator=g)
        x = torch.randn(T, N, device='cuda', generator=g)
        dc, xc = C().amax_cols(dy), C().amax_cols(x)
        out = torch.empty(M, N, device='cuda')
        timed(lambda: C().wgrad_f16(dy, dc, x, xc, out), n=100)   # warm the clock / caches first
        row = []
        for p in os.environ.get('PROBES', '0,1,2,6,7').split(','):
            os.environ['HX_WGRAD_PROBE'] = p
            us = timed(lambda: C().wgrad_f16(dy, dc, x, xc, out))
            row.append('{}: {:.1f} us ({:.0f} TF/s pieces)'.format(p, us, 3 * 2.0 * T * M * N / us / 1e6))
        os.environ.pop('HX_WGRAD_PROBE')
        print('wgrad {}x{} T{}: '.format(M, N, T) + ', '.join(row), flush=True)


if __name__ == '__main__' and len(sys.argv) == 1:
    main()


def gemm_main():
    """The same for the forward / data-gradient GEMM (gemm_f16_k 256 x 192, plain epilogue, fp32 A):
    HX_GEMM_PROBE 0 normal, 2 cache-resident DMA (every k step re-reads stage 0), 3 no split of A,
    4 both."""
    from hetseq_9cme_amd.ops._ext import C
    T = 16384
    g = torch.Generator(device='cuda').manual_seed(0)
    for (N, K) in [(2304, 768), (768, 768), (768, 3072)]:
        x = torch.randn(T, K, device='cuda', generator=g)
        W = torch.randn(N, K, device='cuda', generator=g) * 0.03
        xp = C().amax_rows(x)
        wf, wt, wp, wc = C().split_weight_f16([W])[0]
        row = []
        for p in ('0', '2', '3', '4'):
            os.environ['HX_GEMM_PROBE'] = p
            us = timed(lambda: C().gemm_f16(x, xp, wf, wp))
            row.append('{}: {:.1f} us ({:.0f} TF/s pieces)'.format(p, us, 3 * 2.0 * T * N * K / us / 1e6))
        os.environ.pop('HX_GEMM_PROBE')
        print('gemm N{} K{} T{}: '.format(N, K, T) + ', '.join(row), flush=True)


def tid_main():
    """The add-tid staged weight gradient (HX_WGRAD_TID=1) against the ds_write_b128 one, same
    process, warmed up, alternated three times per shape."""
    from hetseq_9cme_amd.ops._ext import C
    T = int(os.environ.get('T', '16384'))
    g = torch.Generator(device='cuda').manual_seed(0)
    for (M, N) in [(2304, 768), (3072, 768), (768, 3072), (768, 768)]:
        dy = torch.randn(T, M, device='cuda', generator=g)
        x = torch.randn(T, N, device='cuda', generator=g)
        dc, xc = C().amax_cols(dy), C().amax_cols(x)
        out = torch.empty(M, N, device='cuda')
        os.environ['HX_WGRAD_TID'] = '0'
        timed(lambda: C().wgrad_f16(dy, dc, x, xc, out), n=100)
        res = {'0': [], '1': [], '2': []}
        for _ in range(3):
            for v in ('0', '1', '2'):
                os.environ['HX_WGRAD_TID'] = v
                res[v].append(timed(lambda: C().wgrad_f16(dy, dc, x, xc, out)))
        os.environ.pop('HX_WGRAD_TID')
        print('wgrad {}x{} T{}: b128 stores {} us | add-tid 16-token stages {} us | add-tid 32 {} us'.format(
            M, N, T, ' '.join('%.1f' % v for v in res['0']), ' '.join('%.1f' % v for v in res['1']),
            ' '.join('%.1f' % v for v in res['2'])), flush=True)


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'gemm':
    gemm_main()
if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'tid':
    tid_main()
