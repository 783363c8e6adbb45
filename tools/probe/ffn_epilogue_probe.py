"""FFN GELU epilogues vs separate passes at the BERT-base phase-1 shape (16384 tokens): the FFN-up
GEMM with bias + GELU in its epilogue against the plain GEMM + bias_act_fwd, and the FFN-down
data gradient with the GELU backward against the plain GEMM + bias_act_bwd, for both modes
(fp16x3, --precision bf16) and each large tile (HX_GEMM_F16_CFG 0 / 1 / 4).
``python tools/probe/ffn_epilogue_probe.py``."""
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
    dev = torch.device('cuda', 0)
    T, H, I = 16384, 768, 3072
    x = torch.randn(T, H, device=dev)
    W1 = torch.randn(I, H, device=dev) * 0.02
    b1 = torch.randn(I, device=dev) * 0.1
    W2 = torch.randn(H, I, device=dev) * 0.02
    dy = torch.randn(T, H, device=dev) * 1e-3
    xb, W1b, W2b, dyb = x.bfloat16(), W1.bfloat16(), W2.bfloat16(), dy.bfloat16()
    w2tb = W2b.t().contiguous()
    w1f, _, p1 = C().split_weight_f16([W1])[0]
    _, w2t, p2 = C().split_weight_f16([W2])[0]
    xa, dya = C().amax_rows(x), C().amax_rows(dy)
    d16, _ = C().gemm_bf16_gelu(xb, W1b, b1)
    d32, _, _ = C().gemm_f16_gelu(x, xa, w1f, p1, b1, 1)
    u16 = C().gemm_bf16(xb, W1b)
    u32 = C().gemm_f16(x, xa, w1f, p1)
    for cfg in ('0', '1', '4'):
        os.environ['HX_GEMM_F16_CFG'] = cfg
        r = {
            'bf16 up fused': timed(lambda: C().gemm_bf16_gelu(xb, W1b, b1)),
            'bf16 up plain': timed(lambda: C().gemm_bf16(xb, W1b)),
            'bf16 down-dgrad fused': timed(lambda: C().gemm_bf16_dgelu(dyb, w2tb, d16)),
            'bf16 down-dgrad plain': timed(lambda: C().gemm_bf16(dyb, w2tb)),
            'bf16 down-dgrad fused dmode0': timed(lambda: C().gemm_bf16_dgelu(dyb, w2tb, u16, None, b1, 0)),
            'f16x3 up fused': timed(lambda: C().gemm_f16_gelu(x, xa, w1f, p1, b1, 1)),
            'f16x3 up plain': timed(lambda: C().gemm_f16(x, xa, w1f, p1)),
            'f16x3 down-dgrad fused': timed(lambda: C().gemm_f16_dgelu(dy, dya, w2t, p2, d32, None, None, 1)),
            'f16x3 down-dgrad plain': timed(lambda: C().gemm_f16(dy, dya, w2t, p2)),
        }
        print('cfg {}: '.format(cfg) + ', '.join('{} {:.1f} us'.format(k, v) for k, v in r.items()), flush=True)
    os.environ.pop('HX_GEMM_F16_CFG')
    r = {
        'bf16 bias_act fwd': timed(lambda: C().bias_act_fwd(u16, b1, 0)),
        'bf16 bias_act bwd': timed(lambda: C().bias_act_bwd(u16, u16, b1, None, 0, True, None)),
        'fp32 bias_act fwd': timed(lambda: C().bias_act_fwd(u32, b1, 0)),
        'fp32 bias_act bwd': timed(lambda: C().bias_act_bwd(u32, u32, b1, None, 0, True, None)),
    }
    print('separate passes: ' + ', '.join('{} {:.1f} us'.format(k, v) for k, v in r.items()), flush=True)


if __name__ == '__main__':
    main()
