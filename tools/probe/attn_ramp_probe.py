"""Locate the worst dQ rows of the fp16x3 attention backward on ramped Q / dO magnitudes
(tests/test_kernels_gpu.py::test_attention_f16_backward_fp32_class 'ramp')."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda', 0)
    for S, with_bias, keep in ((384, True, 0.9), (384, False, 1.0), (384, True, 1.0), (384, False, 0.9),
                               (256, True, 0.9), (128, True, 0.9)):
        torch.manual_seed(2)
        B, nh, d = 2, 4, 64
        H = nh * d
        qkv = 2 * torch.randn(B, S, 3 * H, device=dev)
        dout = torch.randn(B, S, H, device=dev)
        r = torch.pow(2.0, torch.linspace(-16, 4, S, device=dev))
        dout = dout * r[None, :, None]
        qkv[:, :, :H] *= torch.pow(2.0, torch.linspace(-6, 3, S, device=dev))[None, :, None]
        bias = (0.5 * torch.randn(3 * H, device=dev)) if with_bias else None
        mask = torch.ones(B, S, device=dev)
        mask[1, S - 29:] = 0
        mb = ((1 - mask) * -10000.0).contiguous()
        seed = torch.full((1,), 99, dtype=torch.int64, device=dev)
        out, lse, dm = C().attn_fwd(qkv, mb, nh, keep, seed, 3, bias)
        g16 = C().attn_bwd_f16(dout, qkv, mb, out, lse, dm, nh, keep, bias, None, None, None)[0]
        g32 = C().attn_bwd(dout, qkv, mb, out, lse, dm, nh, keep, bias, None, None, None)[0]
        x = (qkv.double() + (bias.double() if bias is not None else 0)).requires_grad_(True)
        q = x.view(B, S, 3, nh, d).permute(2, 0, 3, 1, 4)
        pn = torch.softmax(q[0] @ q[1].transpose(-1, -2) / 8.0 + mb.double()[:, None, None, :], -1)
        km = torch.ones_like(pn)
        if keep < 1.0:
            bits = dm.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
            Sp = dm.shape[2]
            km = ((bits.unsqueeze(-1) >> torch.arange(32, device=dev)) & 1).reshape(B, nh, Sp, Sp)
            km = km[:, :, :S, :S].transpose(-1, -2).double() / keep
        p = pn * km
        ref = (p @ q[2]).permute(0, 2, 1, 3).reshape(B, S, H)
        ref.backward(dout.double())
        gq = x.grad.view(B, S, 3, nh, d)[:, :, 0]
        with torch.no_grad():
            qd = q.detach()
            do = dout.double().view(B, S, nh, d).transpose(1, 2)
            dd = (do * ref.detach().view(B, S, nh, d).transpose(1, 2)).sum(-1, keepdim=True)
            ds = pn * ((do @ qd[2].transpose(-1, -2)) * km).abs() + pn * dd.abs()
            sc = ((ds @ qd[1].abs()) / 8.0).transpose(1, 2).amax(-1)      # [B, S, nh]
        for name, g in (('f16', g16), ('fp32', g32)):
            a = g.view(B, S, 3, nh, d)[:, :, 0].double()
            rel = (a - gq).abs().amax(-1) / sc
            v, i = rel.flatten().topk(4)
            rows = [(int(j) // (S * nh), (int(j) // nh) % S, int(j) % nh) for j in i]
            print('S={} bias={} keep={} {}: worst natural-scale dQ rows {}'.format(
                S, with_bias, keep, name, [(rw, '{:.2e}'.format(float(x))) for rw, x in zip(rows, v)]), flush=True)
            b_, s_, h_ = rows[0]
            print('    got', a[b_, s_, h_, :3].tolist(), 'ref', gq[b_, s_, h_, :3].tolist(), 'scale',
                  float(sc[b_, s_, h_]), flush=True)


if __name__ == '__main__':
    main()
