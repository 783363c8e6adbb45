"""Forward / data-gradient GEMMs of --fp32-gemm bf16x3/x6: the hand-written LDS-DMA piece GEMM
(csrc/kernels/gemm_split.hip, every tile configuration) vs the library on pass-stacked planes,
BERT-base shapes, checked against fp64; plus the fused FFN epilogues (bias + GELU pieces,
GELU backward pieces + dbias) against the unfused two-kernel path.

    python tools/bench_gemm_split.py [--tokens 16384] [--passes 6] [--cfgs 0,1,2] [--lib]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def relerr(got, ref, scale):
    return ((got.double() - ref).abs() / scale).max().item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--tokens', type=int, default=16384)
    ap.add_argument('--passes', default='6,3')
    ap.add_argument('--cfgs', default='0,1,2')
    ap.add_argument('--lib', action='store_true', help='also time the library on pass-stacked planes')
    a = ap.parse_args()
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    T = a.tokens
    g = torch.Generator(device='cpu').manual_seed(0)
    cfgs = [int(c) for c in a.cfgs.split(',')]
    bn = {0: 192, 1: 256, 2: 128, 7: 128}
    for passes in [int(p) for p in a.passes.split(',')]:
        ops.set_fp32_gemm('bf16x{}'.format(passes))
        # (name, n_in, n_out): forward y[T, n_out] = x W^T; dgrad dx[T, n_in] = dy W
        for name, n_in, n_out in (('qkv', 768, 2304), ('ao', 768, 768), ('up', 768, 3072), ('down', 3072, 768)):
            x = (torch.rand(T, n_in, generator=g) * 2 - 1).cuda()
            W = ((torch.rand(n_out, n_in, generator=g) * 2 - 1) * 0.05).cuda()
            dy = (torch.rand(T, n_out, generator=g) * 2 - 1).cuda()
            xs, dys = sg.pieces(x), sg.pieces(dy)
            wf, wt = sg.weight_pieces(W)
            fl = 2.0 * T * n_in * n_out * passes
            ref_f = x.double() @ W.double().t()
            sc_f = x.double().abs() @ W.double().abs().t()
            ref_d = dy.double() @ W.double()
            sc_d = dy.double().abs() @ W.double().abs()
            for cfg in cfgs:
                os.environ['HX_GEMM_CFG'] = str(cfg)
                line = 'x{} {:5s} cfg {}'.format(passes, name, cfg)
                if n_out % bn[cfg] == 0:
                    t_f = timeit(lambda: sg.gemm(xs, wf))
                    e_f = relerr(sg.gemm(xs, wf), ref_f, sc_f)
                    line += ' | fwd {:7.1f} us {:6.0f} TF/s err {:.2e}'.format(t_f, fl / t_f / 1e6, e_f)
                if n_in % bn[cfg] == 0:
                    t_d = timeit(lambda: sg.gemm(dys, wt))
                    e_d = relerr(sg.gemm(dys, wt), ref_d, sc_d)
                    acc = torch.randn(T, n_in, device='cuda')
                    got = sg.gemm(dys, wt, out=acc.clone(), beta=True)
                    e_b = relerr(got, ref_d + acc.double(), sc_d + acc.double().abs())
                    t_b = timeit(lambda: sg.gemm(dys, wt, out=acc, beta=True))
                    line += ' | dgrad {:7.1f} us {:6.0f} TF/s err {:.2e} | beta {:7.1f} us err {:.2e}'.format(
                        t_d, fl / t_d / 1e6, e_d, t_b, e_b)
                print(line, flush=True)
            os.environ.pop('HX_GEMM_CFG', None)
            if a.lib:
                t_lf = timeit(lambda: sg.forward(x, W))
                print('x{} {:5s} library fwd on pass-stacked planes incl. split {:7.1f} us ({:6.0f} TF/s)'.format(
                    passes, name, t_lf, fl / t_lf / 1e6), flush=True)
            if name == 'up':
                # fused epilogues vs the two-kernel path
                b1 = (torch.randn(n_out, generator=g) * 0.1).cuda()
                u, hp = sg.gemm_gelu(xs, wf, b1)
                y1 = sg.gemm(xs, wf)
                hp_ref = sg.act_pieces(y1, b1, 'gelu')
                e_u = relerr(u, y1.double() + b1.double(), y1.double().abs() + b1.double().abs())
                hv = sum(hp.view(T, -1, n_out)[:, p].float().double() for p in range(sg.npieces()))
                hr = sum(hp_ref.view(T, -1, n_out)[:, p].float().double() for p in range(sg.npieces()))
                e_h = relerr(hv, hr, hr.abs() + 1e-3)
                t_g = timeit(lambda: sg.gemm_gelu(xs, wf, b1))
                t_ref = timeit(lambda: sg.act_pieces(sg.gemm(xs, wf), b1, 'gelu'))
                print('x{} up+gelu fused {:7.1f} us vs gemm+bias_act_planes {:7.1f} us | err u {:.2e} h {:.2e}'.format(
                    passes, t_g, t_ref, e_u, e_h), flush=True)
                # GELU backward fused into the FFN-down data gradient: dh = dy2 W2 (N = 3072)
                W2 = ((torch.rand(n_in, n_out, generator=g) * 2 - 1) * 0.05).cuda()   # [768, 3072]
                dy2 = (torch.rand(T, n_in, generator=g) * 2 - 1).cuda()
                dy2s = sg.pieces(dy2)
                _, w2t = sg.weight_pieces(W2)
                tp, db = sg.gemm_dgelu(dy2s, w2t, u, None, None)
                dh = sg.gemm(dy2s, w2t)
                tp_ref, db_ref = sg.act_grad_pieces(dh, u, None, 'gelu')
                tv = sum(tp.view(T, -1, n_out)[:, p].float().double() for p in range(sg.npieces()))
                tr = sum(tp_ref.view(T, -1, n_out)[:, p].float().double() for p in range(sg.npieces()))
                e_t = relerr(tv, tr, tr.abs() + 1e-3)
                e_db = relerr(db, db_ref.double(), db_ref.double().abs() + 1e-2)
                t_dg = timeit(lambda: sg.gemm_dgelu(dy2s, w2t, u, None, None))
                t_dref = timeit(lambda: sg.act_grad_pieces(sg.gemm(dy2s, w2t), u, None, 'gelu'))
                print('x{} down-dgrad+dgelu fused {:7.1f} us vs gemm+bias_act_planes {:7.1f} us | err t {:.2e} '
                      'dbias {:.2e}'.format(passes, t_dg, t_dref, e_t, e_db), flush=True)
            del x, W, dy, xs, dys, wf, wt
            torch.cuda.empty_cache()
    ops.set_fp32_gemm('native')


if __name__ == '__main__':
    main()
