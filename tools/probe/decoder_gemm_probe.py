"""Probe: the MLM decoder's split-path GEMMs at BERT-base phase 1 (2560 masked rows, H=768,
V=30522, bf16x6): forward logits with V vs V padded to 256 (aligned output rows), and the
data gradient dh = dlogits . W over the padded vocabulary, pass-stacked (K' = 6 Vp) vs the
prefix form (3 distinct pieces, ops/split_gemm.py prefix_mm).

``python tools/probe/decoder_gemm_probe.py`` (one MI355X)."""
import sys
import time

import torch

sys.path.insert(0, '.')


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    from hetseq_9cme_amd.ops import split_gemm
    split_gemm.set_fp32_gemm('bf16x6')
    dev = 'cuda'
    M, H, V = 2560, 768, 30522
    Vp = (V + 255) // 256 * 256
    h = torch.randn(M, H, device=dev)
    W = torch.randn(V, H, device=dev) * 0.02
    Wp = torch.zeros(Vp, H, device=dev)
    Wp[:V] = W
    xs = split_gemm.planes(h, split_gemm.ORDER_P[6])
    wq = split_gemm.planes(W, split_gemm.ORDER_Q[6])
    wqp = split_gemm.planes(Wp, split_gemm.ORDER_Q[6])
    t_fwd = timeit(lambda: torch.mm(xs, wq.t(), out_dtype=torch.float32))
    t_fwdp = timeit(lambda: torch.mm(xs, wqp.t(), out_dtype=torch.float32))
    print(f'forward  V={V}: {t_fwd:7.1f} us | padded Vp={Vp}: {t_fwdp:7.1f} us', flush=True)
    dl = torch.randn(M, V, device=dev) * 1e-3
    dls = split_gemm.grad_planes(dl, dpad=Vp)
    t_dg = timeit(lambda: split_gemm.dgrad(dls, W, rpad=Vp))
    dln = split_gemm.planes(torch.nn.functional.pad(dl, (0, Vp - V)), split_gemm.ORDER_N[6])
    t_dgp = timeit(lambda: split_gemm.dgrad_prefix(dln, Wp))
    ref = split_gemm.dgrad(dls, W, rpad=Vp)
    got = split_gemm.dgrad_prefix(dln, Wp)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    t_split6 = timeit(lambda: split_gemm.grad_planes(dl, dpad=Vp))
    # split-K as a strided batched product: K' = 6 Vp cut into S slabs (batch stride = slab,
    # lda = K'), fp32 partial products summed afterwards (S x 7.9 MB)
    wt = split_gemm.weight_planes_t(W, Vp)
    wb = wt.t()
    Kp = wb.shape[0]
    for S in (4, 8, 12, 16, 24, 32):
        if Kp % S:
            continue
        kc = Kp // S
        a = dls.view(M, S, kc).transpose(0, 1)
        b = wb.reshape(S, kc, H) if wb.is_contiguous() else wb.view(S, kc, H)

        def sk():
            return torch.bmm(a, b, out_dtype=torch.float32).sum(0)
        try:
            got = sk()
        except Exception as e:   # noqa: BLE001
            print('bmm out_dtype unsupported:', e, flush=True)
            break
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        print(f'dgrad    split-K S={S:2d} (bmm + sum): {timeit(sk):7.1f} us (rel diff {err:.1e})', flush=True)
    print(f'dgrad    stacked K\'=6Vp: {t_dg:7.1f} us | prefix form: {t_dgp:7.1f} us (rel diff {err:.1e}) | '
          f'6-plane split of dl {t_split6:7.1f} us', flush=True)


if __name__ == '__main__':
    main()
