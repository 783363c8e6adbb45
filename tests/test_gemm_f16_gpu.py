"""fp16x3 GEMMs (csrc/kernels/gemm_f16.hip) against fp64 references.

Error measure per output element: |C - C64| / (|A| |B|^T) -- the error relative to the sum of
the absolute product terms, the bound an fp32 dot product's rounding obeys.  fp16x3 keeps 22
significant bits of each operand and drops only the h1 h1 term (2^-22 relative), so its error is
of the order of fp32 accumulation rounding; the tests require it within a small factor of the
native fp32 GEMM's own error on the same data, and below an absolute fp32-class bound.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def C():
    from hetseq_9cme_amd.ops._ext import C as _C
    return _C()


def _rel_err(out, ref64, a, b):
    """max over elements of |out - ref| / (|a| |b|^T)."""
    den = a.abs().double() @ b.abs().double().t()
    err = (out.double() - ref64).abs() / den.clamp_min(1e-300)
    return err.max().item()


def _native_err(a, b, ref64):
    torch.backends.cuda.matmul.allow_tf32 = False
    return _rel_err(torch.mm(a, b.t()), ref64, a, b)


def _pieces(W):
    """(wf, wt, rmax, cmax): pieces of W (forward B operand, scaled per row of W) and of W^T (data
    gradient B operand, scaled per column of W) with those per-row scale sources."""
    wf, wt, rmax, cmax = C().split_weight_f16([W.contiguous()])[0]
    return wf, wt, rmax, cmax


@pytest.mark.parametrize('M,N,K,sa', [(16384, 768, 768, 1.0), (16384, 2304, 768, 3e-2), (16384, 3072, 768, 1.0),
                                      (16384, 768, 3072, 5e-3), (4096 + 37, 768, 768, 1.0), (1000, 768, 768, 1e-8),
                                      (2560, 768, 768, 1e8), (100, 128, 256, 1.0)])
def test_gemm_f16_forward(dev, M, N, K, sa):
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    a = torch.randn(M, K, device=dev, generator=g) * sa
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    wf, wt, rmax, cmax = _pieces(W)
    out = C().gemm_f16(a, C().amax_rows(a), wf, rmax)
    ref = a.double() @ W.double().t()
    e16 = _rel_err(out, ref, a, W)
    e32 = _native_err(a, W, ref)
    print('fwd M{} N{} K{} scale {:g}: fp16x3 {:.3g} native fp32 {:.3g}'.format(M, N, K, sa, e16, e32))
    assert e16 < 4e-6 and e16 < 4 * e32 + 1e-7


@pytest.mark.parametrize('M,N,K', [(16384, 768, 768), (16384, 768, 3072), (4096, 3072, 768), (512, 2304, 768)])
def test_gemm_f16_dgrad_beta_bias(dev, M, N, K):
    """dx = dy W (+ acc): the data-gradient operand wt = pieces of W^T; beta accumulates, bias adds."""
    g = torch.Generator(device=dev).manual_seed(7 * M + N)
    dy = torch.randn(M, N, device=dev, generator=g) * 1e-5
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    wf, wt, rmax, cmax = _pieces(W)
    acc = torch.randn(M, K, device=dev, generator=g) * 1e-5
    ref = acc.double() + dy.double() @ W.double()
    out = acc.clone()
    C().gemm_f16(dy, C().amax_rows(dy), wt, cmax, out=out, beta=True)
    den = (dy.abs().double() @ W.abs().double()) + acc.abs().double()
    e = ((out.double() - ref).abs() / den).max().item()
    assert e < 4e-6, e
    bias = torch.randn(K, device=dev, generator=g)
    out2 = C().gemm_f16(dy, C().amax_rows(dy), wt, cmax, bias=bias)
    ref2 = dy.double() @ W.double() + bias.double()
    den2 = (dy.abs().double() @ W.abs().double()) + bias.abs().double()
    assert ((out2.double() - ref2).abs() / den2).max().item() < 4e-6


@pytest.mark.parametrize('cfg', ['plan', '4'])
def test_gemm_f16_gelu_epilogues(dev, monkeypatch, cfg):
    """FFN up (bias + GELU: C = gelu'(u), P = gelu(u), max |P| per (row, N tile) and per (M tile,
    column)) and the FFN-down data gradient with the GELU backward (t = acc * gelu'(u), column sums
    = d bias, the same maxima of t), on the planned tile and on the two-per-CU 128 x 192 one."""
    from hetseq_9cme_amd.ops.fused import gelu_ref
    if cfg != 'plan':
        monkeypatch.setenv('HX_GEMM_F16_CFG', cfg)
    g = torch.Generator(device=dev).manual_seed(11)
    M, H, I = 16384 + 64, 768, 3072
    x = torch.randn(M, H, device=dev, generator=g)
    W1 = torch.randn(I, H, device=dev, generator=g) * 0.02
    b1 = torch.randn(I, device=dev, generator=g) * 0.1
    w1f, w1t, r1, c1 = _pieces(W1)
    d, h, hrow, hcol = C().gemm_f16_gelu(x, C().amax_rows(x), w1f, r1, b1, 1)
    u64 = x.double() @ W1.double().t() + b1.double()
    u = u64.float()
    h64 = gelu_ref(u64)
    den = x.abs().double() @ W1.abs().double().t() + b1.abs().double()
    assert ((h.double() - h64).abs() / den).max().item() < 1e-5
    ug = u.clone().requires_grad_(True)
    gelu_ref(ug).sum().backward()
    torch.testing.assert_close(d, ug.grad, rtol=2e-5, atol=2e-5)
    assert torch.equal(hrow.amax(1), h.abs().amax(1)) and torch.equal(hcol.amax(0), h.abs().amax(0))
    # backward: t = (dy W2) * gelu'(u)
    W2 = torch.randn(H, I, device=dev, generator=g) * 0.02
    w2f, w2t, r2, c2 = _pieces(W2)
    dy = torch.randn(M, H, device=dev, generator=g) * 1e-4
    t, trow, tcol, db = C().gemm_f16_dgelu(dy, C().amax_rows(dy), w2t, c2, d, None, None, 1)
    dh64 = dy.double() @ W2.double()
    t64 = dh64 * d.double()
    den = (dy.abs().double() @ W2.abs().double()) * d.abs().double()
    assert ((t.double() - t64).abs() / den.clamp_min(1e-300)).max().item() < 1e-5
    # d b1 = column sums of t over 16448 rows: relative to the sum of |t| (cancellation), and exactly
    # the kernel's own t summed (the per-wave partials + fold are the only extra rounding)
    assert ((db.double() - t64.sum(0)).abs() / t64.abs().sum(0)).max().item() < 1e-6
    assert ((db.double() - t.double().sum(0)).abs() / t.double().abs().sum(0)).max().item() < 1e-6
    assert torch.equal(trow.amax(1), t.abs().amax(1)) and torch.equal(tcol.amax(0), t.abs().amax(0))


def test_gemm_f16_split_k(dev):
    """The MLM decoder's data gradient shape: 40 output tiles over K = 30720 in split-K slabs."""
    g = torch.Generator(device=dev).manual_seed(5)
    M, N, K = 2560, 768, 30720
    a = torch.randn(M, K, device=dev, generator=g) * 1e-3
    W = torch.randn(N, K, device=dev, generator=g) * 0.02   # W^T of the decoder weight [K, N]
    wf, wt, rmax, cmax = _pieces(W)
    ks = C().gemm_f16_ks(M, N, K, C().gemm_f16_plan(M, N, K))
    assert ks > 1
    out = C().gemm_f16(a, C().amax_rows(a), wf, rmax, ks=0)
    ref = a.double() @ W.double().t()
    assert _rel_err(out, ref, a, W) < 4e-6


@pytest.mark.parametrize('ks', [2, 3, 6])
def test_gemm_f16_split_k_beta_bias(dev, ks):
    """Fine-tuning-sized data gradient (1000 token rows, K = 3072): split-K slabs combined with the
    beta = 1 accumulation and the bias in one pass (slab_combine_k), forced and planned."""
    g = torch.Generator(device=dev).manual_seed(ks)
    M, N, K = 1000, 768, 3072
    a = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    bias = torch.randn(N, device=dev, generator=g)
    acc = torch.randn(M, N, device=dev, generator=g)
    wf, wt, rmax, cmax = _pieces(W)
    ap = C().amax_rows(a)
    out = acc.clone()
    C().gemm_f16(a, ap, wf, rmax, out=out, beta=True, bias=bias, ks=ks)
    ref = acc.double() + a.double() @ W.double().t() + bias.double()
    den = acc.double().abs() + a.double().abs() @ W.double().abs().t() + bias.double().abs()
    assert ((out.double() - ref).abs() / den).max().item() < 4e-6
    assert C().gemm_f16_ks(M, N, K, 2) > 1      # the 128 x 96 tile splits this shape
    out2 = acc.clone()
    C().gemm_f16(a, ap, wf, rmax, out=out2, beta=True)
    ref2 = acc.double() + a.double() @ W.double().t()
    assert ((out2.double() - ref2).abs() / den).max().item() < 4e-6


@pytest.mark.parametrize('T,M,N,mvalid', [(16384, 2304, 768, 2304), (16384, 768, 3072, 768), (16384, 3072, 768, 3072),
                                          (4096, 768, 768, 768), (2560, 30720, 768, 30522), (1000, 256, 384, 256)])
def test_wgrad_f16(dev, T, M, N, mvalid):
    g = torch.Generator(device=dev).manual_seed(T + M)
    dy = torch.randn(T, M, device=dev, generator=g) * 1e-6
    x = torch.randn(T, N, device=dev, generator=g)
    out = torch.empty(mvalid, N, device=dev)
    C().wgrad_f16(dy, C().amax_cols(dy), x, C().amax_cols(x), out)
    ref = dy.double().t()[:mvalid] @ x.double()
    den = dy.abs().double().t()[:mvalid] @ x.abs().double()
    e16 = ((out.double() - ref).abs() / den).max().item()
    e32 = ((torch.mm(dy.t()[:mvalid], x).double() - ref).abs() / den).max().item()
    print('wgrad T{} M{} N{}: fp16x3 {:.3g} native fp32 {:.3g}'.format(T, M, N, e16, e32))
    assert e16 < 4e-6 and e16 < 4 * e32 + 1e-7


def test_f16_scale_extremes(dev):
    """Operands far outside fp16's range (1e-30, 1e30) and an all-zero operand keep fp32 accuracy /
    give exact zeros: the power-of-two scale comes from each tensor's max |x|."""
    g = torch.Generator(device=dev).manual_seed(3)
    W = torch.randn(768, 768, device=dev, generator=g) * 0.02
    wf, wt, rmax, cmax = _pieces(W)
    for s in (1e-30, 1e30):
        a = torch.randn(4096, 768, device=dev, generator=g) * s
        out = C().gemm_f16(a, C().amax_rows(a), wf, rmax)
        ref = a.double() @ W.double().t()
        assert _rel_err(out, ref, a, W) < 4e-6, s
    z = torch.zeros(4096, 768, device=dev)
    assert C().gemm_f16(z, C().amax_rows(z), wf, rmax).abs().max().item() == 0.0


@pytest.mark.parametrize('M,N,K', [(16384, 768, 768), (16384, 3072, 768), (4096, 768, 3072), (300, 2304, 768)])
def test_gemm_bf16_mode(dev, M, N, K):
    """--precision bf16 on the same kernel (one bf16 pass, bf16 or fp32 output, bias / beta): against
    the fp64 product of the same bf16 operands (only fp32 accumulation and the output rounding)."""
    g = torch.Generator(device=dev).manual_seed(M + K)
    a = torch.randn(M, K, device=dev, generator=g).bfloat16()
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    Wb = W.bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    ref = a.double() @ Wb.double().t() + bias.double()
    den = a.double().abs() @ Wb.double().abs().t() + bias.double().abs()
    out32 = C().gemm_bf16(a, Wb, bias=bias, out_bf16=False)
    assert ((out32.double() - ref).abs() / den).max().item() < 1e-5
    out16 = C().gemm_bf16(a, Wb, bias=bias)
    assert out16.dtype == torch.bfloat16
    assert ((out16.double() - ref).abs() / den).max().item() < 8e-3
    # data gradient through W^T (bf16 copy) with beta into a bf16 accumulator
    wt = C().weight_bf16_t([W.contiguous()])[0]
    assert torch.equal(wt, Wb.t().contiguous())
    dy = torch.randn(M, N, device=dev, generator=g).bfloat16()
    acc = torch.randn(M, K, device=dev, generator=g).bfloat16()
    ref2 = acc.double() + dy.double() @ Wb.double()
    den2 = acc.double().abs() + dy.double().abs() @ Wb.double().abs()
    out = acc.clone()
    C().gemm_bf16(dy, wt, out=out, beta=True)
    assert ((out.double() - ref2).abs() / den2).max().item() < 8e-3


@pytest.mark.parametrize('cfg', ['plan', '2', '4'])
def test_gemm_bf16_gelu_epilogues(dev, monkeypatch, cfg):
    """--precision bf16 FFN epilogues on the bf16 variant: up (bias + GELU -> gelu'(u), gelu(u) in
    bf16) and the FFN-down data gradient times gelu'(u) with the bias-gradient column sums, against
    fp64 of the same bf16 operands (bf16 output rounding only); rows not a multiple of the tile."""
    from hetseq_9cme_amd.ops.fused import gelu_ref
    if cfg != 'plan':
        monkeypatch.setenv('HX_GEMM_F16_CFG', cfg)
    g = torch.Generator(device=dev).manual_seed(13)
    M, H, I = 4096 + 37, 768, 3072
    x = torch.randn(M, H, device=dev, generator=g).bfloat16()
    W1 = (torch.randn(I, H, device=dev, generator=g) * 0.02).bfloat16()
    b1 = torch.randn(I, device=dev, generator=g) * 0.1
    d, h = C().gemm_bf16_gelu(x, W1, b1)
    assert d.dtype == h.dtype == torch.bfloat16
    u64 = x.double() @ W1.double().t() + b1.double()
    den = x.abs().double() @ W1.abs().double().t() + b1.abs().double()
    assert ((h.double() - gelu_ref(u64)).abs() / den).max().item() < 8e-3
    ug = u64.float().requires_grad_(True)
    gelu_ref(ug).sum().backward()
    torch.testing.assert_close(d.float(), ug.grad, rtol=8e-3, atol=8e-3)
    W2 = (torch.randn(H, I, device=dev, generator=g) * 0.02).bfloat16()
    w2t = W2.t().contiguous()
    dy = (torch.randn(M, H, device=dev, generator=g) * 1e-3).bfloat16()
    t, db = C().gemm_bf16_dgelu(dy, w2t, d)
    assert t.dtype == torch.bfloat16 and db.dtype == torch.float32
    t64 = (dy.double() @ W2.double()) * d.double()
    den = (dy.abs().double() @ W2.abs().double()) * d.abs().double()
    assert ((t.double() - t64).abs() / den.clamp_min(1e-300)).max().item() < 8e-3
    # d b1: fp32 sums of the fp32 products (before their bf16 rounding)
    assert ((db.double() - t64.sum(0)).abs() / t64.abs().sum(0)).max().item() < 1e-5
    slot = torch.zeros(I, device=dev)
    C().gemm_bf16_dgelu(dy, w2t, d, slot)
    assert torch.equal(slot, db)


@pytest.mark.parametrize('lib', [True, False])
def test_ffn_bf16_autograd(dev, monkeypatch, lib):
    """ops.ffn on bf16 activations (the --precision bf16 BERT FFN): output and every gradient
    against the fp32 reference of the same op on the same bf16-rounded operands -- both routes:
    hipBLASLt products with the bias-GELU passes (default) and the hand-written kernel's fused
    GELU epilogues (HX_BF16_LIB=0)."""
    from hetseq_9cme_amd.ops import fused, gemm16
    from hetseq_9cme_amd.ops.fused import gelu_ref
    monkeypatch.setattr(gemm16, '_BF16_LIB', lib)
    g = torch.Generator(device=dev).manual_seed(17)
    T, H, I = 2048, 768, 3072
    x = torch.randn(4, T // 4, H, device=dev, generator=g).bfloat16().requires_grad_(True)
    W1 = (torch.randn(I, H, device=dev, generator=g) * 0.02).requires_grad_(True)
    b1 = (torch.randn(I, device=dev, generator=g) * 0.1).requires_grad_(True)
    W2 = (torch.randn(H, I, device=dev, generator=g) * 0.02).requires_grad_(True)
    assert fused.ffn_fusable(x, W1, b1, W2)
    y = fused.ffn(x, W1, b1, W2)
    assert y.dtype == torch.bfloat16
    dy = torch.randn(y.shape, device=dev, generator=g).bfloat16()
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    W1r, b1r, W2r = [t.detach().clone().requires_grad_(True) for t in (W1, b1, W2)]
    h = gelu_ref(xr @ W1r.bfloat16().float().t() + b1r)
    yr = h @ W2r.bfloat16().float().t()
    yr.backward(dy.float())
    rel = lambda a, b: ((a.float() - b).norm() / b.norm()).item()
    assert rel(y, yr) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    assert rel(W1.grad, W1r.grad) < 1e-2 and rel(W2.grad, W2r.grad) < 1e-2 and rel(b1.grad, b1r.grad) < 1e-2


@pytest.mark.parametrize('cfg', ['0', '1', '2', '3', '4', '5', '6'])
def test_gemm_f16_every_tile(dev, monkeypatch, cfg):
    """Every tile configuration of gemm_f16_k (HX_GEMM_F16_CFG forces it): forward with bias and the
    beta = 1 data gradient, rows not a multiple of the tile."""
    monkeypatch.setenv('HX_GEMM_F16_CFG', cfg)
    g = torch.Generator(device=dev).manual_seed(int(cfg))
    M, N, K = 4096 + 37, 768, 768
    a = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    bias = torch.randn(N, device=dev, generator=g)
    wf, wt, rmax, cmax = _pieces(W)
    out = C().gemm_f16(a, C().amax_rows(a), wf, rmax, bias=bias)
    ref = a.double() @ W.double().t() + bias.double()
    den = a.abs().double() @ W.abs().double().t() + bias.abs().double()
    assert ((out.double() - ref).abs() / den).max().item() < 4e-6
    acc = torch.randn(M, K, device=dev, generator=g)
    dy = torch.randn(M, N, device=dev, generator=g)
    o2 = acc.clone()
    C().gemm_f16(dy, C().amax_rows(dy), wt, cmax, out=o2, beta=True)
    ref2 = acc.double() + dy.double() @ W.double()
    den2 = acc.abs().double() + dy.abs().double() @ W.abs().double()
    assert ((o2.double() - ref2).abs() / den2).max().item() < 4e-6
    # an odd number of k steps per slab (16 slabs of 3 steps): the loop's last step is unpaired
    o3 = C().gemm_f16(a, C().amax_rows(a), wf, rmax, bias=bias, ks=16)
    assert ((o3.double() - ref).abs() / den).max().item() < 4e-6


@pytest.mark.parametrize('plan', ['0:1', '0:5', '1:1', '1:3'])
def test_wgrad_f16_every_plan(dev, monkeypatch, plan):
    """Both tiles and split counts of wgrad_f16_k (HX_WGRAD_F16="cfg:nsplit" forces them)."""
    monkeypatch.setenv('HX_WGRAD_F16', plan)
    g = torch.Generator(device=dev).manual_seed(len(plan))
    T, M, N = 3000, 768, 512
    dy = torch.randn(T, M, device=dev, generator=g) * 1e-3
    x = torch.randn(T, N, device=dev, generator=g)
    out = torch.empty(M, N, device=dev)
    C().wgrad_f16(dy, C().amax_cols(dy), x, C().amax_cols(x), out)
    ref = dy.double().t() @ x.double()
    den = dy.abs().double().t() @ x.abs().double()
    assert ((out.double() - ref).abs() / den).max().item() < 4e-6


@pytest.mark.parametrize('plan', ['0:1', '1:3', '2:2', '3:4'])
def test_wgrad_bf16_every_plan(dev, monkeypatch, plan):
    """The bf16 weight-gradient kernel's tiles / split counts (HX_WGRAD_CFG="cfg:nsplit")."""
    monkeypatch.setenv('HX_WGRAD_CFG', plan)
    g = torch.Generator(device=dev).manual_seed(7)
    T, M, N = 4096, 768, 512
    dy = torch.randn(T, M, device=dev, generator=g).bfloat16()
    x = torch.randn(T, N, device=dev, generator=g).bfloat16()
    out = torch.empty(M, N, device=dev)
    C().wgrad_bf16(dy, x, out)
    ref = dy.double().t() @ x.double()
    den = dy.double().abs().t() @ x.double().abs()
    assert ((out.double() - ref).abs() / den).max().item() < 1e-5


@pytest.mark.parametrize('plan', ['0:1', '2:3'])
def test_wgrad_bf16_row_limit(dev, monkeypatch, plan):
    """dW over a tile-padded M (the MLM decoder's padded vocabulary) into an output of fewer rows:
    the rows past it are not stored (a canary row right after the output stays untouched), with
    and without the split-K slab sum."""
    monkeypatch.setenv('HX_WGRAD_CFG', plan)
    g = torch.Generator(device=dev).manual_seed(3)
    T, M, N, V = 2048, 1536, 128, 1000
    dy = torch.randn(T, M, device=dev, generator=g).bfloat16()
    dy[:, V:] = 0
    x = torch.randn(T, N, device=dev, generator=g).bfloat16()
    buf = torch.full((V + 8, N), 7.0, device=dev)
    out = buf[:V]
    C().wgrad_bf16(dy, x, out)
    ref = dy[:, :V].double().t() @ x.double()
    den = dy[:, :V].double().abs().t() @ x.double().abs()
    assert ((out.double() - ref).abs() / den).max().item() < 1e-5
    assert (buf[V:] == 7.0).all()


def _row_err(out, ref64, den):
    """per output row: max over its columns of |out - ref| / (|a| |b|^T) -- each row against its own
    magnitude."""
    return ((out.double() - ref64).abs() / den.clamp_min(1e-300)).amax(1)


@pytest.mark.parametrize('side', ['a', 'b'])
def test_gemm_f16_row_ramp(dev, side):
    """The fp16x3 precision envelope across rows (VERDICT r4 Next #2): A's rows (side a) or W's rows
    = output columns (side b) ramped over 2^0 .. 2^-30 of the tensor's largest.  Per-row operand
    scales keep every row at fp32 class: the row-wise error (each row against its own sum of
    |a| |b| products) within 4x the native fp32 GEMM's on every row, the rows within 2^-20 of the
    max included, and the data gradient (W^T's rows = W's columns ramped) likewise."""
    g = torch.Generator(device=dev).manual_seed(21)
    M, N, K = 4096, 768, 768
    a = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    if side == 'a':
        a = a * torch.pow(2.0, -torch.linspace(0, 30, M, device=dev)).unsqueeze(1)
    else:
        W = W * torch.pow(2.0, -torch.linspace(0, 30, N, device=dev)).unsqueeze(1)
    wf, wt, rmax, cmax = _pieces(W)
    out = C().gemm_f16(a, C().amax_rows(a), wf, rmax)
    ref = a.double() @ W.double().t()
    den = a.abs().double() @ W.abs().double().t()
    e16 = _row_err(out, ref, den)
    e32 = _row_err(torch.mm(a, W.t()), ref, den)
    worst = (e16 / (e32 + 1e-9)).max().item()
    print('row ramp {}: max row err fp16x3 {:.3g} native {:.3g}, worst row ratio {:.2f}'.format(
        side, e16.max().item(), e32.max().item(), worst))
    assert (e16 <= 4 * e32 + 2e-7).all(), worst
    # data gradient: dx = dy W, the B operand W^T whose rows are W's (ramped) columns / rows
    dy = torch.randn(M, N, device=dev, generator=g)
    if side == 'a':
        dy = dy * torch.pow(2.0, -torch.linspace(0, 30, M, device=dev)).unsqueeze(1)
    Wt = W.t().contiguous()
    if side == 'b':   # ramp W's columns (the rows of W^T)
        Wt = (W * torch.pow(2.0, -torch.linspace(0, 30, K, device=dev)).unsqueeze(0)).t().contiguous()
    Wd = Wt.t().contiguous()
    wf2, wt2, rmax2, cmax2 = _pieces(Wd)
    dx = C().gemm_f16(dy, C().amax_rows(dy), wt2, cmax2)
    ref = dy.double() @ Wd.double()
    den = dy.abs().double() @ Wd.abs().double()
    e16 = _row_err(dx, ref, den)
    e32 = _row_err(torch.mm(dy, Wd), ref, den)
    assert (e16 <= 4 * e32 + 2e-7).all(), (e16 / (e32 + 1e-9)).max().item()


def test_wgrad_f16_column_ramp(dev):
    """The weight gradient's envelope (VERDICT r4 Next #2): dY's columns (= dW's rows) ramped over
    2^0 .. 2^-30 and X's columns (= dW's columns) over 2^0 .. 2^-20; per-column operand scales
    keep every dW element within 4x the native fp32 GEMM's error relative to its own sum of
    |dy| |x| products."""
    g = torch.Generator(device=dev).manual_seed(23)
    T, M, N = 4096, 768, 512
    dy = torch.randn(T, M, device=dev, generator=g) * torch.pow(2.0, -torch.linspace(0, 30, M, device=dev))
    x = torch.randn(T, N, device=dev, generator=g) * torch.pow(2.0, -torch.linspace(0, 20, N, device=dev))
    out = torch.empty(M, N, device=dev)
    C().wgrad_f16(dy, C().amax_cols(dy), x, C().amax_cols(x), out)
    ref = dy.double().t() @ x.double()
    den = dy.abs().double().t() @ x.abs().double()
    e16 = ((out.double() - ref).abs() / den.clamp_min(1e-300))
    e32 = ((torch.mm(dy.t(), x).double() - ref).abs() / den.clamp_min(1e-300))
    print('wgrad column ramp: max err fp16x3 {:.3g} native {:.3g}'.format(e16.max().item(), e32.max().item()))
    assert (e16.amax(1) <= 4 * e32.amax(1) + 2e-7).all()


@pytest.mark.parametrize('rows,cols', [(16384, 2304), (1000, 768), (77, 4096), (5, 4)])
def test_amax_rows_cols_one_pass(rows, cols):
    """The fused row + column max |x| pass (the scale sources of a tensor no producer described)
    equals the row-wise and column-wise maxima exactly, rows ramped over 2^-20 .. 2^20."""
    from hetseq_9cme_amd.ops._ext import C
    dev = torch.device('cuda')
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(rows, cols, device=dev, generator=g) * torch.pow(
        2.0, torch.linspace(-20, 20, rows, device=dev))[:, None]
    r, c = C().amax_rows_cols(x)
    assert torch.equal(r, x.abs().amax(1, keepdim=True))
    assert torch.equal(c, x.abs().amax(0, keepdim=True))


@pytest.mark.parametrize('cfg', ['plan', '0', '2', '3', '4', '5', '6'])
def test_gemm_f16_presplit_a_bitwise(dev, monkeypatch, cfg):
    """A handed over already split into fp16 P2 pieces at its row scales (split_rows_f16, or a
    LayerNorm's pieces_out) is read as it is (AT 2: no split in the k loop) and gives results
    bit-identical to the fp32 A split in registers -- every epilogue, ragged M, rows ramped over
    2^-20 .. 2^20."""
    if cfg != 'plan':
        monkeypatch.setenv('HX_GEMM_F16_CFG', cfg)
    g = torch.Generator(device=dev).manual_seed(31)
    M, N, K = 4096 + 37, 768, 768
    a = torch.randn(M, K, device=dev, generator=g) * torch.pow(2.0, torch.linspace(-20, 20, M, device=dev))[:, None]
    am = C().amax_rows(a)
    ap = C().split_rows_f16(a, am)
    assert ap.dtype == torch.float16 and ap.shape == (M, 2 * K)
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    wf, wt, rmax, cmax = _pieces(W)
    b = torch.randn(N, device=dev, generator=g)
    assert torch.equal(C().gemm_f16(a, am, wf, rmax, bias=b), C().gemm_f16(ap, am, wf, rmax, bias=b))
    acc = torch.randn(M, N, device=dev, generator=g)
    o0, o1 = acc.clone(), acc.clone()
    C().gemm_f16(a, am, wf, rmax, out=o0, beta=True)
    C().gemm_f16(ap, am, wf, rmax, out=o1, beta=True)
    assert torch.equal(o0, o1)
    for p, q in zip(C().gemm_f16_gelu(a, am, wf, rmax, b, 1), C().gemm_f16_gelu(ap, am, wf, rmax, b, 1)):
        assert torch.equal(p, q)
    u = torch.randn(M, N, device=dev, generator=g)
    for p, q in zip(C().gemm_f16_dgelu(a, am, wf, rmax, u, None, None, 1),
                    C().gemm_f16_dgelu(ap, am, wf, rmax, u, None, None, 1)):
        assert torch.equal(p, q)


def test_gemm_f16_presplit_a_split_k(dev):
    """Pre-split A through the split-K slabs (deep K): bit-identical to the fp32 operand."""
    g = torch.Generator(device=dev).manual_seed(37)
    M, N, K = 512, 768, 3072
    a = torch.randn(M, K, device=dev, generator=g)
    am = C().amax_rows(a)
    W = torch.randn(N, K, device=dev, generator=g) * 0.02
    wf, wt, rmax, cmax = _pieces(W)
    assert torch.equal(C().gemm_f16(a, am, wf, rmax, ks=3), C().gemm_f16(C().split_rows_f16(a, am), am, wf, rmax, ks=3))


def test_layernorm_pieces_out(dev):
    """LayerNorm forward / backward write their output's P2 pieces at the row scales they compute
    (the consumer GEMM's A operand, pre-split): equal to split_rows_f16 of the fp32 output."""
    g = torch.Generator(device=dev).manual_seed(41)
    rows, H = 4096 + 3, 768
    seed = torch.full((1,), 1234, dtype=torch.int64, device=dev)
    y = torch.randn(rows, H, device=dev, generator=g)
    res = torch.randn(rows, H, device=dev, generator=g)
    bias = torch.randn(H, device=dev, generator=g)
    gamma = torch.randn(H, device=dev, generator=g)
    beta = torch.randn(H, device=dev, generator=g)
    am = torch.empty(rows, 1, device=dev)
    pc = torch.empty(rows, 2 * H, dtype=torch.float16, device=dev)
    out, z, mean, rstd = C().ln_fwd(y, bias, res, gamma, beta, 1e-12, 0.9, seed, 3, False, True, am, pc)
    assert torch.equal(am, out.abs().amax(1, keepdim=True))
    assert torch.equal(pc, C().split_rows_f16(out, am))
    dout = torch.randn(rows, H, device=dev, generator=g) * 1e-3
    for want_dy in (True, False):
        bm = torch.empty(rows, 1, device=dev)
        bp = torch.empty(rows, 2 * H, dtype=torch.float16, device=dev)
        dz, dy, _, _, _ = C().ln_bwd(dout, z, mean, rstd, gamma, 0.9, seed, 3, False, want_dy, want_dy, None, None,
                                     None, bm, None, bp)
        src = dy if want_dy else dz
        assert torch.equal(bm, src.abs().amax(1, keepdim=True))
        assert torch.equal(bp, C().split_rows_f16(src, bm))


def test_embed_layernorm_pieces_out(dev):
    """The embedding LayerNorm (gather + sum + LN + dropout) writes its output's P2 pieces at the
    row scales it computes, like ln_fwd: the first layer's QKV GEMM reads them pre-split (AT 2)."""
    g = torch.Generator(device=dev).manual_seed(43)
    B, S, H, V = 8, 128, 768, 1000
    ids = torch.randint(0, V, (B, S), device=dev, generator=g)
    tt = torch.randint(0, 2, (B, S), device=dev, generator=g)
    wte = torch.randn(V, H, device=dev, generator=g) * 0.05
    wpe = torch.randn(512, H, device=dev, generator=g) * 0.05
    wtt = torch.randn(2, H, device=dev, generator=g) * 0.05
    gamma = torch.randn(H, device=dev, generator=g)
    beta = torch.randn(H, device=dev, generator=g)
    seed = torch.full((1,), 99, dtype=torch.int64, device=dev)
    am = torch.empty(B * S, 1, device=dev)
    pc = torch.empty(B * S, 2 * H, dtype=torch.float16, device=dev)
    out, z, mean, rstd = C().embed_ln_fwd(ids, tt, wte, wpe, wtt, gamma, beta, 1e-12, 0.9, seed, 5, False, am, pc)
    o2 = out.view(B * S, H)
    assert torch.equal(am, o2.abs().amax(1, keepdim=True))
    assert torch.equal(pc, C().split_rows_f16(o2, am))
    out_ref = C().embed_ln_fwd(ids, tt, wte, wpe, wtt, gamma, beta, 1e-12, 0.9, seed, 5, False, am)[0]
    assert torch.equal(out, out_ref)   # the pieces output changes nothing else


def test_split_weight_virtual_padding(dev):
    """split_weight_f16 with a padded row count reads the rows past W's own as zero: bit-identical
    to splitting a zero-padded copy (the MLM decoder's vocabulary, 30522 -> 30720 rows)."""
    g = torch.Generator(device=dev).manual_seed(43)
    V, H, Vp = 30522, 768, 30720
    W = torch.randn(V, H, device=dev, generator=g) * 0.05
    Wp = torch.zeros(Vp, H, device=dev)
    Wp[:V] = W
    a = C().split_weight_f16([W], [Vp])[0]
    b = C().split_weight_f16([Wp])[0]
    for p, q in zip(a, b):
        assert p.shape == q.shape and torch.equal(p, q)


def test_ffn_large_partials_fit(dev):
    """BERT-large's FFN at 20480 token rows (phase 2, batch 40): the GELU epilogues' partials can
    exceed the consumers' limits (64 row partials for a GEMM, 256 column partials for a weight
    gradient); gemm16 folds them, and the FFN-down forward and both weight gradients run on them."""
    from hetseq_9cme_amd.ops import gemm16
    g = torch.Generator(device=dev).manual_seed(3)
    M, H, I = 20480, 1024, 4096
    x = torch.randn(M, H, device=dev, generator=g)
    W1 = torch.randn(I, H, device=dev, generator=g) * 0.02
    b1 = torch.randn(I, device=dev, generator=g) * 0.1
    W2 = torch.randn(H, I, device=dev, generator=g) * 0.02
    was = gemm16.enabled()
    gemm16.set_enabled(True)
    try:
        d, h, hrow, hcol, w1t, p1 = gemm16.gemm_gelu(x, C().amax_rows(x), W1, b1)
        assert hrow.shape[1] <= gemm16.MAX_ROW_PARTS and hcol.shape[0] <= gemm16.MAX_COL_PARTS
        assert torch.equal(hrow.amax(1), h.abs().amax(1)) and torch.equal(hcol.amax(0), h.abs().amax(0))
        y, w2t, p2 = gemm16.linear(h, hrow, W2)
        ref = h.double() @ W2.double().t()
        assert _rel_err(y, ref, h, W2) < 4e-6
        dy = torch.randn(M, H, device=dev, generator=g) * 1e-4
        dW2 = gemm16.wgrad(dy, C().amax_cols(dy), h, hcol, H, I)
        ref = dy.double().t() @ h.double()
        den = dy.abs().double().t() @ h.abs().double()
        assert ((dW2.double() - ref).abs() / den).max().item() < 4e-6
        t, trow, tcol, db = gemm16.gemm_dgelu(dy, C().amax_rows(dy), w2t, p2, d, None)
        assert trow.shape[1] <= gemm16.MAX_ROW_PARTS and tcol.shape[0] <= gemm16.MAX_COL_PARTS
        dW1 = gemm16.wgrad(t, tcol, x, C().amax_cols(x), I, H)
        ref = t.double().t() @ x.double()
        den = t.abs().double().t() @ x.abs().double()
        assert ((dW1.double() - ref).abs() / den).max().item() < 4e-6
    finally:
        gemm16.set_enabled(was)


@pytest.mark.parametrize('T,M,N,mvalid', [(16384, 2304, 768, 2304), (16384, 768, 3072, 768), (4096, 768, 768, 768),
                                          (2560, 30720, 768, 30522), (1000, 3072, 768, 3072), (333, 768, 768, 768)])
def test_wgrad_f16_addtid_staging_bitwise(dev, monkeypatch, T, M, N, mvalid):
    """The 256 x 256 weight gradient with add-tid piece staging (the default; HX_WGRAD_TID=0 selects
    the ds_write_b128 kernel): b64 column-pair loads, ds_write_addtid_b32 stores into a row-rotated
    image, against the ds_write_b128 kernel:
    the same pieces in the same MFMA order, so bit for bit -- token counts off the 16-token stage,
    split-K slabs and the MLM decoder's padded rows included."""
    g = torch.Generator(device=dev).manual_seed(T + M + N)
    dy = torch.randn(T, M, device=dev, generator=g) * 1e-3
    x = torch.randn(T, N, device=dev, generator=g)
    dc, xc = C().amax_cols(dy), C().amax_cols(x)
    ref = torch.full((mvalid, N), float('nan'), device=dev)
    monkeypatch.setenv('HX_WGRAD_TID', '0')
    C().wgrad_f16(dy, dc, x, xc, ref)
    for variant in ('1', '2'):   # 16- and 32-token stages
        out = torch.full((mvalid, N), float('nan'), device=dev)
        monkeypatch.setenv('HX_WGRAD_TID', variant)
        C().wgrad_f16(dy, dc, x, xc, out)
        torch.cuda.synchronize()
        assert torch.isfinite(out).all()
        assert torch.equal(out, ref), (variant, (out - ref).abs().max().item())
    r64 = dy.double().t()[:mvalid] @ x.double()
    den = dy.abs().double().t()[:mvalid] @ x.abs().double()
    assert ((out.double() - r64).abs() / den).max().item() < 4e-6
