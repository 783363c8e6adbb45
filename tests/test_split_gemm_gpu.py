"""fp32 GEMMs emulated on bf16 matrix cores (ops/split_gemm.py, csrc/kernels/split.hip).

* the plane kernel reproduces a torch reference split bit for bit (interleaved and
  stacked layouts, 2 and 3 pieces, any plane order);
* linear / fused-QKV forward, data gradient (with and without the fused residual
  gradient) and weight gradient in bf16x3 / bf16x6 match an fp64 reference to the
  error class of each mode (bf16x6 within a small factor of native fp32);
* a BERT-tiny training run in each mode tracks the native fp32 run.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _split_small_gemms(monkeypatch):
    """The tests' GEMMs are small: take the split path regardless of the row threshold."""
    from hetseq_9cme_amd.ops import split_gemm
    monkeypatch.setattr(split_gemm, 'MIN_ROWS', {3: 0, 6: 0})
    monkeypatch.setattr(split_gemm, 'PIECE_MIN_ROWS', 0)


def _ref_pieces(x, n):
    out, r = [], x.clone()
    for _ in range(n):
        p = r.to(torch.bfloat16)
        out.append(p)
        r = r - p.float()
    return out


@pytest.mark.parametrize('npieces,order,stacked', [(2, (0, 1, 0), False), (2, (0, 0, 1), True),
                                                   (3, (0, 1, 0, 2, 1, 0), False), (3, (0, 0, 1, 0, 1, 2), True)])
def test_split_planes_bitwise(dev, npieces, order, stacked):
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(3)
    x = (torch.randn(37, 264, generator=g) * torch.logspace(-6, 6, 264)).to(dev)
    out = C().split_planes(x, list(order), npieces, stacked, 0, 0)
    pcs = _ref_pieces(x, npieces)
    if stacked:
        ref = torch.cat([pcs[k] for k in order], 0)
    else:
        ref = torch.stack([pcs[k] for k in order], 1).reshape(x.shape[0], -1)
    assert out.shape == ref.shape
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))
    # the pieces reconstruct x to 2^-17 (2 pieces) / 2^-26 (3 pieces) relative
    s = sum(p.double() for p in pcs)
    tol = 2.0 ** -16 if npieces == 2 else 2.0 ** -25
    assert ((s - x.double()).abs() <= tol * x.double().abs()).all()


@pytest.mark.parametrize('stacked', [False, True])
def test_split_planes_padded_unaligned(dev, stacked):
    """General path: odd width, unaligned rows (a column slice), zero padding of rows
    (stacked) or columns (interleaved) -- the MLM decoder's 30522-wide case."""
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(4)
    big = torch.randn(21, 131, generator=g).to(dev)
    x = big[:, 1:122]                       # [21, 121], row stride 131, misaligned start
    order = (0, 0, 1)
    rpad, dpad = (32, 0) if stacked else (0, 128)
    out = C().split_planes(x, list(order), 2, stacked, rpad, dpad)
    pcs = _ref_pieces(x.contiguous(), 2)
    if stacked:
        ref = torch.zeros(3, 32, 121, dtype=torch.bfloat16, device=dev)
        for j, k in enumerate(order):
            ref[j, :21] = pcs[k]
        ref = ref.reshape(96, 121)
    else:
        ref = torch.zeros(21, 3, 128, dtype=torch.bfloat16, device=dev)
        for j, k in enumerate(order):
            ref[:, j, :121] = pcs[k]
        ref = ref.reshape(21, 384)
    assert out.shape == ref.shape
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize('npieces,order,N,npad', [(3, (0, 1, 0, 2, 1, 0), 192, 0), (2, (0, 1, 0), 128, 0),
                                                  (3, (0, 1, 0, 2, 1, 0), 150, 192)])
def test_split_planes_transposed_bitwise(dev, npieces, order, N, npad):
    """Transposed weight planes (the NT data-gradient operand): out[k][j * Np + n] =
    piece order[j] of W[n][k], rows n >= N zero (the MLM decoder's padded vocabulary)."""
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(5)
    K = 128
    W = (torch.randn(N, K, generator=g) * torch.logspace(-5, 5, K)).to(dev)
    out = C().split_planes_t(W, list(order), npieces, npad)
    Np = max(N, npad)
    pcs = _ref_pieces(W, npieces)
    ref = torch.zeros(K, len(order), Np, dtype=torch.bfloat16, device=dev)
    for j, k in enumerate(order):
        ref[:, j, :N] = pcs[k].t()
    ref = ref.reshape(K, -1)
    assert out.shape == ref.shape
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))


@pytest.mark.parametrize('npieces,order', [(3, (0, 0, 1, 0, 1, 2)), (2, (0, 0, 1))])
def test_split_planes_padded_even_stride(dev, npieces, order):
    """Vector path for odd-width rows with an even (8-B aligned) row stride -- the MLM
    decoder's [rows, 30522] logits gradient padded to 256 columns."""
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(6)
    big = torch.randn(37, 1006, generator=g).to(dev)
    x = big[:, :1001]                     # row stride 1006 floats (8-B aligned rows), width 1001
    out = C().split_planes(x, list(order), npieces, False, 0, 1024)
    pcs = _ref_pieces(x.contiguous(), npieces)
    ref = torch.zeros(37, len(order), 1024, dtype=torch.bfloat16, device=dev)
    for j, k in enumerate(order):
        ref[:, j, :1001] = pcs[k]
    ref = ref.reshape(37, -1)
    assert out.shape == ref.shape
    assert torch.equal(out.view(torch.int16), ref.view(torch.int16))


def _err(a, ref, scale):
    return ((a.double() - ref).abs() / scale.clamp(min=1e-30)).max().item()


@pytest.mark.parametrize('mode,tol', [('bf16x3', 6e-6), ('bf16x6', 2e-6)])
def test_linear_split_numerics(dev, mode, tol):
    from hetseq_9cme_amd import ops
    g = torch.Generator(device='cpu').manual_seed(5)
    T, K, N = 512, 768, 384
    x = torch.randn(T, K, generator=g).to(dev).requires_grad_(True)
    W = torch.randn(N, K, generator=g).to(dev).requires_grad_(True)
    dy = torch.randn(T, N, generator=g).to(dev)
    try:
        ops.set_fp32_gemm(mode)
        y = ops.linear(x, W)
        y.backward(dy)
    finally:
        ops.set_fp32_gemm('native')
    xd, Wd, dyd = x.detach().double(), W.detach().double(), dy.double()
    checks = [(y, xd @ Wd.t(), xd.abs() @ Wd.abs().t()),
              (x.grad, dyd @ Wd, dyd.abs() @ Wd.abs()),
              (W.grad, dyd.t() @ xd, dyd.abs().t() @ xd.abs())]
    for k, (got, ref, scale) in enumerate(checks):
        e = _err(got, ref, scale)
        assert e < tol, (mode, k, e)


def test_linear3_residual_split(dev):
    """Fused QKV projection + the residual-gradient mailbox (dgrad GEMM with beta = 1)."""
    from hetseq_9cme_amd import ops
    g = torch.Generator(device='cpu').manual_seed(9)
    T, H = 256, 256
    x = torch.randn(T, H, generator=g).to(dev).requires_grad_(True)
    ws = [torch.randn(H, H, generator=g).to(dev).requires_grad_(True) for _ in range(3)]
    dres = torch.randn(T, H, generator=g).to(dev)
    dy = torch.randn(T, 3 * H, generator=g).to(dev)
    mbox = ops.ResidualGrad()
    try:
        ops.set_fp32_gemm('bf16x6')
        y = ops.linear3(x, ws[0], ws[1], ws[2], None, None, None, res_grad=mbox)
        mbox.deposit(dres.clone())
        y.backward(dy)
    finally:
        ops.set_fp32_gemm('native')
    W = torch.cat([w.detach() for w in ws], 0).double()
    ref_y = x.detach().double() @ W.t()
    assert _err(y, ref_y, x.detach().double().abs() @ W.abs().t()) < 2e-6
    ref_dx = dres.double() + dy.double() @ W
    assert _err(x.grad, ref_dx, dres.double().abs() + dy.double().abs() @ W.abs()) < 2e-6
    dW = torch.cat([w.grad for w in ws], 0)
    assert _err(dW, dy.double().t() @ x.detach().double(), dy.double().abs().t() @ x.detach().double().abs()) < 2e-6


def test_training_split_modes_track_native(dev, tmp_path):
    """BERT-tiny, 3 updates, dropout 0: bf16x6 / bf16x3 weights stay within fp32-noise of
    the native fp32 run (native vs CPU reference is checked in test_kernels_gpu)."""
    import argparse
    import os
    import subprocess
    import sys
    from hetseq_9cme_amd.data.synthetic import BERT_TINY, write_bert_config, write_synthetic_bert_shards, write_vocab
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = tmp_path / 'data'
    write_synthetic_bert_shards(str(d), n_files=1, samples_per_file=64, seq_len=128, max_pred=20, vocab_size=1024,
                                split='train')
    cfg = write_bert_config(str(tmp_path / 'c.json'), **dict(BERT_TINY, hidden_dropout_prob=0.0,
                                                               attention_probs_dropout_prob=0.0))
    vocab = write_vocab(str(tmp_path / 'v.txt'), 1024)
    outs = {}
    for mode in ('native', 'bf16x6', 'bf16x3'):
        save = str(tmp_path / mode)
        cmd = [sys.executable, '-m', 'hetseq_9cme_amd.train', '--task', 'bert', '--data', str(d), '--dict', vocab,
               '--config_file', cfg, '--max-sentences', '8', '--fast-stat-sync', '--max-update', '3',
               '--disable-validation', '--num-workers', '1', '--lr', '1e-3', '--weight-decay', '0.01',
               '--clip-norm', '0.5', '--save-dir', save, '--distributed-world-size', '1', '--fp32-gemm', mode]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           env=dict(os.environ, PYTHONPATH=root, HETSEQ_SPLIT_MIN_ROWS_X6='0', HX_PIECE_MIN_ROWS='0'),
                           timeout=300)
        assert r.returncode == 0, r.stdout[-3000:]
        with torch.serialization.safe_globals([argparse.Namespace]):
            outs[mode] = torch.load(os.path.join(save, 'checkpoint_last.pt'), map_location='cpu', weights_only=True)
    for mode in ('bf16x6', 'bf16x3'):
        worst = 0.0
        for k, v in outs['native']['model'].items():
            if k.endswith('attention.self.key.bias'):
                continue   # exact gradient is 0 (softmax shift invariance): pure rounding noise that Adam amplifies
            d_ = (outs[mode]['model'][k].double() - v.double()).abs().max().item()
            worst = max(worst, d_ / (v.double().abs().max().item() + 1e-12))
        assert worst < (1e-4 if mode == 'bf16x6' else 5e-4), (mode, worst)


@pytest.mark.parametrize('mode,tol', [('bf16x3', 6e-6), ('bf16x6', 2e-6)])
def test_decoder_xent_split(dev, mode, tol):
    """MLM decoder + softmax-xent with a vocabulary that is not a multiple of 8 (padded planes)."""
    from hetseq_9cme_amd import ops
    g = torch.Generator(device='cpu').manual_seed(11)
    M, H, V = 96, 128, 1001
    h = torch.randn(M, H, generator=g).to(dev).requires_grad_(True)
    W = (torch.randn(V, H, generator=g) * 0.1).to(dev).requires_grad_(True)
    b = torch.randn(V, generator=g).to(dev).requires_grad_(True)
    labels = torch.randint(0, V, (M,), generator=g).to(dev)
    labels[::7] = -1
    try:
        ops.set_fp32_gemm(mode)
        loss = ops.decoder_xent(h, W, b, labels)
        loss.backward()
    finally:
        ops.set_fp32_gemm('native')
    hd, Wd, bd = h.detach().double().requires_grad_(True), W.detach().double().requires_grad_(True), \
        b.detach().double().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy(hd @ Wd.t() + bd, labels, ignore_index=-1)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-5 * abs(ref.item())
    for got, r in ((h.grad, hd.grad), (W.grad, Wd.grad), (b.grad, bd.grad)):
        e = (got.double() - r).abs().max().item() / r.abs().max().item()
        assert e < 50 * tol, (mode, e)


@pytest.mark.parametrize('prefix', ['1', '0'])
@pytest.mark.parametrize('mode,tol', [('bf16x3', 8e-6), ('bf16x6', 3e-6)])
def test_ffn_split_block(dev, mode, tol, prefix, monkeypatch):
    """FFN block as one node (GELU epilogue writes the FFN-down planes, GELU backward the
    FFN-up gradient planes + dbias) against an fp64 autograd reference; with and without the
    prefix form of the deep products (split_gemm.prefix_mm: distinct pieces only)."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as _sg
    monkeypatch.setattr(_sg, '_PREFIX_GEMM', prefix != '0')
    g = torch.Generator(device='cpu').manual_seed(13)
    T, H, I = 384, 256, 1024
    x = torch.randn(T, H, generator=g).to(dev).requires_grad_(True)
    W1 = (torch.randn(I, H, generator=g) * 0.05).to(dev).requires_grad_(True)
    b1 = (torch.randn(I, generator=g) * 0.1).to(dev).requires_grad_(True)
    W2 = (torch.randn(H, I, generator=g) * 0.05).to(dev).requires_grad_(True)
    dy = torch.randn(T, H, generator=g).to(dev)
    try:
        ops.set_fp32_gemm(mode)
        assert ops.ffn_fusable(x, W1, b1, W2)
        y = ops.ffn(x, W1, b1, W2)
        y.backward(dy)
    finally:
        ops.set_fp32_gemm('native')
    ps = [t.detach().double().requires_grad_(True) for t in (x, W1, b1, W2)]
    ref = ops.gelu_ref(ps[0] @ ps[1].t() + ps[2]) @ ps[3].t()
    ref.backward(dy.double())
    e = (y.double() - ref).abs().max().item() / ref.abs().max().item()
    assert e < tol, ('y', e)
    for name, got, r in zip(('x', 'W1', 'b1', 'W2'), (x.grad, W1.grad, b1.grad, W2.grad), ps):
        e = (got.double() - r.grad).abs().max().item() / r.grad.abs().max().item()
        assert e < tol, (name, e)


@pytest.mark.parametrize('mode,tol', [('bf16x3', 4e-6), ('bf16x6', 1.5e-6)])
def test_piece_gemm_kernels(dev, mode, tol):
    """Hand-written piece GEMM (gemm_split.hip, opt-in path) + weight pieces in both layouts
    (split_weight_k): forward, data gradient with beta = 1, rows that are not a multiple
    of the 256-row tile."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    g = torch.Generator(device='cpu').manual_seed(21)
    T, n_in, n_out = 300, 256, 384
    x = torch.randn(T, n_in, generator=g).to(dev)
    W = torch.randn(n_out, n_in, generator=g).to(dev)
    dy = torch.randn(T, n_out, generator=g).to(dev)
    acc0 = torch.randn(T, n_in, generator=g).to(dev)
    try:
        ops.set_fp32_gemm(mode)
        wf, wt = sg.weight_pieces(W)

        def lay(p, b16):   # natural pieces -> the layout weight_pieces chose
            if not b16:
                return p
            return p.view(p.shape[0], 3, -1, 16).permute(0, 2, 1, 3).contiguous().view(p.shape[0], -1)
        pw = lay(sg.pieces(W), sg.b16(n_out))
        assert torch.equal(wf.view(torch.int16), pw.view(torch.int16))
        pwt = lay(sg.pieces(W.t().contiguous()), sg.b16(n_in))
        assert torch.equal(wt.view(torch.int16), pwt.view(torch.int16))
        y = sg.gemm(sg.pieces(x), wf)
        acc = acc0.clone()
        sg.dgrad_pieces(sg.pieces(dy), wt, acc=acc)
    finally:
        ops.set_fp32_gemm('native')
    xd, Wd, dyd = x.double(), W.double(), dy.double()
    e = ((y.double() - xd @ Wd.t()).abs() / (xd.abs() @ Wd.abs().t())).max().item()
    assert e < tol, ('fwd', e)
    ref = acc0.double() + dyd @ Wd
    e = ((acc.double() - ref).abs() / (acc0.double().abs() + dyd.abs() @ Wd.abs())).max().item()
    assert e < tol, ('dgrad', e)


@pytest.mark.parametrize('mode,has_bias,keep', [('bf16x6', True, 0.9), ('bf16x3', False, 1.0), ('bf16x6', False, 0.9)])
def test_ln_bwd_planes_equal_split_of_dy(dev, mode, has_bias, keep):
    """LayerNorm backward writing dy as the upstream linear's gradient planes: bit-identical
    to splitting the fp32 dy of the plain backward, same dz / dgamma / dbeta / dbias."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm(mode)
    try:
        torch.manual_seed(3)
        T, H = 300, 768
        y = torch.randn(T, H, device=dev)
        res = torch.randn(T, H, device=dev)
        bias = torch.randn(H, device=dev) if has_bias else None
        gamma = torch.rand(H, device=dev) + 0.5
        beta = torch.randn(H, device=dev)
        seed = torch.tensor([1234], dtype=torch.int64, device=dev)
        out, z, mean, rstd = C().ln_fwd(y, bias, res, gamma, beta, 1e-12, keep, seed, 5, False, True)[:4]
        dout = torch.randn_like(out)
        dz, dy, dg, db, dbias = C().ln_bwd(dout, z, mean, rstd, gamma, keep, seed, 5, False, True, has_bias,
                                          None, None, None)
        n = split_gemm.passes()
        dz2, planes, dg2, db2, dbias2 = C().ln_bwd_planes(dout, z, mean, rstd, gamma, keep, seed, 5, has_bias,
                                                          list(split_gemm.ORDER_Q[n]), split_gemm.PIECES[n],
                                                          None, None, None)
        ref = split_gemm.grad_planes(dy)
        assert planes.shape == ref.shape
        assert torch.equal(planes.view(torch.int16), ref.view(torch.int16))
        assert torch.equal(dz, dz2) and torch.equal(dg, dg2) and torch.equal(db, db2)
        if has_bias:
            assert torch.equal(dbias, dbias2)
    finally:
        ops.set_fp32_gemm('native')


@pytest.mark.parametrize('natural', [False, True])
@pytest.mark.parametrize('mode,S,with_bias,keep', [('bf16x6', 128, True, 0.9), ('bf16x6', 77, False, 1.0),
                                                   ('bf16x3', 100, True, 0.9)])
def test_attn_bwd_planes_equal_split_of_dqkv(dev, mode, S, with_bias, keep, natural):
    """Split-piece attention backward writing dQKV as the QKV projection's gradient planes:
    bit-identical to splitting the fp32 dQKV of the same kernel, same QKV-bias gradient."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm(mode)
    try:
        torch.manual_seed(5)
        B, nh = 3, 4
        H = nh * 64
        qkv = torch.randn(B, S, 3 * H, device=dev)
        bias = 0.3 * torch.randn(3 * H, device=dev) if with_bias else None
        mb = torch.zeros(B, S, device=dev)
        mb[1, S - 9:] = -10000.0
        seed = torch.tensor([77], dtype=torch.int64, device=dev)
        out, lse, dm = C().attn_fwd_x6(qkv, mb, nh, keep, seed, 2, bias)[:3]
        dout = torch.randn_like(out)
        dqkv, db = C().attn_bwd_x6(dout, qkv, mb, out, lse, dm, nh, keep, bias, None, None, None)
        n = split_gemm.passes()
        order = split_gemm.ORDER_N[n] if natural else split_gemm.ORDER_Q[n]   # prefix form / pass-stacked
        planes, db2 = C().attn_bwd_x6_planes(dout, qkv, mb, out, lse, dm, nh, keep, bias, None, None, None,
                                             list(order))
        ref = split_gemm.planes(dqkv.view(B * S, 3 * H), order)
        assert planes.shape == ref.shape
        assert torch.equal(planes.view(torch.int16), ref.view(torch.int16))
        if with_bias:
            assert torch.equal(db, db2)
    finally:
        ops.set_fp32_gemm('native')


@pytest.mark.parametrize('piece_gemm', [True, False])
def test_grad_planes_handoff_in_bert_layer(dev, piece_gemm, monkeypatch):
    """A BERT layer under bf16x6 takes the LayerNorm -> linear and attention -> QKV projection
    gradient hand-offs (pieces for the hand-written piece GEMMs, pass-stacked planes for the
    library path): no linear splits its output gradient itself in the backward, and the
    gradients equal those of the same layer with the hand-offs disabled (to fp32 atomic-order
    noise)."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.models.bert import BertConfig, BertLayer
    from hetseq_9cme_amd.ops import fused, split_gemm
    monkeypatch.setattr(split_gemm._State, 'piece_gemm', piece_gemm)
    ops.set_fp32_gemm('bf16x6')
    try:
        torch.manual_seed(0)
        cfg = BertConfig(100, hidden_size=128, num_hidden_layers=1, num_attention_heads=2, intermediate_size=512,
                         hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        layer = BertLayer(cfg).to(dev)
        x = torch.randn(4, 64, 128, device=dev, requires_grad=True)
        mb = torch.zeros(4, 64, device=dev)
        splits = []
        orig_split, orig_pieces = split_gemm.grad_planes, split_gemm.pieces

        def spy_split(*a, **k):
            splits.append(1)
            return orig_split(*a, **k)

        def spy_pieces(*a, **k):
            splits.append(2)
            return orig_pieces(*a, **k)
        loss = layer(x, mb).pow(2).sum()
        split_gemm.grad_planes, split_gemm.pieces = spy_split, spy_pieces
        try:
            loss.backward()
        finally:
            split_gemm.grad_planes, split_gemm.pieces = orig_split, orig_pieces
        assert not splits, 'a linear split its output gradient itself (hand-off missed)'
        g1 = [p.grad.clone() for p in layer.parameters()] + [x.grad.clone()]
        for p in layer.parameters():
            p.grad = None
        x.grad = None
        orig_cls = fused.GradPlanes
        fused.GradPlanes = lambda: None
        ops.GradPlanes = fused.GradPlanes
        try:
            layer(x, mb).pow(2).sum().backward()
        finally:
            fused.GradPlanes = orig_cls
            ops.GradPlanes = orig_cls
        g2 = [p.grad.clone() for p in layer.parameters()] + [x.grad.clone()]
        for a, b in zip(g1, g2):
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
    finally:
        ops.set_fp32_gemm('native')


@pytest.mark.parametrize('T', [96, 4096])
def test_wgrad_split_row_padded_output(dev, T):
    """Split-piece weight gradient over a tile-padded M whose output holds only the valid
    rows (the MLM decoder's vocabulary): direct stores (small T) and the split-K sum (large
    T) both leave the rows past the output untouched and match the full product."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    ops.set_fp32_gemm('bf16x6')
    try:
        g = torch.Generator(device='cpu').manual_seed(13)
        Mv, Mp, N = 1001, 1024, 256
        dy = torch.zeros(T, Mp)
        dy[:, :Mv] = torch.randn(T, Mv, generator=g)
        x = torch.randn(T, N, generator=g)
        dys = sg.grad_planes(dy.to(dev))
        xs = sg.planes(x.to(dev), sg.ORDER_P[6])
        full = torch.empty(Mp, N, device=dev)
        sg.wgrad(dys, xs, Mp, N, full)
        buf = torch.full((Mv + 8, N), 7.0, device=dev)
        part = sg.wgrad(dys, xs, Mp, N, buf[:Mv])
        assert torch.equal(part, full[:Mv])
        assert (buf[Mv:] == 7.0).all()
        ref = dy[:, :Mv].double().t() @ x.double()
        scale = dy[:, :Mv].double().abs().t() @ x.double().abs()
        assert ((part.double().cpu() - ref).abs() / scale).max().item() < 2e-6
    finally:
        ops.set_fp32_gemm('native')


@pytest.mark.parametrize('T', [77, 1000, 4096])
def test_wgrad_split_pipeline_variants(dev, T, monkeypatch):
    """Every tile configuration and pipeline variant of the split-piece weight-gradient kernel
    (register staging two or one step ahead, LDS-DMA staging into two or three stages; both
    work orders) matches the fp64 product, also for token counts that end inside a pipeline
    step.  The planes are row views of a larger NaN-filled buffer, so a read past the last
    token would poison the result."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    try:
        g = torch.Generator(device='cpu').manual_seed(T)
        M, N = 768, 256
        dy = torch.randn(T, M, generator=g).to(dev)
        x = torch.randn(T, N, generator=g).to(dev)

        def nan_tail(p):
            big = torch.full((p.shape[0] + 64, p.shape[1]), float('nan'), device=dev).to(p.dtype)
            big[:p.shape[0]].copy_(p)
            return big[:p.shape[0]]
        dys, xs = nan_tail(sg.grad_planes(dy)), nan_tail(sg.planes(x, sg.ORDER_P[6]))
        po, px = sg._piece_offsets(sg.ORDER_Q[6], M), sg._piece_offsets(sg.ORDER_P[6], N)
        ref = dy.double().t() @ x.double()
        scale = dy.double().abs().t() @ x.double().abs()
        for cfg in ['0:3', '1:2', '2:3', '2:1']:
            monkeypatch.setenv('HX_WGRAD_SPLIT_CFG', cfg)
            outs = {}
            for var in ['2,0', '2,1', '1,0', '1,1', '0,0', '0,1']:
                monkeypatch.setenv('HX_WGRAD_SPLIT_VAR', var)
                slot = torch.empty(M, N, device=dev)
                C().wgrad_split(dys, po, xs, px, 6, M, N, slot)
                torch.cuda.synchronize()
                outs[var] = slot
                assert ((slot.double() - ref).abs() / scale).max().item() < 2e-6, (cfg, var)
            # same token-split plan and summation order: the staging path does not change a bit
            assert torch.equal(outs['0,0'], outs['2,0']) and torch.equal(outs['0,1'], outs['2,1']), cfg
    finally:
        ops.set_fp32_gemm('native')


@pytest.mark.parametrize('cfg,pipe', [(c, '3') for c in range(8)])
def test_piece_gemm_every_cfg(dev, cfg, pipe, monkeypatch):
    """Every tile / pipeline configuration of the LDS-DMA piece GEMM (HX_GEMM_CFG, HX_GEMM_PIPE) in bf16x6: forward and beta = 1
    accumulation against fp64, rows not a multiple of the 256-row tile, a reduction that is not
    a multiple of the 3-stage ring (K = 272: 17 steps of 16)."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    monkeypatch.setenv('HX_GEMM_CFG', str(cfg))
    monkeypatch.setenv('HX_GEMM_PIPE', pipe)
    g = torch.Generator(device='cpu').manual_seed(40 + cfg)
    M, N, K = 531, 768, 272 if cfg != 2 else 288
    a = (torch.rand(M, K, generator=g) * 2 - 1).to(dev)
    W = (torch.rand(N, K, generator=g) * 2 - 1).to(dev)
    c0 = torch.randn(M, N, generator=g).to(dev)
    from hetseq_9cme_amd.ops._ext import C
    try:
        ops.set_fp32_gemm('bf16x6')
        ap = sg.pieces(a)
        wf = sg.pieces(W)   # natural layout (every cfg reads it)
        y = C().gemm_split(ap, wf, 6)
        acc = c0.clone()
        C().gemm_split(ap, wf, 6, acc, True)
        if cfg in (0, 1, 7):   # and the B16 layouts (B operand; both) on the tiles that read them
            wb = wf.view(N, 3, K // 16, 16).permute(0, 2, 1, 3).contiguous().view(N, -1)
            yb = C().gemm_split(ap, wb, 6, None, False, 2)
            assert torch.equal(y, yb)
            ab = ap.view(M, 3, K // 16, 16).permute(0, 2, 1, 3).contiguous().view(M, -1)
            assert torch.equal(y, C().gemm_split(ab, wb, 6, None, False, 3))
    finally:
        ops.set_fp32_gemm('native')
    ref = a.double() @ W.double().t()
    sc = a.double().abs() @ W.double().abs().t()
    assert ((y.double() - ref).abs() / sc).max().item() < 1.5e-6
    e = ((acc.double() - ref - c0.double()).abs() / (sc + c0.double().abs())).max().item()
    assert e < 1.5e-6, e


@pytest.mark.parametrize('mode,cfg,pipe', [('bf16x6', None, None), ('bf16x3', None, None), ('bf16x6', '7', None),
                                           ])
def test_gemm_gelu_epilogues(dev, mode, cfg, pipe, monkeypatch):
    """FFN epilogues of the piece GEMM against fp64: bias + GELU (pre-activation u and the
    pieces of gelu(u)), and the GELU backward (pieces of dh * gelu'(u) and its column sums =
    the FFN-up bias gradient), with rows that are not a multiple of the tile; every tile and
    pipeline that runs them (HX_GEMM_CFG / HX_GEMM_PIPE)."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    if cfg is not None:
        monkeypatch.setenv('HX_GEMM_CFG', cfg)   # e.g. the two-workgroups-per-CU tile
    if pipe is not None:
        monkeypatch.setenv('HX_GEMM_PIPE', pipe)
    g = torch.Generator(device='cpu').manual_seed(31)
    T, H, I = 300, 256, 768
    x = torch.randn(T, H, generator=g).to(dev)
    W1 = (torch.randn(I, H, generator=g) * 0.1).to(dev)
    b1 = (torch.randn(I, generator=g) * 0.5).to(dev)
    W2 = (torch.randn(H, I, generator=g) * 0.05).to(dev)
    dy = torch.randn(T, H, generator=g).to(dev)
    try:
        ops.set_fp32_gemm(mode)
        n = sg.passes()
        xs = sg.pieces(x)
        w1f, _ = sg.weight_pieces(W1)
        u, hp = sg.gemm_gelu(xs, w1f, b1)
        _, w2t = sg.weight_pieces(W2)
        tp, db = sg.gemm_dgelu(sg.pieces(dy), w2t, u, None, None)
        npc = sg.npieces()
    finally:
        ops.set_fp32_gemm('native')
    tol = 2e-6 if mode == 'bf16x6' else 8e-6
    ud = x.double() @ W1.double().t() + b1.double()
    us = x.double().abs() @ W1.double().abs().t() + b1.double().abs()
    assert ((u.double() - ud).abs() / us).max().item() < tol
    h = sum(hp.view(T, npc, I)[:, p].double() for p in range(npc))
    hr = ops.gelu_ref(u.double())
    # fp32 erf-GELU (a few ulp of |u|) + the representation error of the pieces
    assert ((h - hr).abs() / (u.double().abs() + 1e-6)).max().item() < (5e-7 if npc == 3 else 2 ** -15)
    ud_ = u.double().requires_grad_(True)
    ops.gelu_ref(ud_).backward(dy.double() @ W2.double())
    t = sum(tp.view(T, npc, I)[:, p].double() for p in range(npc))
    ts = (dy.double().abs() @ W2.double().abs()) * 1.13   # |gelu'| <= 1.13
    assert ((t - ud_.grad).abs() / (ts + 1e-30)).max().item() < 5 * tol
    dbr = ud_.grad.sum(0)
    assert ((db.double() - dbr).abs() / ts.sum(0)).max().item() < 5 * tol


@pytest.mark.parametrize('cfg', [None, '1'])
def test_gemm_gelu_derivative_mode(dev, cfg, monkeypatch):
    """The FFN path's epilogue pair (deriv=True): the FFN-up GEMM stores gelu'(u) instead of u
    (from the erf it computes for gelu(u) anyway) and the FFN-down data gradient multiplies by it
    with no erf / exp of its own.  Same values bit for bit as the u-storing pair: gelu(u)
    pieces, the dGELU pieces and the bias gradient."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    if cfg is not None:
        monkeypatch.setenv('HX_GEMM_CFG', cfg)
    g = torch.Generator(device='cpu').manual_seed(37)
    T, H, I = 1100, 256, 768
    x = torch.randn(T, H, generator=g).to(dev)
    W1 = (torch.randn(I, H, generator=g) * 0.1).to(dev)
    b1 = (torch.randn(I, generator=g) * 0.5).to(dev)
    W2 = (torch.randn(H, I, generator=g) * 0.05).to(dev)
    dy = torch.randn(T, H, generator=g).to(dev)
    try:
        ops.set_fp32_gemm('bf16x6')
        xs = sg.pieces(x)
        w1f, _ = sg.weight_pieces(W1)
        _, w2t = sg.weight_pieces(W2)
        dys = sg.pieces(dy)
        u, hp = sg.gemm_gelu(xs, w1f, b1)
        gd, hp2 = sg.gemm_gelu(xs, w1f, b1, deriv=True)
        tp, db = sg.gemm_dgelu(dys, w2t, u, None, None)
        tp2, db2 = sg.gemm_dgelu(dys, w2t, gd, None, None, deriv=True)
    finally:
        ops.set_fp32_gemm('native')
    assert torch.equal(hp, hp2)
    assert torch.equal(tp, tp2) and torch.equal(db, db2)
    # gelu'(u) of the reference's GELU (x / 2 (1 + erf(x / 1.41421)))
    ud = u.double()
    ref = 0.5 * (1 + torch.erf(ud / 1.41421)) + ud * torch.exp(-ud * ud / (1.41421 ** 2)) / (1.41421 * 3.141592653589793 ** 0.5)
    assert ((gd.double() - ref).abs()).max().item() < 2e-6


def test_piece_gemm_b16_layouts(dev):
    """B16 operand layouts [rows][K / 16][3][16]: B only (the weights written by split_weight) and
    A and B give the natural layout's product bit for bit; split_weight's B16 outputs equal the
    permuted natural pieces."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(5)
    M, N, K = 512, 768, 256
    a = torch.randn(M, K, generator=g).to(dev)
    W = torch.randn(N, K, generator=g).to(dev)

    def blk(p):
        return p.view(p.shape[0], 3, -1, 16).permute(0, 2, 1, 3).contiguous().view(p.shape[0], -1)
    try:
        ops.set_fp32_gemm('bf16x6')
        ap = sg.pieces(a)
        wf, wt = C().split_weight(W, 3, 0)
        wfb, wtb = C().split_weight(W, 3, 3)
        assert torch.equal(wfb, blk(wf)) and torch.equal(wtb, blk(wt))
        y0 = C().gemm_split(ap, wf, 6)
        y2 = C().gemm_split(ap, wfb, 6, None, False, 2)
        y3 = C().gemm_split(blk(ap), wfb, 6, None, False, 3)
    finally:
        ops.set_fp32_gemm('native')
    assert torch.equal(y0, y2) and torch.equal(y0, y3)


def test_layernorm_writes_consumer_pieces(dev, monkeypatch):
    """LayerNorm / embedding forward write the next piece GEMM's input pieces next to their
    fp32 output (bit-identical to splitting it), and the consuming linear takes them instead
    of a separate split pass (none runs in the layer's forward)."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.models.bert import BertConfig, BertLayer
    from hetseq_9cme_amd.ops import split_gemm
    from hetseq_9cme_amd.ops._ext import C
    ops.set_fp32_gemm('bf16x6')
    try:
        T, H = 300, 768
        y = torch.randn(T, H, device=dev)
        g = torch.rand(H, device=dev) + 0.5
        b = torch.randn(H, device=dev)
        seed = torch.tensor([9], dtype=torch.int64, device=dev)
        out, _, _, _, pcs = C().ln_fwd(y, None, None, g, b, 1e-12, 0.9, seed, 3, False, True, 3)
        ref = split_gemm.pieces(out)
        assert torch.equal(pcs.view(torch.int16), ref.view(torch.int16))
        ids = torch.randint(0, 100, (4, 75), device=dev)
        wte, wpe, wtt = (torch.randn(100, H, device=dev), torch.randn(128, H, device=dev),
                         torch.randn(2, H, device=dev))
        out, _, _, _, pcs = C().embed_ln_fwd(ids, None, wte, wpe, wtt, g, b, 1e-12, 1.0, seed, 0, False, 3)
        assert torch.equal(pcs.view(torch.int16), split_gemm.pieces(out.view(-1, H)).view(torch.int16))
        # in a BERT layer: no split pass in the forward (LN -> FFN-up pieces hand-off)
        torch.manual_seed(0)
        monkeypatch.setattr(split_gemm, 'MIN_ROWS', {3: 0, 6: 0})
        cfg = BertConfig(100, hidden_size=256, num_hidden_layers=1, num_attention_heads=4, intermediate_size=1024)
        layer = BertLayer(cfg).to(dev)
        x = torch.randn(2, 128, 256, device=dev)
        calls = []
        orig = split_gemm.pieces

        def spy(*a, **k):
            calls.append(a[0].shape)
            return orig(*a, **k)
        split_gemm.pieces = spy
        try:
            layer(x, torch.zeros(2, 128, device=dev))
        finally:
            split_gemm.pieces = orig
        # only the layer input is split (no producer here): the attention output and the
        # LayerNorm output come with their pieces
        assert len(calls) == 1, calls
    finally:
        ops.set_fp32_gemm('native')


@pytest.mark.parametrize('pair', ['attn', 'ffn'])
def test_wgrad_split_group_matches_separate(dev, pair):
    """Grouped weight-gradient launch (wgrad_split.hip, hx_wgrad_split_group): the QKV + attention-
    output pair and the FFN W1 + W2 pair in one launch give the same dW as two launches (token
    splits differ, so to fp32 rounding) and both match fp64; T not a multiple of the token block."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(11)
    T = 3000
    shapes = ((768, 256), (256, 256)) if pair == 'attn' else ((1024, 256), (256, 1024))
    try:
        ops.set_fp32_gemm('bf16x6')
        items, refs = [], []
        for M, N in shapes:
            dy = torch.randn(T, M, generator=g).to(dev)
            x = torch.randn(T, N, generator=g).to(dev)
            items.append((sg.pieces(dy), sg.pieces(x), M, N, None))
            refs.append((dy.double().t() @ x.double(), dy.double().abs().t() @ x.double().abs()))
        grouped = sg.wgrad_pieces_group(items)
        assert grouped is not None
        sep = [sg.wgrad_pieces(d, x, M, N, None) for d, x, M, N, _ in items]
    finally:
        ops.set_fp32_gemm('native')
    for got, s, (ref, sc) in zip(grouped, sep, refs):
        assert ((got.double() - ref).abs() / sc).max().item() < 2e-6
        torch.testing.assert_close(got, s, rtol=1e-5, atol=1e-5)


def test_bert_grouped_wgrads_match_ungrouped(dev, monkeypatch):
    """BERT layer (H = 256, so every weight gradient qualifies for the grouped launch) on the
    split path: the attention-output dW deferred into the QKV backward and grouped with it
    (ops.WgradDefer), the FFN's two dW grouped -- every parameter gradient matches the
    one-launch-per-weight run to fp32 rounding."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import fused, split_gemm
    from hetseq_9cme_amd.models.bert import BertConfig, BertForPreTraining
    from hetseq_9cme_amd.parallel.flat_params import FlatParamSpace
    monkeypatch.setitem(split_gemm.MIN_ROWS, 6, 0)
    cfg = BertConfig(1024, hidden_size=256, num_hidden_layers=1, num_attention_heads=4, intermediate_size=1024,
                     max_position_embeddings=128, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    grads = []
    for grouped in (True, False):
        monkeypatch.setattr(split_gemm, '_WGRAD_GROUP', grouped)
        monkeypatch.setattr(fused, '_GROUP_FFN', grouped)
        torch.manual_seed(0)
        model = BertForPreTraining(cfg).to(dev)
        model.max_predictions_per_seq = 4
        flat = FlatParamSpace(model, dev, contiguous_groups=model.flat_contiguous_groups())
        g = torch.Generator(device='cpu').manual_seed(3)
        ids = torch.randint(5, 1024, (16, 128), generator=g).to(dev)
        labels = torch.full_like(ids, -1)
        labels[:, 7] = ids[:, 7]
        nsp = torch.randint(0, 2, (16,), generator=g).to(dev)
        try:
            ops.set_fp32_gemm('bf16x6')
            ops.set_step_seed(1)
            model.train()
            flat.zero_grad()
            loss = model(ids, torch.zeros_like(ids), torch.ones_like(ids), labels, nsp)
            loss.backward()
            flat.adopt_all()
        finally:
            ops.set_fp32_gemm('native')
        grads.append({n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None})
    assert grads[0].keys() == grads[1].keys()
    for n in grads[0]:
        torch.testing.assert_close(grads[0][n], grads[1][n], rtol=1e-4, atol=1e-6, msg=n)


@pytest.mark.parametrize('ks', [0, 2, 3, 5])
def test_piece_gemm_split_k(dev, ks):
    """Split-K slabs of the piece GEMM (gemm_split_k: slab z reduces its share of the k steps
    into its own partial product, summed after) against fp64, for explicit slab counts and the
    planned one (ks = 0), on a narrow output over a deep reduction."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm as sg
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(90 + ks)
    M, N, K = 700, 768, (240 * 16 * ks if ks else 9600)
    a = (torch.rand(M, K, generator=g) * 2 - 1).to(dev)
    W = (torch.rand(N, K, generator=g) * 2 - 1).to(dev)
    try:
        ops.set_fp32_gemm('bf16x6')
        if ks == 0:
            assert C().gemm_split_ks(M, N, K, 6) > 1
        y = C().gemm_split_k(sg.pieces(a), sg.pieces(W), 6, ks, 0)
    finally:
        ops.set_fp32_gemm('native')
    ref = a.double() @ W.double().t()
    sc = a.double().abs() @ W.double().abs().t()
    assert ((y.double() - ref).abs() / sc).max().item() < 1.5e-6


def test_decoder_pieces_path_matches_fp64(dev, monkeypatch):
    """The MLM decoder + softmax-xent on the piece GEMMs (forward over the padded vocabulary,
    split-K data gradient, split-piece weight gradient) against fp64 autograd, and against the
    pass-planes path it replaces (fused._DECODER_PIECES = False)."""
    from hetseq_9cme_amd import ops
    g = torch.Generator(device='cpu').manual_seed(91)
    M, H, V = 512, 768, 9000
    h0 = (torch.randn(M, H, generator=g) * 0.5).to(dev)
    W0 = (torch.randn(V, H, generator=g) * 0.05).to(dev)
    b0 = (torch.randn(V, generator=g) * 0.1).to(dev)
    labels = torch.randint(0, V, (M,), generator=g).to(dev)
    labels[::7] = -1

    def run():
        h = h0.clone().requires_grad_(True)
        W = W0.clone().requires_grad_(True)
        b = b0.clone().requires_grad_(True)
        loss = ops.decoder_xent(h, W, b, labels)
        loss.backward()
        return loss.detach(), h.grad, W.grad, b.grad

    try:
        ops.set_fp32_gemm('bf16x6')
        got = run()
        from hetseq_9cme_amd.ops import fused as _fused
        monkeypatch.setattr(_fused, '_DECODER_PIECES', False)
        old = run()
    finally:
        ops.set_fp32_gemm('native')
    hd, Wd, bd = h0.double().requires_grad_(True), W0.double().requires_grad_(True), b0.double().requires_grad_(True)
    ref_loss = torch.nn.functional.cross_entropy(hd @ Wd.t() + bd, labels, ignore_index=-1)
    ref_loss.backward()
    ref = (ref_loss.detach(), hd.grad, Wd.grad, bd.grad)
    for name, x, o, r in zip(('loss', 'dh', 'dW', 'dbias'), got, old, ref):
        scale = r.abs().max().item()
        err = (x.double() - r).abs().max().item() / scale
        assert err < 2e-6, (name, err)
        err_old = (o.double() - r).abs().max().item() / scale
        assert err_old < 1e-5, (name, 'planes path', err_old)


@pytest.mark.parametrize('npc', [3, 2])
def test_split_weight_many_matches_single(dev, npc):
    """The one-launch batch weight split (split_weight_many: every weight of a forward, 64 x 64
    tiles numbered across the batch) writes the same pieces, in the same layouts, as one
    split_weight launch per weight."""
    from hetseq_9cme_amd.ops._ext import C
    g = torch.Generator(device='cpu').manual_seed(12)
    shapes = [(2304, 768), (768, 768), (3072, 768), (768, 3072), (192, 128)]
    Ws = [torch.randn(n, k, generator=g).to(dev) for n, k in shapes]
    masks = [3, 1, 2, 0, 1] if npc == 3 else [0] * len(shapes)
    outs = C().split_weight_many(Ws, npc, masks)
    for W, m, (wf, wt) in zip(Ws, masks, outs):
        rf, rt = C().split_weight(W, npc, m)
        assert torch.equal(wf, rf) and torch.equal(wt, rt)


def test_bert_batch_weight_split_matches_per_call(dev, monkeypatch):
    """BERT on the piece GEMMs with the encoder's weights split in one launch per forward
    (ops.weight_pieces_scope) gives the same loss and gradients as the per-linear splits."""
    from hetseq_9cme_amd import ops
    from hetseq_9cme_amd.ops import split_gemm
    from hetseq_9cme_amd.models.bert import BertConfig, BertForPreTraining
    from hetseq_9cme_amd.parallel.flat_params import FlatParamSpace
    monkeypatch.setitem(split_gemm.MIN_ROWS, 6, 0)
    cfg = BertConfig(1024, hidden_size=256, num_hidden_layers=2, num_attention_heads=4, intermediate_size=1024,
                     max_position_embeddings=128, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    res = []
    for batch in ('1', '0'):
        from hetseq_9cme_amd.ops import fused as _fused
        monkeypatch.setattr(_fused, '_WSPLIT_BATCH', batch == '1')
        torch.manual_seed(0)
        model = BertForPreTraining(cfg).to(dev)
        model.max_predictions_per_seq = 4
        flat = FlatParamSpace(model, dev, contiguous_groups=model.flat_contiguous_groups())
        g = torch.Generator(device='cpu').manual_seed(3)
        ids = torch.randint(5, 1024, (16, 128), generator=g).to(dev)
        labels = torch.full_like(ids, -1)
        labels[:, 7] = ids[:, 7]
        nsp = torch.randint(0, 2, (16,), generator=g).to(dev)
        try:
            ops.set_fp32_gemm('bf16x6')
            ops.set_step_seed(1)
            model.train()
            flat.zero_grad()
            loss = model(ids, torch.zeros_like(ids), torch.ones_like(ids), labels, nsp)
            loss.backward()
            flat.adopt_all()
        finally:
            ops.set_fp32_gemm('native')
        assert split_gemm._State.wp is None   # scope closed
        res.append((loss.detach().clone(),
                    {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}))
    assert torch.equal(res[0][0], res[1][0])
    for n in res[0][1]:
        torch.testing.assert_close(res[0][1][n], res[1][1][n], rtol=1e-4, atol=1e-6, msg=n)
