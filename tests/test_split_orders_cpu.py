"""CPU checks of the split-GEMM pass structure (ops/split_gemm.py): the plane orders make
the forward, data-gradient and weight-gradient GEMMs each pair exactly the intended piece
products (emulated here in fp64 on CPU, where every bf16 product is exact), and the
pieces reconstruct fp32 values to the stated bounds."""
import os

import pytest
import torch

from hetseq_9cme_amd.ops import split_gemm as sg

PAIRS = {3: {(0, 0), (1, 0), (0, 1)}, 6: {(0, 0), (1, 0), (0, 1), (2, 0), (1, 1), (0, 2)}}


def _pieces(x, n):
    out, r = [], x.clone()
    for _ in range(n):
        p = r.to(torch.bfloat16)
        out.append(p.double())
        r = r - p.float()
    return out


def _stack_cols(p, order):          # [R, n*D] interleaved along the reduction (column) dim
    return torch.cat([p[k] for k in order], 1)


def _stack_rows(p, order):          # [n*R, D] stacked
    return torch.cat([p[k] for k in order], 0)


@pytest.mark.parametrize('passes', [3, 6])
def test_plane_orders_pair_the_right_pieces(passes):
    g = torch.Generator().manual_seed(0)
    T, K, N = 7, 16, 5
    x, W, dy = torch.randn(T, K, generator=g), torch.randn(N, K, generator=g), torch.randn(T, N, generator=g)
    n = sg.PIECES[passes]
    px, pw, pd = _pieces(x, n), _pieces(W, n), _pieces(dy, n)
    P, Q = sg.ORDER_P[passes], sg.ORDER_Q[passes]
    # forward y = x' . W_Q'^T
    y = _stack_cols(px, P) @ _stack_cols(pw, Q).t()
    want = sum(px[a] @ pw[b].t() for a, b in PAIRS[passes])
    assert torch.allclose(y, want, rtol=0, atol=1e-12)
    # data gradient dx = dy' [T, nN] . W_P'' [nN, K]
    dx = _stack_cols(pd, Q) @ _stack_rows(pw, P)
    want = sum(pd[a] @ pw[b] for a, b in PAIRS[passes])
    assert torch.allclose(dx, want, rtol=0, atol=1e-12)
    # weight gradient over the [T, n, D] -> [nT, D] views
    dys = torch.stack([pd[k] for k in Q], 1).reshape(-1, N)
    xs = torch.stack([px[k] for k in P], 1).reshape(-1, K)
    dW = dys.t() @ xs
    want = sum(pd[a].t() @ px[b] for a, b in PAIRS[passes])
    assert torch.allclose(dW, want, rtol=0, atol=1e-12)
    # and the piece offsets the split-piece wgrad kernel reads from those layouts
    assert [Q[o // N] for o in sg._piece_offsets(Q, N)] == list(range(n))
    assert [P[o // K] for o in sg._piece_offsets(P, K)] == list(range(n))


@pytest.mark.parametrize('passes,bound', [(3, 2.0 ** -16), (6, 2.0 ** -25)])
def test_pieces_reconstruct(passes, bound):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(4096, generator=g) * torch.logspace(-8, 8, 4096)
    s = sum(_pieces(x, sg.PIECES[passes]))
    assert ((s - x.double()).abs() <= bound * x.double().abs()).all()


def test_mode_switch_and_cpu_inactive():
    with pytest.raises(ValueError):
        sg.set_fp32_gemm('tf32')
    try:
        sg.set_fp32_gemm('bf16x6')
        assert sg.fp32_gemm_mode() == 'bf16x6' and sg.passes() == 6
        assert not sg.active(torch.randn(16384, 8))      # CPU tensors keep the torch reference path
    finally:
        sg.set_fp32_gemm('native')


def test_option_default_is_fp16x3():
    from hetseq_9cme_amd import options
    args = options.parse_training_args(['--task', 'mnist', '--data', '/tmp'])
    assert args.fp32_gemm == 'fp16x3'


def test_dispatch_plans(monkeypatch):
    """Which product form each BERT-base GEMM takes (pure host logic of ops/split_gemm.py):
    split path from 4096 tokens per GEMM under bf16x6 (the 32 x 128-token batch), split-K
    only for the MLM decoder's data gradient, prefix form only for the deep narrow products."""
    if 'HETSEQ_SPLIT_MIN_ROWS_X6' not in os.environ:
        assert sg.MIN_ROWS[6] == 4096
    # decoder dgrad: 2560 masked rows x 768 from K' = 6 x 30720 -> 16 reduction slabs
    assert sg._splitk(2560, 768, 6 * 30720) == 16
    # encoder products fill the chip without it
    for (m, n, k) in [(16384, 768, 6 * 768), (16384, 3072, 6 * 768), (16384, 768, 6 * 2304)]:
        assert sg._splitk(m, n, k) == 1
    try:
        sg.set_fp32_gemm('bf16x6')
        assert sg.prefix_ok(3072, 768)          # FFN-down forward / FFN-up data gradient
        assert not sg.prefix_ok(768, 2304)      # QKV forward: k < 2 n
        assert not sg.prefix_ok(768, 768)
        monkeypatch.setattr(sg, '_PREFIX_GEMM', False)
        assert not sg.prefix_ok(3072, 768)
        monkeypatch.setattr(sg, '_PREFIX_GEMM', True)
    finally:
        sg.set_fp32_gemm('native')
    assert not sg.prefix_ok(3072, 768)          # native mode: no split products at all


def test_piece_gemm_row_threshold(monkeypatch):
    """The piece GEMMs take a linear only from PIECE_MIN_ROWS tokens (8192: below it the
    256-row tiles leave CUs idle and the planes path on the library GEMMs is faster); an
    explicit HETSEQ_PIECE_GEMM=1 (piece_gemm True) overrides the threshold."""
    monkeypatch.delenv('HX_PIECE_MIN_ROWS', raising=False)
    monkeypatch.setattr(sg._State, 'piece_gemm', None)
    try:
        sg.set_fp32_gemm('bf16x6')
        assert sg.PIECE_MIN_ROWS == 8192 or 'HX_PIECE_MIN_ROWS' in os.environ
        assert not sg.nt_ok(768, 768, sg.PIECE_MIN_ROWS - 1)
        assert sg.nt_ok(768, 768, sg.PIECE_MIN_ROWS) and sg.nt_ok(768, 3072, 16384)
        assert sg.nt_ok(768, 768)                       # no row count: shape rule only
        assert not sg.nt_ok(768, 100, 16384)            # 128-multiple shapes only
        monkeypatch.setattr(sg._State, 'piece_gemm', True)
        assert sg.nt_ok(768, 768, 1024)
        sg.set_fp32_gemm('bf16x3')
        monkeypatch.setattr(sg._State, 'piece_gemm', None)
        assert not sg.nt_ok(768, 768, 16384)            # bf16x3: opt-in only
    finally:
        sg.set_fp32_gemm('native')


def test_overlap_wgrad_modes():
    """--overlap-wgrad is tri-state: default 'auto' (side stream on the piece-GEMM backward
    paths only), '--overlap-wgrad' = every path, '--no-overlap-wgrad' = none; CPU tensors never
    get a side stream."""
    from hetseq_9cme_amd import options
    from hetseq_9cme_amd.ops import fused
    base = ['--task', 'mnist', '--data', '/tmp']
    assert options.parse_training_args(base).overlap_wgrad == 'auto'
    assert options.parse_training_args(base + ['--overlap-wgrad']).overlap_wgrad == 'on'
    assert options.parse_training_args(base + ['--no-overlap-wgrad']).overlap_wgrad == 'off'
    prev = fused._Side.mode
    try:
        for flag, mode in ((True, 'on'), (False, 'off'), ('auto', 'auto'), ('on', 'on')):
            fused.set_side_stream(flag)
            assert fused._Side.mode == mode
            assert fused.side_begin(torch.device('cpu'), True) is None
        with pytest.raises(AssertionError):
            fused.set_side_stream('sometimes')
    finally:
        fused._Side.mode = prev
