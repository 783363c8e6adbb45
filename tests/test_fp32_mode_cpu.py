"""CPU checks of the fp32 GEMM mode (ops/fp32_mode.py, ops/gemm16.py): the fp16x3 split's
numerics (emulated in fp64 on the host: x = 2^-E (h0 + h1), three piece products), the mode
switch and its option, and the dispatch -- every BERT linear of every BASELINE config (phase 1
at 128 and 32 sequences per GPU, phase 2, NER batches, the MLM decoder) takes the ONE
hand-written GEMM family: the host-side plans of gemm_f16.hip return a tile for each shape."""
import math

import pytest
import torch

from hetseq_9cme_amd.ops import fp32_mode, gemm16


def _scale_exp(amax):
    """gemm_f16.hip / hx_gemm.h f16_scale_exp: max |x| lands in [2^14, 2^15) after scaling."""
    if amax == 0 or not math.isfinite(amax):
        return 0
    e = math.frexp(amax)[1]
    return max(-120, min(120, 15 - e))


def _split(x):
    E = _scale_exp(x.abs().max().item())
    y = x.float() * 2.0 ** E
    h0 = y.half()
    h1 = (y - h0.float()).half()
    return E, h0, h1


@pytest.mark.parametrize('scale', [1.0, 1e-8, 1e8, 3e-5])
def test_fp16_pieces_hold_22_bits(scale):
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(1 << 14, generator=g) * scale).float()
    E, h0, h1 = _split(x)
    rec = (h0.double() + h1.double()) * 2.0 ** -E
    amax = x.abs().max().double()
    # RNE pieces: |x - rec| <= 2^-22 max |x| (subnormal tail of h1 included)
    assert ((rec - x.double()).abs() <= 2.0 ** -22 * amax).all()


def test_three_piece_products_match_fp32_class():
    g = torch.Generator().manual_seed(1)
    a = torch.randn(64, 768, generator=g)
    b = torch.randn(96, 768, generator=g) * 0.02
    Ea, a0, a1 = _split(a)
    Eb, b0, b1 = _split(b)
    p = (a0.double() @ b0.double().t() + a0.double() @ b1.double().t() + a1.double() @ b0.double().t())
    p = p * 2.0 ** -(Ea + Eb)
    ref = a.double() @ b.double().t()
    den = a.double().abs() @ b.double().abs().t()
    assert ((p - ref).abs() / den).max().item() < 2e-6   # fp32 MFMA class (2^-22 per operand)


def test_mode_switch_and_option():
    from hetseq_9cme_amd import options
    args = options.parse_training_args(['--task', 'mnist', '--data', '/tmp'])
    assert args.fp32_gemm == 'fp16x3'
    with pytest.raises(SystemExit):
        options.parse_training_args(['--task', 'mnist', '--data', '/tmp', '--fp32-gemm', 'bf16x6'])
    with pytest.raises(ValueError):
        fp32_mode.set_fp32_gemm('tf32')
    prev = fp32_mode.fp32_gemm_mode()
    try:
        fp32_mode.set_fp32_gemm('native')
        assert fp32_mode.fp32_gemm_mode() == 'native' and not gemm16.enabled()
        fp32_mode.set_fp32_gemm('fp16x3')
        assert fp32_mode.fp32_gemm_mode() == 'fp16x3' and gemm16.enabled()
        x = torch.randn(4096, 768)
        assert not gemm16.ok(x, 768)                  # CPU tensors keep the torch reference path
        assert not fp32_mode.attention_split(x)
    finally:
        fp32_mode.set_fp32_gemm(prev)


def test_attention_switch_removed():
    """--fp32-attention is gone (round 5: the x6 attention was deleted; fp32 attention runs on the
    fp16x3 kernels under --fp32-gemm fp16x3, on f32 MFMA under native)."""
    from hetseq_9cme_amd import options
    with pytest.raises(SystemExit):
        options.parse_training_args(['--task', 'mnist', '--data', '/tmp', '--fp32-attention', 'x6'])
    assert not hasattr(fp32_mode, 'set_fp32_attention')


# (tokens, [(n_out, n_in)]) of every BERT-base GEMM the BASELINE configs run
_SHAPES = [(n_out, n_in) for (n_out, n_in) in [(2304, 768), (768, 768), (3072, 768), (768, 3072)]]
_ROWS = {'phase1_b128': 16384, 'phase1_b32': 4096, 'phase2_b32': 16384, 'ner_b32': 32 * 40, 'tiny': 100}


@pytest.mark.parametrize('config', sorted(_ROWS))
def test_dispatch_single_backend(monkeypatch, config):
    """gemm16.ok accepts every encoder linear at every row count (fp32 operands) and the
    kernel's host plan has a tile for its forward, data gradient and weight gradient."""
    from hetseq_9cme_amd.ops._ext import C
    monkeypatch.setattr(gemm16, 'use_kernels', lambda t: True)
    prev = fp32_mode.fp32_gemm_mode()
    try:
        fp32_mode.set_fp32_gemm('fp16x3')
        T = _ROWS[config]
        for (n_out, n_in) in _SHAPES:
            x = torch.empty(T, n_in)
            assert gemm16.ok(x, n_out), (config, n_out, n_in)
            assert C().gemm_f16_plan(T, n_out, n_in) >= 0             # forward
            assert C().gemm_f16_plan(T, n_in, n_out) >= 0             # data gradient
            assert gemm16.wgrad_ok(n_out, n_in)                        # weight gradient
            cfg, ns = C().wgrad_f16_plan(n_out, n_in, T)
            assert cfg in (0, 1) and ns >= 1
        # MLM decoder: vocabulary padded to a multiple of 768, masked rows x H
        Vp = (30522 + 767) // 768 * 768
        assert C().gemm_f16_plan(20 * 128, Vp, 768) >= 0 and C().gemm_f16_plan(20 * 128, 768, Vp) >= 0
        # heads narrower than 64 outputs (NSP, NER labels) stay on the library GEMM
        assert not gemm16.ok(torch.empty(T, 768), 2) and not gemm16.ok(torch.empty(T, 768), 9)
    finally:
        fp32_mode.set_fp32_gemm(prev)


def test_overlap_wgrad_modes():
    """--overlap-wgrad is tri-state: default 'auto' (the side stream from 8192 token rows),
    '--overlap-wgrad' = on, '--no-overlap-wgrad' = off; CPU tensors never get a side stream."""
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
            assert fused.side_begin(torch.device('cpu'), 16384) is None
        with pytest.raises(AssertionError):
            fused.set_side_stream('sometimes')
    finally:
        fused._Side.mode = prev


def test_graph_train_step_modes():
    """--graph-train-step is tri-state: default 'auto' = on for GPU token-classification
    fine-tuning only; explicit on / off win; --cpu never captures."""
    from types import SimpleNamespace as NS
    from hetseq_9cme_amd import options
    on = options.graph_train_step_enabled
    assert on(NS(graph_train_step='auto', task='BertForTokenClassification', cpu=False))
    assert not on(NS(graph_train_step='auto', task='BertForTokenClassification', cpu=True))
    assert not on(NS(graph_train_step='auto', task='bert', cpu=False))
    assert on(NS(graph_train_step='on', task='bert', cpu=False))
    assert not on(NS(graph_train_step='off', task='BertForTokenClassification', cpu=False))
    base = ['--task', 'mnist', '--data', '/tmp']
    assert options.parse_training_args(base).graph_train_step == 'auto'
    assert options.parse_training_args(base + ['--graph-train-step']).graph_train_step == 'on'
    assert options.parse_training_args(base + ['--no-graph-train-step']).graph_train_step == 'off'
