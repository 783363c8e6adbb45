"""How fp32 runs (``--precision fp32``, the reference's precision) use the matrix cores
(``--fp32-gemm``).

gfx950 has no TF32/xf32; its f32-input MFMA runs at the f32 vector rate, 157 TF/s, 1/16 of the
fp16/bf16 MFMA rate.  Two modes:

* ``fp16x3`` (default): every linear-layer GEMM -- forward, data gradient, weight gradient, the
  MLM decoder included -- on the hand-written fp16x3 kernels (ops/gemm16.py,
  csrc/kernels/gemm_f16.hip): operands scaled by a power of two from their max |x| and split
  into two fp16 pieces (22 significant bits), three exact piece products per GEMM.  Measured
  GEMM error vs fp64 0.6-0.7x that of native f32 MFMA (tests/test_gemm_f16_gpu.py).  The
  attention products run as three fp16 passes (attention_f16.hip; or, with ``--fp32-attention
  x6``, six bf16 piece passes, attention_x6.hip) from ``ATTN_X6_MIN_ROWS`` token rows, f32 MFMA
  below.
* ``native``: f32 MFMA everywhere (library GEMMs, attention.hip) -- bitwise the reference's fp32
  FMA chain class; the numerics oracle of the parity runs (tools/parity_run.py).
"""
import torch

from ._ext import use_kernels

MODES = ('native', 'fp16x3')
ATTN_MODES = ('x6', 'fp16x3')

# Token rows from which the x6 attention (attention_x6.hip) runs the fp32 attention: at 4096 rows
# (BERT-base 32 x 128) and above it wins; NER fine-tuning batches (~1000 rows) keep the f32-MFMA
# kernel under x6 (rounds 2-3 measurements).  The fp16x3 kernels run at every size.
ATTN_X6_MIN_ROWS = 4096


def set_fp32_gemm(mode):
    """``'fp16x3'`` or ``'native'``."""
    from . import gemm16
    if mode not in MODES:
        raise ValueError('--fp32-gemm must be one of {}'.format(list(MODES)))
    gemm16.set_enabled(mode == 'fp16x3')


class _Attn(object):
    kernel = 'fp16x3'


def set_fp32_attention(mode):
    """``--fp32-attention``: the kernels of the fp32 attention products under fp16x3 GEMMs, from
    ``ATTN_X6_MIN_ROWS`` rows: ``'fp16x3'`` (default; three fp16 passes over scaled two-piece
    operands, attention_f16.hip -- the backward 21-25 % faster than x6 at two waves per SIMD,
    profiles/r4_attention_bwd_pmc.md; per-tile / per-wave power-of-two scales, so a dQ / dK row more
    than 2^40 below its tile's largest dS is flushed, the fp16x3 GEMMs' per-tensor floor) or
    ``'x6'`` (six bf16 piece passes, attention_x6.hip: bf16's exponent range, every row fp32
    class whatever its magnitude)."""
    if mode not in ATTN_MODES:
        raise ValueError('--fp32-attention must be one of {}'.format(list(ATTN_MODES)))
    _Attn.kernel = mode


def fp32_attention_mode():
    return _Attn.kernel


def fp32_gemm_mode():
    from . import gemm16
    return 'fp16x3' if gemm16.enabled() else 'native'


def attention_split(x2):
    """Does the fp32 attention over the [rows, 3H] projection ``x2`` run its products on the piece
    kernels (attention_f16.hip at any size -- faster than the f32-MFMA kernel from fine-tuning
    batches up, tools/probe/attn_bwd_probe.py; attention_x6.hip from ``ATTN_X6_MIN_ROWS`` rows)?"""
    from . import gemm16
    rows = x2.numel() // max(1, x2.shape[-1])
    min_rows = ATTN_X6_MIN_ROWS if _Attn.kernel == 'x6' else 1
    return gemm16.enabled() and x2.dtype == torch.float32 and use_kernels(x2) and rows >= min_rows
