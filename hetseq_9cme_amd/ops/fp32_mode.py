"""How fp32 runs (``--precision fp32``, the reference's precision) use the matrix cores
(``--fp32-gemm``).

gfx950 has no TF32/xf32; its f32-input MFMA runs at the f32 vector rate, 157 TF/s, 1/16 of the
fp16/bf16 MFMA rate.  Two modes:

* ``fp16x3`` (default): every linear-layer GEMM -- forward, data gradient, weight gradient, the
  MLM decoder included -- on the hand-written fp16x3 kernels (ops/gemm16.py,
  csrc/kernels/gemm_f16.hip): operands scaled by a power of two from their max |x| and split
  into two fp16 pieces (22 significant bits), three exact piece products per GEMM.  Measured
  GEMM error vs fp64 0.6-0.7x that of native f32 MFMA (tests/test_gemm_f16_gpu.py).  The
  attention products run as three fp16 passes over scaled two-piece operands (attention_f16.hip)
  at every batch size.
* ``native``: f32 MFMA everywhere (library GEMMs, attention.hip) -- bitwise the reference's fp32
  FMA chain class; the numerics oracle of the parity runs (tools/parity_run.py).
"""
import torch

from ._ext import use_kernels

MODES = ('native', 'fp16x3')


def set_fp32_gemm(mode):
    """``'fp16x3'`` or ``'native'``."""
    from . import gemm16
    if mode not in MODES:
        raise ValueError('--fp32-gemm must be one of {}'.format(list(MODES)))
    gemm16.set_enabled(mode == 'fp16x3')


def fp32_gemm_mode():
    from . import gemm16
    return 'fp16x3' if gemm16.enabled() else 'native'


def attention_split(x2):
    """Does the fp32 attention over the [rows, 3H] projection ``x2`` run its products on the fp16x3
    piece kernels (attention_f16.hip, at any size -- faster than the f32-MFMA kernel from
    fine-tuning batches up, tools/probe/attn_bwd_probe.py)?"""
    from . import gemm16
    return gemm16.enabled() and x2.dtype == torch.float32 and use_kernels(x2) and x2.numel() > 0
