"""MI355X (gfx950) compute ops.

Public functional API used by the models and the engine.  Each op runs a
hand-written HIP kernel for GPU tensors and a torch reference for CPU tensors.
"""
from ._ext import C, use_kernels, set_fused, fused_enabled  # noqa: F401
from .rng import get_rng, set_step_seed  # noqa: F401
from .fp32_mode import set_fp32_gemm, fp32_gemm_mode  # noqa: F401
from .fused import (  # noqa: F401
    embed_ln, bias_dropout_residual_ln, layer_norm, bias_act, dropout, linear3, attention,
    decoder_xent, masked_rows, gelu_ref, layer_norm_ref, linear, grad_slot, ResidualGrad,
    set_side_stream, active_side_stream, side_join, ffn, ffn_fusable, qkv_weight_view, weight_pieces_scope,
)


def flat_grad_norm_clip(grad_flat, gscale, out_norm, clipped, max_norm):
    """One reduction over the flat grad buffer: norm = ||g|| * |gscale|; clip
    coefficient folded into ``gscale`` on device."""
    C().grad_norm_clip(grad_flat, gscale, out_norm, clipped, float(max_norm))


def fused_adam(p, g, m, v, gscale, start, end, beta1, beta2, eps, step_size, wd_lr, bf16_shadow=None, hp=None):
    """``hp``: optional device [2] (step size, wd * lr) that overrides the host values."""
    C().adam(p, g, m, v, bf16_shadow, gscale, int(start), int(end), beta1, beta2, eps, step_size, wd_lr, hp)


def fused_adadelta(p, g, sq, acc, gscale, start, end, lr, rho, eps, wd, hp=None):
    C().adadelta(p, g, sq, acc, gscale, int(start), int(end), lr, rho, eps, wd, hp)


def set_reserved_cus(n):
    """CUs the one-round GEMM / weight-gradient plans leave to a concurrent comm kernel
    (csrc/kernels/cu_reserve.hip; ``--comm-cus``).  0 = plan for the whole chip."""
    C().set_reserved_cus(int(n))
