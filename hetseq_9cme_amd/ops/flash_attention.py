"""Scaled-dot-product attention over the packed QKV projection.

Reference math (hetseq/bert_modeling.py:351-377): scores = Q K^T / sqrt(d) +
mask_bias; probs = dropout(softmax(scores)); ctx = probs V; heads merged back
to [B, S, H].  The additive mask is the reference's (1 - m) * -10000 (not -inf).

GPU path: the fused flash-style HIP kernel (``_C.attn_fwd`` / ``attn_bwd``,
csrc/kernels/attention.hip) for head_dim 64 at any sequence length (keys past
S are masked, rows past S are neither computed into nor stored), with fp32 or
bf16 activations (bf16 is converted at load; the math is fp32 MFMA either way);
other shapes / dtypes use the composite below (batched GEMMs + softmax), which
is also the CPU path and the test oracle.
"""
import math

import torch
import torch.nn.functional as F

from ._ext import C, use_kernels
from .rng import get_rng


def attention_ref(qkv, mask_bias, num_heads, p, generator_dropout=True):
    B, S, H3 = qkv.shape
    H = H3 // 3
    d = H // num_heads
    x = qkv.view(B, S, 3, num_heads, d).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    scores = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(d)
    scores = scores + mask_bias.to(scores.dtype)[:, None, None, :]
    probs = torch.softmax(scores.float(), dim=-1).to(qkv.dtype)
    if p > 0:
        probs = F.dropout(probs, p, True)
    ctx = torch.matmul(probs, v)
    return ctx.permute(0, 2, 1, 3).reshape(B, S, H)


def _fused_ok(qkv, num_heads):
    if not use_kernels(qkv):
        return False
    try:
        ext = C()
    except RuntimeError:
        return False
    if not hasattr(ext, 'attn_fwd'):
        return False
    B, S, H3 = qkv.shape
    d = (H3 // 3) // num_heads
    return qkv.dtype in (torch.float32, torch.bfloat16) and d == 64 and S >= 1


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, mask_bias, num_heads, p):
        keep = 1.0 - p
        seed, stream = get_rng().next() if p > 0 else (0, 0)
        out, lse, dmask = C().attn_fwd(qkv, mask_bias, num_heads, keep, seed, stream)
        ctx.save_for_backward(qkv, mask_bias, out, lse, dmask)
        ctx.meta = (num_heads, keep)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, mask_bias, out, lse, dmask = ctx.saved_tensors
        num_heads, keep = ctx.meta
        dqkv = C().attn_bwd(dout.contiguous(), qkv, mask_bias, out, lse, dmask, num_heads, keep)
        return dqkv, None, None, None


def attention(qkv, mask_bias, num_heads, p):
    if _fused_ok(qkv, num_heads):
        return _AttnFn.apply(qkv.contiguous(), mask_bias.float().contiguous(), int(num_heads), float(p))
    return attention_ref(qkv, mask_bias, num_heads, p)
