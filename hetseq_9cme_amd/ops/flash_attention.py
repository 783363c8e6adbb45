"""Scaled-dot-product attention over the packed QKV projection.

Reference math (hetseq/bert_modeling.py:351-377): scores = Q K^T / sqrt(d) +
mask_bias; probs = dropout(softmax(scores)); ctx = probs V; heads merged back
to [B, S, H].  The additive mask is the reference's (1 - m) * -10000 (not -inf).

GPU path: the fused flash-style HIP kernel (``_C.attn_fwd`` / ``attn_bwd``,
csrc/kernels/attention.hip) for head_dim 64 at any sequence length (keys past
S are masked, rows past S are neither computed into nor stored), with fp32 or
bf16 activations (bf16 activations: bf16 MFMA, attention_bf16.hip; fp32 activations under
``--fp32-gemm fp16x3``: the products as three fp16 passes over scaled two-piece operands,
attention_f16.hip; fp32 MFMA under ``--fp32-gemm native``, attention.hip);
other shapes / dtypes use the composite below (batched GEMMs + softmax), which
is also the CPU path and the test oracle.
"""
import math

import torch
import torch.nn.functional as F

from . import fp32_mode, gemm16
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


def _bias3(bq, bk, bv):
    """[3H] view over the adjacent Q/K/V bias storage (FlatParamSpace keeps them
    back to back), or a concatenated copy."""
    from .fused import _adjacent_view
    v = _adjacent_view([bq, bk, bv])
    return v if v is not None else torch.cat([bq, bk, bv], 0)


class _AttnFn(torch.autograd.Function):
    """Fused attention; with ``bq/bk/bv`` the QKV-projection bias's gradient -- the column
    sums of dQ/dK/dV -- comes out of the backward kernel's registers, straight into the flat
    gradient slots, instead of a separate pass over the [B*S, 3H] gradient.  ``add``: the
    kernels also add the bias to Q/K/V as they load them (a bias-less projection); else it is
    already in qkv (the projection GEMM's epilogue, the default)."""

    @staticmethod
    def forward(ctx, qkv, mask_bias, bq, bk, bv, num_heads, p, add=True):
        from .fused import grad_slot  # noqa: F401  (import cycle guard)
        keep = 1.0 - p
        seed, stream = get_rng().next(qkv.device) if p > 0 else (get_rng().seed_tensor(qkv.device), 0)
        # add: the bias is added here; else it is already in qkv (the projection's epilogue) and
        # only its gradient comes out of the backward
        bias = _bias3(bq, bk, bv).float().contiguous() if bq is not None and add else None
        ctx.want_db = bq is not None
        # fp32 under fp16x3: the fp16x3 piece kernels (fp32_mode.attention_split), which also write
        # the context's max |x| per (row, head) -- the attention-output GEMM's per-row scale
        ctx.split = qkv.dtype == torch.float32 and fp32_mode.attention_split(qkv.reshape(-1, qkv.shape[-1]))
        if ctx.split:
            B, S, H = qkv.shape[0], qkv.shape[1], qkv.shape[2] // 3
            am = torch.empty(B * S, num_heads, dtype=torch.float32, device=qkv.device)
            cm = torch.empty(B * ((S + 127) // 128), H, dtype=torch.float32, device=qkv.device)
            out, lse, dmask = C().attn_fwd_f16(qkv, mask_bias, num_heads, keep, seed, stream, bias, am, cm)
            # per-row (output projection) and per-column (its weight gradient) max |context|
            gemm16.attach_cols(gemm16.attach(out, am), gemm16.fit_cols(cm))
        else:
            out, lse, dmask = C().attn_fwd(qkv, mask_bias, num_heads, keep, seed, stream, bias)
        ctx.save_for_backward(qkv, mask_bias, out, lse, dmask)
        ctx.bias = bias
        ctx.bparams = (bq, bk, bv)
        ctx.meta = (num_heads, keep)
        return out

    @staticmethod
    def backward(ctx, dout):
        from .fused import grad_slot
        qkv, mask_bias, out, lse, dmask = ctx.saved_tensors
        num_heads, keep = ctx.meta
        bq, bk, bv = ctx.bparams
        slots = [None, None, None]
        if ctx.want_db:
            slots = [grad_slot(t) for t in (bq, bk, bv)]
            if not all(t is not None for t in slots):
                slots = [None, None, None]
        if ctx.split:
            # the kernel writes max |dQKV| per (row, head) -- the QKV projection's per-row operand
            # scale -- and per (batch, key block, column) -- its weight gradient's column scale.
            # Several key blocks (S > 128): dK / dV only; dQ (summed by atomics over the blocks)
            # gets its row and column maxima from one pass over the dQ third
            B, S, H3 = qkv.shape
            kb = (S + 127) // 128
            am = torch.empty(B * S, num_heads, dtype=torch.float32, device=qkv.device)
            cm = torch.empty(B * kb, H3, dtype=torch.float32, device=qkv.device)
            dqkv, dbias = C().attn_bwd_f16(dout.contiguous(), qkv, mask_bias, out, lse, dmask, num_heads, keep,
                                           ctx.bias, *slots, am, cm, want_dbias=ctx.want_db)
            if kb > 1:
                rq, cq = C().amax_rows_cols(dqkv.view(B * S, H3)[:, :H3 // 3])
                am = torch.cat([am, rq], 1)
                q = torch.zeros(1, H3, dtype=torch.float32, device=qkv.device)
                q[:, :H3 // 3] = cq
                cm = torch.cat([q, cm], 0)
            # per-row (QKV data gradient) and per-column (QKV weight gradient) max |dQKV|; more
            # than 256 column partials (B * key blocks) are folded to one row (same maxima)
            gemm16.attach_cols(gemm16.attach(dqkv, am), gemm16.fit_cols(cm))
        else:
            dqkv, dbias = C().attn_bwd(dout.contiguous(), qkv, mask_bias, out, lse, dmask, num_heads, keep, ctx.bias,
                                       *slots, want_dbias=ctx.want_db)
        if not ctx.want_db:
            return dqkv, None, None, None, None, None, None, None
        if slots[0] is not None:
            db = slots
        else:
            H = dbias.numel() // 3
            db = [dbias[:H].view_as(bq), dbias[H:2 * H].view_as(bk), dbias[2 * H:].view_as(bv)]
        return dqkv, None, db[0], db[1], db[2], None, None, None


class _BiasGradTap(torch.autograd.Function):
    """Identity on qkv whose backward also returns the column sums of dqkv as the gradients of the
    (bq, bk, bv) already added into it (the composite path of ``attention(bias_grad=...)``)."""

    @staticmethod
    def forward(ctx, qkv, bq, bk, bv):
        ctx.n = (bq.numel(), bk.numel())
        return qkv.view_as(qkv)

    @staticmethod
    def backward(ctx, dqkv):
        a, b = ctx.n
        low = dqkv.dtype in (torch.float16, torch.bfloat16)
        db = dqkv.reshape(-1, dqkv.shape[-1]).sum(0, dtype=torch.float32 if low else dqkv.dtype)
        return dqkv, db[:a], db[a:a + b], db[a + b:]


def attention(qkv, mask_bias, num_heads, p, bias=None, bias_grad=None):
    """``bias``: optional (bq, bk, bv) of the QKV projection, applied here; ``bias_grad``: the
    (bq, bk, bv) already added into qkv by the projection GEMM's epilogue -- only their gradient
    (the column sums of dQKV) is produced here, by the backward kernel."""
    if _fused_ok(qkv, num_heads):
        if bias_grad is not None:
            bq, bk, bv = bias_grad
            return _AttnFn.apply(qkv.contiguous(), mask_bias.float().contiguous(), bq, bk, bv, int(num_heads),
                                 float(p), False)
        bq, bk, bv = bias if bias is not None else (None, None, None)
        return _AttnFn.apply(qkv.contiguous(), mask_bias.float().contiguous(), bq, bk, bv, int(num_heads), float(p))
    if bias_grad is not None:
        qkv = _BiasGradTap.apply(qkv, *bias_grad)
    if bias is not None:
        qkv = qkv + torch.cat(list(bias), 0).to(qkv.dtype)
    return attention_ref(qkv, mask_bias, num_heads, p)
