"""Autograd wrappers around the gfx950 kernels + torch reference implementations.

Every public op dispatches on the device of its input: GPU tensors run the
hand-written HIP kernels (``_C``), CPU tensors run the plain-torch reference of
the same math (used by the CPU test-suite and as the numerics oracle for the GPU
kernel tests).  Semantics follow the reference model (hetseq/bert_modeling.py).
"""
import math

import torch
import torch.nn.functional as F

from ._ext import C, use_kernels
from .rng import get_rng

ACT_IDS = {'gelu': 0, 'tanh': 1, 'relu': 2, 'none': 3}


def _is_bf16(t):
    return t.dtype == torch.bfloat16


# ----------------------------------------------------------------- references
def gelu_ref(x):
    return x * 0.5 * (1.0 + torch.erf(x / 1.41421))


def _act_ref(x, act):
    if act == 'gelu':
        return gelu_ref(x)
    if act == 'tanh':
        return torch.tanh(x)
    if act == 'relu':
        return F.relu(x)
    return x


def layer_norm_ref(x, w, b, eps):
    u = x.mean(-1, keepdim=True)
    s = (x - u).pow(2).mean(-1, keepdim=True)
    x = (x - u) / torch.sqrt(s + eps)
    return w * x + b


# ----------------------------------------------------------------- embedding
class _EmbedLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, tt, wte, wpe, wtt, gamma, beta, eps, p, out_bf16):
        keep = 1.0 - p
        seed, stream = get_rng().next() if p > 0 else (0, 0)
        out, z, mean, rstd = C().embed_ln_fwd(ids, tt, wte, wpe, wtt, gamma, beta, eps, keep, seed, stream,
                                              out_bf16)
        ctx.save_for_backward(ids, tt if tt is not None else torch.Tensor(), z, mean, rstd, gamma)
        ctx.has_tt = tt is not None
        ctx.meta = (keep, seed, stream, wte.shape[0], wpe.shape[0], wtt.shape[0])
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, tt, z, mean, rstd, gamma = ctx.saved_tensors
        keep, seed, stream, V, P, NT = ctx.meta
        dout = dout.contiguous()
        dz, _, dgamma, dbeta, _ = C().ln_bwd(dout, z, mean, rstd, gamma, keep, seed, stream, True, False, False)
        dwte, dwpe, dwtt = C().embed_grads(dz, ids, tt if ctx.has_tt else None, V, P, NT)
        return None, None, dwte, dwpe, dwtt, dgamma, dbeta, None, None, None


def embed_ln(ids, tt, wte, wpe, wtt, gamma, beta, eps, p, training, out_dtype=torch.float32):
    """dropout(LN(word[ids] + pos[arange(S)] + type[tt]))  -> [B, S, H]"""
    p = p if training else 0.0
    if use_kernels(ids):
        return _EmbedLNFn.apply(ids.contiguous(), None if tt is None else tt.contiguous(), wte, wpe, wtt, gamma,
                                beta, float(eps), float(p), out_dtype == torch.bfloat16)
    S = ids.shape[1]
    pos = torch.arange(S, device=ids.device).unsqueeze(0).expand_as(ids)
    if tt is None:
        tt = torch.zeros_like(ids)
    z = F.embedding(ids, wte) + F.embedding(pos, wpe) + F.embedding(tt, wtt)
    out = layer_norm_ref(z, gamma, beta, eps)
    return F.dropout(out, p, training).to(out_dtype)


# ----------------------------------------------------------------- bias + dropout + residual + LN
class _BiasDropResLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias, res, gamma, beta, eps, p):
        keep = 1.0 - p
        seed, stream = get_rng().next() if p > 0 else (0, 0)
        out, z, mean, rstd = C().ln_fwd(y, bias, res, gamma, beta, eps, keep, seed, stream, False, True)
        ctx.save_for_backward(z, mean, rstd, gamma)
        ctx.meta = (keep, seed, stream, bias is not None, res is not None, y.numel() != z.numel())
        return out

    @staticmethod
    def backward(ctx, dout):
        z, mean, rstd, gamma = ctx.saved_tensors
        keep, seed, stream, has_bias, has_res, _ = ctx.meta
        need_dy = has_bias or keep < 1.0
        dz, dy, dgamma, dbeta, dbias = C().ln_bwd(dout.contiguous(), z, mean, rstd, gamma, keep, seed, stream,
                                                  False, need_dy, has_bias)
        dy_ret = dy if need_dy else dz
        return dy_ret, (dbias if has_bias else None), (dz if has_res else None), dgamma, dbeta, None, None


def bias_dropout_residual_ln(y, bias, res, gamma, beta, eps, p, training):
    """LN(dropout(y + bias) + res)  (BertSelfOutput / BertOutput, bert_modeling.py:387-391)."""
    p = p if training else 0.0
    if use_kernels(y):
        return _BiasDropResLNFn.apply(y.contiguous(), bias, None if res is None else res.contiguous(), gamma, beta,
                                      float(eps), float(p))
    x = y if bias is None else y + bias
    x = F.dropout(x, p, training)
    if res is not None:
        x = x + res
    return layer_norm_ref(x, gamma, beta, eps)


def layer_norm(x, gamma, beta, eps):
    return bias_dropout_residual_ln(x, None, None, gamma, beta, eps, 0.0, False)


# ----------------------------------------------------------------- bias + activation
class _BiasActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias, act):
        aid = ACT_IDS[act]
        out = C().bias_act_fwd(y, bias, aid)
        if act == 'gelu':
            ctx.save_for_backward(y, bias if bias is not None else torch.Tensor())
        else:
            ctx.save_for_backward(out, torch.Tensor())
        ctx.meta = (aid, bias is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        a, b = ctx.saved_tensors
        aid, has_bias = ctx.meta
        if aid == 0:
            dy, dbias = C().bias_act_bwd(dout.contiguous(), a, b if has_bias else None, None, aid, has_bias)
        else:
            dy, dbias = C().bias_act_bwd(dout.contiguous(), None, None, a, aid, has_bias)
        return dy, (dbias if has_bias else None), None


def bias_act(y, bias, act):
    """act(y + bias) -- LinearActivation's fused bias_gelu / bias_tanh (bert_modeling.py:104-116)."""
    if use_kernels(y) and y.shape[-1] % 4 == 0:
        return _BiasActFn.apply(y.contiguous(), bias, act)
    x = y if bias is None else y + bias
    return _act_ref(x, act)


# ----------------------------------------------------------------- dropout
class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        keep = 1.0 - p
        seed, stream = get_rng().next()
        ctx.meta = (keep, seed, stream)
        return C().dropout(x, keep, seed, stream)

    @staticmethod
    def backward(ctx, dout):
        keep, seed, stream = ctx.meta
        return C().dropout(dout.contiguous(), keep, seed, stream), None


def dropout(x, p, training):
    if not training or p == 0.0:
        return x
    if use_kernels(x):
        return _DropoutFn.apply(x.contiguous(), float(p))
    return F.dropout(x, p, True)


# ----------------------------------------------------------------- fused Q/K/V projection
def _adjacent_view(ts):
    """If tensors ``ts`` are laid out back to back in one storage (FlatParamSpace
    guarantees it for Q/K/V), return a single [sum(rows), cols] view without copying."""
    t0 = ts[0]
    es = t0.element_size()
    base = t0.data_ptr()
    off = 0
    for t in ts:
        if not t.is_contiguous() or t.data_ptr() != base + off * es or t.dtype != t0.dtype:
            return None
        off += t.numel()
    if t0.untyped_storage().data_ptr() != ts[-1].untyped_storage().data_ptr():
        return None
    rows = sum(t.shape[0] for t in ts)
    shape = (rows,) + tuple(t0.shape[1:])
    stride = t0.stride() if t0.dim() > 1 else (1,)
    return t0.detach().as_strided(shape, stride)


class _Linear3Fn(torch.autograd.Function):
    """y = x @ [Wq;Wk;Wv]^T + [bq;bk;bv] as ONE GEMM (N = 3H)."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, bq, bk, bv):
        W = _adjacent_view([wq, wk, wv])
        if W is None:
            W = torch.cat([wq, wk, wv], 0)
        b = _adjacent_view([bq, bk, bv])
        if b is None:
            b = torch.cat([bq, bk, bv], 0)
        x2 = x.reshape(-1, x.shape[-1])
        y = torch.addmm(b.to(x.dtype), x2, W.t().to(x.dtype))
        ctx.save_for_backward(x2, W)
        ctx.xshape = x.shape
        ctx.n = [wq.shape[0], wk.shape[0], wv.shape[0]]
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, W = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = (dy2 @ W.to(dy2.dtype)).view(ctx.xshape)
        dW = (dy2.t() @ x2).float()
        if use_kernels(dy2) and dy2.shape[-1] % 4 == 0:
            db = C().colsum(dy2.contiguous(), None)
        else:
            db = dy2.float().sum(0)
        a, b_, _ = ctx.n
        return (dx, dW[:a], dW[a:a + b_], dW[a + b_:], db[:a], db[a:a + b_], db[a + b_:])


def linear3(x, wq, wk, wv, bq, bk, bv):
    return _Linear3Fn.apply(x, wq, wk, wv, bq, bk, bv)


# ----------------------------------------------------------------- attention core
def attention(qkv, mask_bias, num_heads, p, training):
    """softmax(Q K^T / sqrt(d) + mask) -> dropout -> @ V  on the packed [B, S, 3H]
    projection; returns [B, S, H] (reference BertSelfAttention, :351-377).
    ``mask_bias`` is the additive [B, S] key mask ((1 - m) * -10000)."""
    from .flash_attention import attention as _attention
    return _attention(qkv, mask_bias, num_heads, p if training else 0.0)


# ----------------------------------------------------------------- MLM decoder + softmax-xent
class _DecoderXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, W, bias, labels):
        logits = torch.mm(h, W.t().to(h.dtype))
        loss_rows = C().softmax_xent_(logits, bias, labels, -1)   # logits <- softmax - onehot
        count = (labels != -1).sum().to(torch.float32)
        loss = loss_rows.sum() / count
        ctx.save_for_backward(h, W, logits, count)
        return loss

    @staticmethod
    def backward(ctx, g):
        h, W, dl, count = ctx.saved_tensors
        scale = (g.float() / count).reshape(1)
        dbias = C().colsum(dl, scale)          # scales dl in place, returns column sums
        dh = torch.mm(dl, W.to(dl.dtype))
        dW = torch.mm(dl.t(), h).float()
        return dh, dW, dbias, None


def decoder_xent(h, W, bias, labels):
    """mean CE(h @ W^T + bias, labels, ignore_index=-1)."""
    if use_kernels(h):
        return _DecoderXentFn.apply(h.contiguous(), W, bias, labels.contiguous())
    logits = F.linear(h, W.to(h.dtype)) + bias
    return F.cross_entropy(logits.float(), labels, ignore_index=-1)


def masked_rows(labels_flat, cap):
    """Indices of the rows whose label != -1, first ``cap`` of them in order, with
    NO host synchronisation (stable sort puts masked rows first; tail rows are
    ignored rows and contribute nothing).  cap=None -> all rows."""
    n = labels_flat.numel()
    if cap is None or cap >= n:
        return None
    key = (labels_flat == -1).to(torch.int8)
    return torch.argsort(key, stable=True)[:cap]
