"""fp32 GEMMs as three fp16 piece products (``--fp32-gemm fp16x3``; csrc/kernels/gemm_f16.hip).

Every fp32 operand row x is used as 2^-E (h0 + h1) with h0 = fp16(2^E x), h1 = fp16(2^E x - h0):
22 significant bits per element; the product a.b is a0 b0 + a0 b1 + a1 b0 (the dropped a1 b1
is 2^-22 relative) -- three fp16 MFMA passes where the bf16 emulation needs six
(the round-3 ``bf16x6`` mode).  E is chosen PER ROW of each operand (per row of A and per row
of B = output column; the epilogue multiplies by 2^-(Ea[r] + Eb[c])), so a row keeps 22 bits
however far below the tensor's largest row it lies.  Every tensor handed to these GEMMs
travels with **max |x| partials per row**: a [rows, P] fp32 tensor whose row-wise max is that
row's max |x| (its producer writes it -- LayerNorm [rows, 1], attention [rows, heads], this
module's GELU epilogues [rows, N tiles] -- or ``amax`` computes it in one read pass).  A 1-D
tensor instead is a per-tensor bound (e.g. ``bound``).  The GEMMs read activations and gradients
AS fp32 and split them in registers -- except the forward LayerNorms' outputs, which travel with
their pieces already split (``attach_pieces``, ``HX_PRESPLIT``); weights are split ahead of time
(one launch per forward for the whole encoder, ``weight_scope``), W's rows scaled by their own
maxima and W^T's rows (= W's columns) by the column maxima.

Reference sites: hetseq/bert_modeling.py:334-336 (Q/K/V), :383 (attention output), :409 +
:166-168 (FFN up, bias_gelu), :419 (FFN down), :509 (pooler), :522 (MLM transform), :538-547
(MLM decoder), :1221 (NER classifier) and their backward products.
"""
import os

import torch

from ._ext import C, use_kernels


class _State(object):
    on = False
    scope = None        # {(data_ptr, shape): (wf, wt, parts)} for the running forward
    min_rows = 1


def set_enabled(flag):
    _State.on = bool(flag)


def enabled():
    return _State.on


def ok(x2, n_out):
    """The fp16x3 GEMMs take the product [rows, K] x [K, n_out]: fp32 GPU operands, 16-deep k
    steps and an output width with a tile shape (multiples of 64; smaller heads -- the NSP
    classifier, NER's num_labels -- stay on the library fp32 GEMM, microseconds each)."""
    return (_State.on and x2.dtype == torch.float32 and use_kernels(x2) and x2.shape[-1] % 64 == 0 and
            n_out % 64 == 0 and x2.numel() > 0)


def wgrad_ok(n_out, n_in):
    return n_out % 128 == 0 and n_in % 128 == 0


def _aligned(t):
    return t.stride(-1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0


def rows2(x):
    """[.., K] -> a 2-D [rows, K] operand the kernels can read (contiguous copy if not)."""
    x2 = x.reshape(-1, x.shape[-1])
    return x2 if _aligned(x2) else x2.contiguous()


# ---------------------------------------------------------------- max |x| partials
def attach(t, parts):
    """Hand ``parts`` (max |t| partials, written by t's producer) to the GEMMs that consume t."""
    if parts is not None:
        t._hx_amax = parts
        t._hx_amax_ver = t._version
    return t


def amax(t, t2=None):
    """max |t| partials per row ([rows, P]): the producer's (if ``t`` has not changed since), else
    one read pass ([rows, 1])."""
    p = getattr(t, '_hx_amax', None)
    if p is not None and getattr(t, '_hx_amax_ver', -1) == t._version:
        return p
    x2 = t2 if t2 is not None else rows2(t)
    if not (x2.shape[-1] % 4 == 0 and _aligned(x2)):
        x2 = x2.contiguous()
    if cols_peek(t) is None and x2.shape[-1] <= 4096:
        # no producer wrote either scale source (e.g. dQKV of the multi-key-block attention
        # backward): the row maxima and the column maxima its weight gradient will ask for, from
        # one read
        r, c = C().amax_rows_cols(x2)
        attach_cols(t, c)
        return attach(t, r)._hx_amax
    return attach(t, C().amax_rows(x2))._hx_amax


# LayerNorm outputs (forward) and gradients (backward) also travel with their fp16 P2 pieces, split
# at the same row scales by the LayerNorm kernel (the values are in its registers anyway): the
# consumer GEMM (QKV / FFN up forward, attention-output / FFN-down data gradient) then reads the
# pieces instead of splitting fp32 in its k loop -- bit-identical results, 5-7 % faster products
# (profiles/r5as_presplit_gemm_ab.log) for one extra 4 B / element write by the LayerNorm (+8 us per
# call at BERT-base phase 1).  That pays in the forward (QKV -14 us, FFN up -15 us in the step) but
# not in the backward (attention-output dgrad -4 us, FFN-down dgrad with its GELU epilogue -4 us):
# the default splits in the forward LayerNorms only (profiles/r5av_presplit_step_ab.txt: 36.60 /
# 36.67 / 36.77 ms for forward / off / both, medians of three on one box).
_PRESPLIT = int(os.environ.get('HX_PRESPLIT', '1'))   # 0 off, 1 forward LayerNorms, 2 and backward


def presplit(H, bwd=False):
    """Should a LayerNorm of width H write its output's (bwd: its gradient's) pieces?"""
    return _PRESPLIT >= (2 if bwd else 1) and _State.on and H % 16 == 0


def attach_pieces(t, pieces):
    if pieces is not None:
        t._hx_p2 = pieces
        t._hx_p2_ver = t._version
    return t


def take_pieces(t):
    """The producer-written pieces of ``t`` (None if none / stale), handed over once: the attribute
    is dropped so the pieces die with their one consumer GEMM."""
    p = getattr(t, '_hx_p2', None)
    if p is None:
        return None
    ok = getattr(t, '_hx_p2_ver', -1) == t._version
    del t._hx_p2
    return p if ok else None


def attach_cols(t, src):
    """Hand the weight gradients that consume ``t`` its per-COLUMN scale source: a [P, C] tensor of
    column-max partials (producer-written), or ``('affine', gamma, beta, z, mul)`` for a LayerNorm
    output gamma zhat + beta (|column c| <= (|gamma_c| z + |beta_c|) mul, z = sqrt(H - 1) bounds
    |zhat| of any normalised row)."""
    if src is not None:
        t._hx_cmax = src
        t._hx_cmax_ver = t._version
    return t


def cols(t, t2=None):
    """``t``'s per-column scale source: the producer's (if ``t`` has not changed since), else one
    column-max read pass ([1, C])."""
    c = getattr(t, '_hx_cmax', None)
    if c is not None and getattr(t, '_hx_cmax_ver', -1) == t._version:
        return c
    x2 = t2 if t2 is not None else rows2(t)
    if not (x2.shape[-1] % 4 == 0 and _aligned(x2)):
        x2 = x2.contiguous()
    return attach_cols(t, C().amax_cols(x2))._hx_cmax


def cols_peek(t):
    """The producer-attached column scale source of ``t`` (None if there is none / it is stale)."""
    c = getattr(t, '_hx_cmax', None)
    return c if c is not None and getattr(t, '_hx_cmax_ver', -1) == t._version else None


def ln_affine(gamma, beta, keep=1.0):
    """The column scale source of a LayerNorm output (``attach_cols``)."""
    H = gamma.numel()
    return ('affine', gamma.detach(), beta.detach(), float(max(H - 1, 1)) ** 0.5, 1.0 / keep)


_ONES = {}


def bound(dev, v=1.0):
    """A constant max |x| bound (a valid partials vector: the scale only needs an upper bound)."""
    key = (dev, float(v))
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.full((1,), float(v), dtype=torch.float32, device=dev)
    return t


# ---------------------------------------------------------------- weight pieces
class weight_scope(object):
    """Split every weight in ``Ws`` into P2 fp16 pieces in ONE launch pair (max |W| + split) on
    entry; ``weight_pieces`` returns them until exit (scoped to one forward: weights change at
    every optimizer step, and an activation-checkpointing recompute outside the scope splits
    again)."""

    def __init__(self, Ws):
        self.Ws = [W for W in Ws if W is not None]

    def __enter__(self):
        self.prev = _State.scope
        Ws = [W for W in self.Ws if W.dim() == 2 and W.shape[0] % 64 == 0 and W.shape[1] % 64 == 0 and
              W.is_contiguous() and W.dtype == torch.float32 and W.is_cuda]
        if _State.on and Ws:
            d = {}
            for i in range(0, len(Ws), 64):
                chunk = Ws[i:i + 64]
                for W, o in zip(chunk, C().split_weight_f16(chunk)):
                    d[(W.data_ptr(), tuple(W.shape))] = tuple(o)
            _State.scope = d
        return self

    def __exit__(self, *exc):
        _State.scope = self.prev
        return False


def weight_pieces(W):
    """(wf [N, 2K], wt [K, 2N], rmax [N, 1], cmax [K, 1]) of W [N, K] (N, K multiples of 64): the
    pieces of W and of W^T, and the per-row scale sources of each (W's row / column maxima)."""
    if _State.scope is not None:
        e = _State.scope.get((W.data_ptr(), tuple(W.shape)))
        if e is not None:
            return e
    return tuple(C().split_weight_f16([W.detach().contiguous()])[0])


# ---------------------------------------------------------------- products
def mm(a2, a_parts, b, b_parts, out=None, beta=False, bias=None, ks=0):
    """a2 [M, K] (fp32, or its fp16 P2 pieces [M, 2K] at the row scales of a_parts) . b^T (b = P2 pieces [N, 2K]) (+ out if beta) (+ bias) -> fp32 [M, N];
    ``a_parts`` / ``b_parts``: per-row max |x| partials of a2 and of b's rows;
    ``ks``: split-K slabs (0 = the kernel's plan: deep reductions with few output tiles)."""
    return C().gemm_f16(a2, a_parts, b, b_parts, out=out, beta=beta, bias=bias, ks=ks)


def linear(x2, xparts, W, bias=None):
    """y = x2 W^T (+ bias); also returns W^T's pieces and their row scale source (W's column
    maxima) for the backward."""
    wf, wt, rmax, cmax = weight_pieces(W)
    return mm(x2, xparts, wf, rmax, bias=bias), wt, cmax


def dgrad(dy2, dparts, wt, wt_parts, acc=None):
    """dx = dy2 W from W^T's pieces, accumulated into ``acc`` (beta = 1) when given."""
    if acc is not None:
        return mm(dy2, dparts, wt, wt_parts, out=acc, beta=True)
    return mm(dy2, dparts, wt, wt_parts)


def wgrad(dy2, dcols, x2, xcols, n_out, n_in, slot=None):
    """dW [n_out, n_in] = dy2^T x2 over the token rows, straight into ``slot`` when given
    (shapes without a tile: the library fp32 product).  ``dcols`` / ``xcols``: the operands' column
    scale sources (``cols``): dW's rows are scaled by dy2's column maxima, its columns by x2's."""
    out = slot if slot is not None else torch.empty(n_out, n_in, device=dy2.device)
    if wgrad_ok(dy2.shape[1], n_in) and dy2.shape[1] >= n_out and _aligned(dy2) and _aligned(x2):
        if isinstance(xcols, tuple):   # ('affine', gamma, beta, z, mul)
            _, g, b, z, mul = xcols
            return C().wgrad_f16(dy2, dcols, x2, bound(x2.device), out, x_gamma=g, x_beta=b, x_z=z, x_mul=mul)
        return C().wgrad_f16(dy2, dcols, x2, xcols, out)
    return torch.mm(dy2[:, :n_out].t(), x2, out=out)


def gemm_gelu(x2, xparts, W1, b1):
    """FFN up with its bias + GELU epilogue: (gelu'(u), h = gelu(u), h's per-row max |.| partials
    [M, N tiles], h's column maxima per M tile [M tiles, N], W1^T's pieces, W1's column maxima)."""
    wf, wt, rmax, cmax = weight_pieces(W1)
    d, h, hrow, hcol = C().gemm_f16_gelu(x2, xparts, wf, rmax, b1, 1)
    return d, h, fit_rows(hrow), fit_cols(hcol), wt, cmax


def gemm_dgelu(dy2, dparts, wt2, wt2_parts, d, dbias_out):
    """FFN-down data gradient with the GELU backward: (t = (dy W2) * gelu'(u), t's per-row max |.|
    partials, t's column maxima per M tile, d b1)."""
    t, trow, tcol, db = C().gemm_f16_dgelu(dy2, dparts, wt2, wt2_parts, d, None, dbias_out, 1)
    return t, fit_rows(trow), fit_cols(tcol), db


# the consumers' limits on producer-written partials (csrc/bindings.cpp: a GEMM's row scale source
# has at most 64 partials per row, a weight gradient's column source at most 256 per column)
MAX_ROW_PARTS = 64
MAX_COL_PARTS = 256


def fit_rows(p):
    """Row partials [M, P] with P over the GEMMs' limit (an epilogue tile narrower than N / 64,
    e.g. the 64-wide tile of an intermediate size > 4096) folded to [M, 1]: same maxima."""
    return p.amax(1, keepdim=True) if p is not None and p.dim() == 2 and p.shape[1] > MAX_ROW_PARTS else p


def fit_cols(p):
    """Column partials [P, N] with P over the weight gradient's limit (more than 256 M tiles, e.g.
    BERT-large's 64-row FFN tile above 16384 token rows) folded to [1, N]: same maxima."""
    return p.amax(0, keepdim=True) if p is not None and p.dim() == 2 and p.shape[0] > MAX_COL_PARTS else p


# ---------------------------------------------------------------- --precision bf16 (same kernel, one pass)
class _B16(object):
    scope = None        # {(data_ptr, shape): W^T in bf16} for the running forward


def bf16_ok(x2, n_out, n_in):
    """--precision bf16 products on gemm_f16.hip's bf16 variant: bf16 GPU activations, 32-deep k
    steps, tile-able widths (the tiny heads stay on the library GEMM)."""
    return (x2.dtype == torch.bfloat16 and use_kernels(x2) and n_in % 64 == 0 and n_out % 64 == 0 and
            x2.numel() > 0)


class bf16_scope(object):
    """W^T in bf16 for every weight in ``Ws`` (the data-gradient operands of the NT kernel), one
    launch per forward; ``bf16_wt`` returns them until exit."""

    def __init__(self, Ws):
        self.Ws = [W for W in Ws if W is not None and W.dim() == 2 and W.shape[0] % 64 == 0 and
                   W.shape[1] % 64 == 0 and W.is_contiguous() and W.dtype == torch.float32 and W.is_cuda]

    def __enter__(self):
        self.prev = _B16.scope
        if self.Ws:
            d = {}
            for i in range(0, len(self.Ws), 64):
                chunk = self.Ws[i:i + 64]
                for W, wt in zip(chunk, C().weight_bf16_t(chunk)):
                    d[(W.data_ptr(), tuple(W.shape))] = wt
            _B16.scope = d
        return self

    def __exit__(self, *exc):
        _B16.scope = self.prev
        return False


def bf16_wt(W):
    """W^T [K, N] in bf16 (the running forward's, or converted now)."""
    if _B16.scope is not None:
        e = _B16.scope.get((W.data_ptr(), tuple(W.shape)))
        if e is not None:
            return e
    return C().weight_bf16_t([W.detach().contiguous()])[0]


_BF16_LIB = os.environ.get('HX_BF16_LIB', '1') != '0'


def bf16_lib():
    """--precision bf16 runs its plain products on hipBLASLt (HX_BF16_LIB=0: all on gemm_f16.hip)."""
    return _BF16_LIB


def mm_bf16(a2, b, out=None, beta=False, bias=None, out_bf16=True):
    """a2 [M, K] bf16 . b^T (b bf16 [N, K]) (+ out) (+ bias).  Plain and beta products with a bf16
    output go to hipBLASLt (the library's bf16 kernels are 20-35 % faster than the hand-written
    bf16 variant on these shapes, r5m); the products with fused epilogues (bias + GELU, GELU
    backward) stay on gemm_f16.hip."""
    if _BF16_LIB and out_bf16 and a2.dtype == torch.bfloat16 and b.dtype == torch.bfloat16:
        if beta:
            return out.view(a2.shape[0], b.shape[0]).addmm_(a2, b.t())
        if bias is not None:
            # the library epilogue takes the bias in the operands' dtype: it is rounded to bf16 before
            # the add (the hand-written kernel adds it in fp32) -- one extra bf16 rounding of the bias
            # on an output that is rounded to bf16 anyway
            if out is not None:
                return torch.addmm(bias.to(torch.bfloat16), a2, b.t(), out=out.view(a2.shape[0], b.shape[0]))
            return torch.addmm(bias.to(torch.bfloat16), a2, b.t())
        if out is not None:
            return torch.mm(a2, b.t(), out=out.view(a2.shape[0], b.shape[0]))
        return torch.mm(a2, b.t())
    return C().gemm_bf16(a2, b, out=out, beta=beta, bias=bias, out_bf16=out_bf16)
