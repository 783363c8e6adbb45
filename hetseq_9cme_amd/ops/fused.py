"""Autograd wrappers around the gfx950 kernels + torch reference implementations.

Every public op dispatches on the device of its input: GPU tensors run the
hand-written HIP kernels (``_C``), CPU tensors run the plain-torch reference of
the same math (used by the CPU test-suite and as the numerics oracle for the GPU
kernel tests).  Semantics follow the reference model (hetseq/bert_modeling.py).
"""
import os
import torch
import torch.nn.functional as F

from . import gemm16
from ._ext import C, use_kernels
from .rng import get_rng

ACT_IDS = {'gelu': 0, 'tanh': 1, 'relu': 2, 'none': 3}


def cast_w(w, dtype):
    """Parameter ``w`` in compute dtype: its bf16 shadow view when one exists
    (``FlatParamSpace.enable_bf16_shadow``), else a cast."""
    if w is None or w.dtype == dtype:
        return w
    sh = getattr(w, '_hx_bf16', None) if dtype == torch.bfloat16 else None
    return sh if sh is not None else w.to(dtype)


def _wgrad(dy2, x2, slot):
    """dW = dy2^T x2 in fp32; written straight into ``slot`` when given.  bf16
    operands use the hand-written split-K bf16-MFMA kernel (csrc/kernels/wgrad_bf16.hip,
    ~3x the library's rate on these tokens-as-reduction shapes), else the library
    bf16 x bf16 -> fp32 GEMM; neither makes a bf16 result or a cast pass."""
    if dy2.dtype == torch.float32:
        return torch.mm(dy2.t(), x2, out=slot) if slot is not None else torch.mm(dy2.t(), x2)
    if use_kernels(dy2) and C().wgrad_bf16_ok(dy2, x2):
        out = slot if slot is not None else torch.empty(dy2.shape[1], x2.shape[1], device=dy2.device)
        return C().wgrad_bf16(dy2, x2, out)
    if slot is not None:
        return torch.mm(dy2.t(), x2, out_dtype=torch.float32, out=slot)
    return torch.mm(dy2.t(), x2, out_dtype=torch.float32)


def _nullctx():
    import contextlib
    return contextlib.nullcontext()


def grad_slot(p):
    """The flat-buffer gradient slot of parameter ``p`` if this backward may write
    p's gradient there directly (first contribution of the step), else None."""
    flat = getattr(p, '_hx_flat', None)
    if flat is None or not p.is_cuda:
        return None
    return flat.claim(p)


class ResidualGrad(object):
    """Per-forward mailbox that fuses a residual branch's gradient into a GEMM.

    In a post-LN transformer block the block input ``x`` feeds both a linear
    (QKV / FFN-up) and the residual of the block's closing LayerNorm, so its
    gradient is ``dres + dY . W`` -- autograd would materialise both and launch
    an add kernel (3 x 50 MB of HBM traffic per block at B*S = 16384, H = 768).
    Instead the LayerNorm backward (which always runs first: the LN is
    downstream of the linear) deposits ``dres`` here and returns no gradient
    for the residual, and the linear's backward computes
    ``dx = dres.addmm_(dY, W)`` -- one GEMM with beta = 1, no extra kernel.
    Falls back to the plain path whenever the order or dtypes do not allow it.
    """
    __slots__ = ('grad', 'consumed')

    def __init__(self):
        self.grad = None
        self.consumed = False

    def deposit(self, g):
        """LN backward: hand over ``g`` unless the consumer already ran."""
        if self.consumed:
            return False
        self.grad = g
        return True

    def take(self, dtype):
        self.consumed = True
        g, self.grad = self.grad, None
        if g is not None and g.dtype != dtype:
            return None, g
        return g, None


def _dgrad(dy2, W, xshape, mbox):
    """dx = dy2 @ W, accumulated into the deposited residual gradient if any."""
    Wc = cast_w(W, dy2.dtype)
    if mbox is None:
        return torch.mm(dy2, Wc).view(xshape)
    g, other = mbox.take(dy2.dtype)
    if g is not None:
        return g.view(-1, W.shape[1]).addmm_(dy2, Wc).view(xshape)
    dx = torch.mm(dy2, Wc).view(xshape)
    return dx if other is None else dx + other.view(xshape).to(dx.dtype)


def _dgrad_bf16(dy2, W, xshape, mbox, wt=None):
    """``_dgrad`` for --precision bf16 on the hand-written kernel: dy . (W^T)^T with the bf16 W^T
    (``wt``: kept by the forward from its one-launch batch, so the backward converts nothing),
    beta = 1 into the deposited residual gradient if any."""
    wt = wt if wt is not None else gemm16.bf16_wt(W)
    dy2 = gemm16.rows2(dy2)
    if mbox is not None:
        g, other = mbox.take(dy2.dtype)
        if g is not None:
            return gemm16.mm_bf16(dy2, wt, out=g.view(-1, xshape[-1]), beta=True).view(xshape)
        dx = gemm16.mm_bf16(dy2, wt).view(xshape)
        return dx if other is None else dx + other.view(xshape).to(dx.dtype)
    return gemm16.mm_bf16(dy2, wt).view(xshape)


# ----------------------------------------------------------------- weight-grad side stream
class _Side(object):
    # 'auto' (default): the side stream for products of >= AUTO_ROWS token rows (BERT-base phase 1
    # at 128 sequences per GPU, phase 2), the compute stream below (batch 32, fine-tuning).  Round 6,
    # same box, alternated: batch 128 35.38 / 35.43 vs 36.56 / 35.48 ms/step with / without
    # (profiles/r6e_overlap_ab.txt); batch 32 13.52 vs 13.32.  (Round 4, before the attention and
    # GEMM changes since, had measured the compute stream ahead: profiles/r4p_overlap_ab.md.)
    # 'on' (--overlap-wgrad) / 'off' (--no-overlap-wgrad): every product / none.
    mode = 'auto'
    AUTO_ROWS = 8192
    auto_rows = AUTO_ROWS   # set_side_stream(..., auto_rows=): 4096 for hidden sizes >= 1024
    priority = os.environ.get('HX_SIDE_PRIO', 'low')   # 'low' (default) or 'normal' HIP priority
    # CUs the side-stream plans leave free (-1: a quarter of the device's, 64 on MI355X).  Alternated
    # on one box (profiles/r6ah_side_reserve_ab.txt): batch 128 35.34 / 35.35 -> 35.04 / 35.05 ms/step,
    # phase 2 40.36 / 40.47 -> 39.24 / 39.28 at 64; 48 and 80 in between / worse
    reserve = int(os.environ.get('HX_SIDE_RESERVE', '-1'))
    streams = {}          # (device index, low priority) -> stream
    active = {}           # device index -> the side stream this backward queued work on


def set_side_stream(flag, auto_rows=None):
    """Weight-gradient work on a side stream: True / 'on', False / 'off', or 'auto' (on for products
    of >= ``auto_rows`` token rows, default _Side.AUTO_ROWS, the measured default)."""
    _Side.mode = {True: 'on', False: 'off'}.get(flag, flag) if isinstance(flag, bool) else str(flag)
    assert _Side.mode in ('on', 'off', 'auto'), flag
    _Side.auto_rows = int(auto_rows) if auto_rows else _Side.AUTO_ROWS


def side_begin(device, rows=0):
    """Side stream for off-critical-path weight-gradient work (dW GEMMs, bias
    column sums) of the running backward, ordered after everything already
    queued on the compute stream.  While the compute stream continues with the
    dgrad chain (attention / LayerNorm / GELU backward: mostly memory-bound),
    the side stream's GEMMs fill the matrix cores.  Joined back into the compute
    stream by an end-of-backward callback (``side_join``)."""
    if device.type != 'cuda' or _Side.mode == 'off' or (_Side.mode == 'auto' and rows < _Side.auto_rows):
        return None
    if torch.cuda.is_current_stream_capturing():
        # a captured update (utils/train_graph.py) stays on one stream: replays of updates captured
        # with the side-stream branch ran at twice the device time (NER 17.6-19.2 vs 8.3 ms/update,
        # profiles/r6ae_side_stream_low_priority_ab.txt)
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _Side.active.get(idx)
    if st is None:
        st = _side_stream(idx)
        if not _Side.active:
            torch.autograd.Variable._execution_engine.queue_callback(side_join)
        C().reducer_set_side_stream(st.cuda_stream)   # bucket collectives order after it
        _Side.active[idx] = st
    st.wait_stream(torch.cuda.current_stream(idx))
    return st


def _side_stream(idx):
    low = _Side.priority == 'low'
    key = (idx, low)
    st = _Side.streams.get(key)
    if st is None:
        if low:
            # HIP's LOWEST stream priority (1; the compute stream is at 0, RCCL's streams at -1): when
            # CUs free up, the dispatcher serves the critical path (attention, LayerNorm, data
            # gradients) before these weight gradients.  Same box, alternated 3x: phase 2 41.19-41.38
            # -> 40.14-40.15 ms/step, batch 128 35.14-35.22 -> 34.95-35.02
            # (profiles/r6ad_stream_priority_ab.txt).  (A high-priority side stream measured no
            # different in round 3.)
            with torch.cuda.device(idx):
                st = torch.cuda.ExternalStream(C().priority_stream(1), device=torch.device('cuda', idx))
        else:
            st = torch.cuda.Stream(device=idx)
        _Side.streams[key] = st
    return st


class _SideCtx(object):
    """Launches on the side stream, planned for ``_Side.reserve`` fewer workgroup slots than CUs:
    the one-workgroup-per-CU weight gradients then leave those CUs to the compute stream's
    LayerNorm / attention backward instead of holding every CU for a whole kernel (the CU
    reservation of cu_reserve.hip, set only while side-stream work is launched)."""
    __slots__ = ('st', 'sc', 'prev')

    def __init__(self, st):
        self.st = st

    def __enter__(self):
        self.sc = torch.cuda.stream(self.st)
        self.sc.__enter__()
        self.prev = None
        if _Side.reserve < 0:
            _Side.reserve = C().num_cus() // 4
        if _Side.reserve > 0:
            self.prev = C().reserved_cus()
            C().set_reserved_cus(max(self.prev, _Side.reserve))
        return self

    def __exit__(self, *exc):
        if self.prev is not None:
            C().set_reserved_cus(self.prev)
        return self.sc.__exit__(*exc)


def side_ctx(side):
    """``with side_ctx(side_begin(...))``: the side stream (+ its CU reservation), or nothing."""
    return _SideCtx(side) if side is not None else _nullctx()


def active_side_stream(device):
    """The side stream if this backward queued work on it (reducer ordering)."""
    if device.type != 'cuda':
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _Side.active.get(idx)


def side_join():
    """Make the compute stream wait for all queued side-stream work."""
    if not _Side.active:
        return
    for idx, st in list(_Side.active.items()):
        torch.cuda.current_stream(idx).wait_stream(st)
    _Side.active.clear()
    C().reducer_set_side_stream(0)


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
        seed, stream = get_rng().next(ids.device) if p > 0 else (get_rng().seed_tensor(ids.device), 0)
        am = _amax_buf(ids.numel(), wte, out_bf16)
        pc = _pieces_buf(ids.numel(), wte.shape[1], wte) if am is not None else None
        out, z, mean, rstd = C().embed_ln_fwd(ids, tt, wte, wpe, wtt, gamma, beta, eps, keep, seed, stream,
                                              out_bf16, am, pc)
        gemm16.attach(out, am)   # fp16x3: its max |x| partials for the first layer's QKV GEMM
        gemm16.attach_pieces(out, pc)   # and its pieces at those row scales
        if am is not None:       # and the column bound of LN (+ dropout) for its weight gradient
            gemm16.attach_cols(out, gemm16.ln_affine(gamma, beta, keep))
        ctx.save_for_backward(ids, tt if tt is not None else torch.Tensor(), z, mean, rstd, gamma)
        ctx.params = (wte, wpe, wtt, beta)
        ctx.has_tt = tt is not None
        ctx.meta = (keep, seed, stream, wte.shape[0], wpe.shape[0], wtt.shape[0])
        return out

    @staticmethod
    def backward(ctx, dout):
        side_join()   # the tied decoder's dW may still be in flight on the side stream
        ids, tt, z, mean, rstd, gamma = ctx.saved_tensors
        keep, seed, stream, V, P, NT = ctx.meta
        dout = dout.contiguous()
        wte, wpe, wtt, beta = ctx.params
        dz, _, dgamma, dbeta, _ = C().ln_bwd(dout, z, mean, rstd, gamma, keep, seed, stream, True, False, False,
                                             grad_slot(gamma), grad_slot(beta), None)
        H = z.shape[-1]
        # word embeddings: scatter straight into the flat slot; when the tied MLM
        # decoder already claimed (and filled) it this step, add on top and return
        # None so autograd adopts the decoder's slot view holding both contributions
        ret_wte = grad_slot(wte)
        if ret_wte is not None:
            ret_wte.zero_()
            dwte = ret_wte
        elif getattr(wte, '_hx_flat', None) is not None and wte.grad is None and wte._hx_flat.is_claimed(wte):
            dwte = wte._hx_flat.slots[wte._hx_index]
        else:
            dwte = ret_wte = torch.zeros(V, H, device=z.device, dtype=torch.float32)
        dwpe = grad_slot(wpe)
        dwpe = (dwpe.zero_() if dwpe is not None else torch.zeros(P, H, device=z.device, dtype=torch.float32))
        dwtt = grad_slot(wtt)
        dwtt = dwtt if dwtt is not None else torch.empty(NT, H, device=z.device, dtype=torch.float32)
        B, S = ids.shape
        dz2 = dz.reshape(-1, H)
        ids_f = ids.reshape(-1)
        # word embeddings: segmented sums over id-sorted rows (few atomics even for
        # the very frequent ids of real text); accumulates into dwte
        C().embed_word_grad(dz2, ids_f, torch.argsort(ids_f), dwte)
        # positions: a column sum over the batch of the [B, S*H] view
        C().colsum(dz.reshape(B, S * H), None, dwpe[:S].reshape(-1))
        # token types: per-type column sums (one pass over dz) for the usual 2 types; one_hot(tt)^T . dz
        # (one small GEMM) for more
        if ctx.has_tt and NT <= 3 and dwtt.is_contiguous():
            C().embed_type_grad(dz2, tt.reshape(-1), dwtt)
        elif ctx.has_tt:
            oh = F.one_hot(tt.reshape(-1), NT).to(dz2.dtype)
            if dz2.dtype == torch.float32:
                torch.mm(oh.t(), dz2, out=dwtt)
            else:
                dwtt.copy_(torch.mm(oh.t(), dz2).float())
        else:
            dwtt.zero_()
            torch.sum(dwpe[:S], 0, out=dwtt[0])
        return None, None, ret_wte, dwpe, dwtt, dgamma, dbeta, None, None, None


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


def _amax_buf(rows, ref, bf16, bwd=False):
    """[rows, 1] buffer for a LayerNorm kernel's max |out| of every row (the per-row operand scale
    of the fp16x3 GEMMs that consume its output, ops/gemm16.py), or None when no such GEMM runs."""
    if bf16 or not gemm16.enabled() or not ref.is_cuda:
        return None
    return torch.empty(rows, 1, dtype=torch.float32, device=ref.device)


def _pieces_buf(rows, H, ref, bwd=False):
    """[rows, 2H] fp16 buffer for a LayerNorm kernel's output pieces (gemm16.attach_pieces), or None."""
    if not gemm16.presplit(H, bwd):
        return None
    return torch.empty(rows, 2 * H, dtype=torch.float16, device=ref.device)


# ----------------------------------------------------------------- bias + dropout + residual + LN
class _BiasDropResLNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, bias, res, gamma, beta, eps, p, mbox):
        keep = 1.0 - p
        seed, stream = get_rng().next(y.device) if p > 0 else (get_rng().seed_tensor(y.device), 0)
        rows, H = y.numel() // y.shape[-1], y.shape[-1]
        am = _amax_buf(rows, y, y.dtype != torch.float32)
        pc = _pieces_buf(rows, H, y) if am is not None else None
        out, z, mean, rstd = C().ln_fwd(y, bias, res, gamma, beta, eps, keep, seed, stream, False, True, am, pc)
        gemm16.attach(out, am)   # fp16x3: its max |x| partials for the next QKV / FFN-up GEMM
        gemm16.attach_pieces(out, pc)   # and its pieces, split at those row scales
        if am is not None:       # and its column bound for their weight gradients
            gemm16.attach_cols(out, gemm16.ln_affine(gamma, beta))
        ctx.save_for_backward(z, mean, rstd, gamma)
        ctx.params = (bias, beta)
        ctx.mbox = mbox
        ctx.meta = (keep, seed, stream, bias is not None, res is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        z, mean, rstd, gamma = ctx.saved_tensors
        keep, seed, stream, has_bias, has_res = ctx.meta
        bias, beta = ctx.params
        need_dy = has_bias or keep < 1.0
        rows, H = z.numel() // z.shape[-1], z.shape[-1]
        am = _amax_buf(rows, z, z.dtype != torch.float32, bwd=True)
        cm = torch.empty(1, H, dtype=torch.float32, device=z.device) if am is not None else None
        pc = _pieces_buf(rows, H, z, True) if am is not None else None
        dz, dy, dgamma, dbeta, dbias = C().ln_bwd(dout.contiguous(), z, mean, rstd, gamma, keep, seed, stream,
                                                  False, need_dy, has_bias, grad_slot(gamma), grad_slot(beta),
                                                  grad_slot(bias) if has_bias else None, am, cm, pc)
        # fp16x3: max |dy| per row (data gradient) and per column (weight gradient), and dy's pieces
        dy_ret = gemm16.attach_pieces(gemm16.attach_cols(gemm16.attach(dy if need_dy else dz, am), cm), pc)
        dres = dz if has_res else None
        # dz is a private buffer only when dy is separate: then it can become the
        # accumulator of the consumer linear's dgrad GEMM
        if dres is not None and need_dy and ctx.mbox is not None and ctx.mbox.deposit(dz):
            dres = None
        return dy_ret, (dbias if has_bias else None), dres, dgamma, dbeta, None, None, None


def bias_dropout_residual_ln(y, bias, res, gamma, beta, eps, p, training, res_grad=None):
    """LN(dropout(y + bias) + res)  (BertSelfOutput / BertOutput, bert_modeling.py:387-391).
    ``res_grad``: a ``ResidualGrad`` shared with the linear that also consumed ``res``."""
    p = p if training else 0.0
    if use_kernels(y):
        return _BiasDropResLNFn.apply(y.contiguous(), bias, None if res is None else res.contiguous(), gamma, beta,
                                      float(eps), float(p), res_grad)
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
        ctx.bias = bias
        return out

    @staticmethod
    def backward(ctx, dout):
        a, b = ctx.saved_tensors
        aid, has_bias = ctx.meta
        slot = grad_slot(ctx.bias) if has_bias else None
        if aid == 0:
            dy, dbias = C().bias_act_bwd(dout.contiguous(), a, b if has_bias else None, None, aid, has_bias, slot)
        else:
            dy, dbias = C().bias_act_bwd(dout.contiguous(), None, None, a, aid, has_bias, slot)
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
        seed, stream = get_rng().next(x.device)
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


# ----------------------------------------------------------------- linear (direct grad write)
class _LinearFn(torch.autograd.Function):
    """y = x W^T (+ b).  Backward writes dW (one GEMM) and db (one column-sum
    kernel) straight into the parameters' flat gradient slots.  fp32 runs: the fp16x3 GEMMs
    (ops/gemm16.py); --precision bf16: the same kernel's bf16 variant; --fp32-gemm native and
    shapes without a tile (heads narrower than 64 outputs): the library fp32 / bf16 GEMM."""

    @staticmethod
    def forward(ctx, x, W, b, mbox):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.f16 = gemm16.ok(x2, W.shape[0])
        ctx.W, ctx.b, ctx.mbox, ctx.xshape = W, b, mbox, x.shape
        if ctx.f16:   # fp32 operands split inside the GEMM kernels
            x2 = gemm16.rows2(x)
            ctx.xparts = gemm16.amax(x, x2)
            ctx.xcols = gemm16.cols_peek(x)
            xp = gemm16.take_pieces(x)   # the LayerNorm's pre-split copy of x, if it wrote one
            y, wt, ctx.wparts = gemm16.linear(x2 if xp is None else xp, ctx.xparts, W, b)
            ctx.save_for_backward(x2, wt)
            return y.view(*x.shape[:-1], y.shape[-1])
        Wc = cast_w(W, x.dtype)
        ctx.b16 = gemm16.bf16_ok(x2, W.shape[0], W.shape[1]) and Wc.is_contiguous()
        ctx.wt_b16 = None
        if ctx.b16:   # --precision bf16 on the hand-written kernel (bias in the epilogue)
            y = gemm16.mm_bf16(gemm16.rows2(x), Wc, bias=b)
            if ctx.needs_input_grad[0]:
                ctx.wt_b16 = gemm16.bf16_wt(W)   # the forward's batched W^T, for the data gradient
        else:
            y = torch.mm(x2, Wc.t()) if b is None else torch.addmm(cast_w(b, x.dtype), x2, Wc.t())
        ctx.save_for_backward(x2, Wc)
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        if ctx.f16:
            return _linear_backward_f16(ctx, dy)
        x2, _ = ctx.saved_tensors
        W, b = ctx.W, ctx.b
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not ctx.needs_input_grad[0]:
            dx = None
        elif ctx.b16:
            dx = _dgrad_bf16(dy2, W, ctx.xshape, ctx.mbox, ctx.wt_b16)
        else:
            dx = _dgrad(dy2, W, ctx.xshape, ctx.mbox)
        slot = grad_slot(W)
        side = side_begin(dy2.device, dy2.shape[0]) if slot is not None else None
        with side_ctx(side):
            dW = _wgrad(dy2, x2, slot)
            db = None
            if b is not None:
                if dy2.shape[-1] % 4 == 0:
                    db = C().colsum(dy2.contiguous(), None, grad_slot(b))
                else:
                    db = dy2.float().sum(0)
        if side is not None:
            dy2.record_stream(side)
            x2.record_stream(side)
        return dx, dW, db, None


def _record(side, *ts):
    """``record_stream(side)`` on every tensor a side-stream weight gradient reads -- operands and
    their scale sources (per-row / per-column max partials, which may be fresh allocations held
    only by an attribute): without it the caching allocator could hand their memory to the
    compute stream while the side-stream kernel still reads it.  Non-tensors (None, the LayerNorm's
    ('affine', ...) column bound) are skipped."""
    if side is None:
        return
    for t in ts:
        if torch.is_tensor(t):
            t.record_stream(side)
        elif isinstance(t, (tuple, list)):
            for u in t:
                if torch.is_tensor(u):
                    u.record_stream(side)


def _f16_dgrad(dy2, dparts, wt, wparts, xshape, mbox):
    """``_dgrad`` on the fp16x3 GEMM: beta = 1 into the deposited residual gradient if any."""
    K = xshape[-1]
    if mbox is not None:
        g, other = mbox.take(torch.float32)
        if g is not None:
            return gemm16.dgrad(dy2, dparts, wt, wparts, acc=g.view(-1, K)).view(xshape)
        dx = gemm16.dgrad(dy2, dparts, wt, wparts).view(xshape)
        return dx if other is None else dx + other.view(xshape).to(dx.dtype)
    return gemm16.dgrad(dy2, dparts, wt, wparts).view(xshape)


def _linear_backward_f16(ctx, dy):
    x2, wt = ctx.saved_tensors
    W, b = ctx.W, ctx.b
    dy2 = gemm16.rows2(dy)
    dparts = gemm16.amax(dy, dy2)
    dcols = gemm16.cols(dy, dy2)
    dp = gemm16.take_pieces(dy)
    xcols = ctx.xcols if ctx.xcols is not None else gemm16.cols(x2, x2)
    dx = (_f16_dgrad(dy2 if dp is None else dp, dparts, wt, ctx.wparts, ctx.xshape, ctx.mbox)
          if ctx.needs_input_grad[0] else None)
    slot = grad_slot(W)
    side = side_begin(dy2.device, dy2.shape[0]) if slot is not None else None
    with side_ctx(side):
        dW = gemm16.wgrad(dy2, dcols, x2, xcols, W.shape[0], W.shape[1], slot)
        db = None
        if b is not None:
            db = C().colsum(dy2, None, grad_slot(b)) if dy2.shape[-1] % 4 == 0 else dy2.sum(0)
    _record(side, dy2, x2, dparts, ctx.xparts, dcols, xcols)
    return dx, dW, db, None


def linear(x, W, b=None, res_grad=None):
    """F.linear with direct-to-slot weight/bias gradients on the GPU;
    ``res_grad``: see ``ResidualGrad``."""
    if use_kernels(x):
        return _LinearFn.apply(x, W, b, res_grad)
    return F.linear(x, cast_w(W, x.dtype), cast_w(b, x.dtype))


# ----------------------------------------------------------------- FFN block (fp16x3)
class _FFNFn(torch.autograd.Function):
    """y2 = gelu(x W1^T + b1) W2^T for fp32 runs as one autograd node: the FFN-up GEMM's
    epilogue applies bias + GELU (hetseq/bert_modeling.py:166-168, :409) and writes gelu(u) with
    its max |.| partials -- the FFN-down GEMM's operand -- and gelu'(u) for the backward, whose
    FFN-down data-gradient epilogue applies the GELU backward and the FFN-up bias gradient (:419):
    no separate bias / activation pass in either direction."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, mbox):
        x2 = gemm16.rows2(x)
        xparts = gemm16.amax(x, x2)
        ctx.xcols = gemm16.cols_peek(x)
        xp = gemm16.take_pieces(x)
        d, h, hparts, hcols, w1t, p1 = gemm16.gemm_gelu(x2 if xp is None else xp, xparts, W1, b1)
        y2, w2t, p2 = gemm16.linear(h, hparts, W2)
        ctx.save_for_backward(x2, d, h, w1t, w2t)
        ctx.parts = (xparts, hparts, p1, p2)
        ctx.hcols = hcols
        ctx.W, ctx.b1, ctx.mbox, ctx.xshape = (W1, W2), b1, mbox, x.shape
        return y2.view(*x.shape[:-1], y2.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        return _ffn_backward_f16(ctx, dy)


def _ffn_backward_f16(ctx, dy):
    x2, d, h, w1t, w2t = ctx.saved_tensors
    xparts, hparts, p1, p2 = ctx.parts
    W1, W2 = ctx.W
    dy2 = gemm16.rows2(dy)
    dparts = gemm16.amax(dy, dy2)
    dcols = gemm16.cols(dy, dy2)
    dp = gemm16.take_pieces(dy)
    slot2, slot1 = grad_slot(W2), grad_slot(W1)
    # each weight gradient on the side stream, beside the next data-gradient GEMM
    side = side_begin(dy2.device, dy2.shape[0]) if slot2 is not None and slot1 is not None else None
    with side_ctx(side):
        dW2 = gemm16.wgrad(dy2, dcols, h, ctx.hcols, W2.shape[0], W2.shape[1], slot2)
    _record(side, dy2, dparts, h, hparts, ctx.hcols, dcols)
    # GELU backward in the FFN-down data-gradient epilogue: t = (dy W2) * gelu'(u), d b1
    t, tparts, tcols, db1 = gemm16.gemm_dgelu(dy2 if dp is None else dp, dparts, w2t, p2, d, grad_slot(ctx.b1))
    if side is not None:
        side = side_begin(dy2.device, dy2.shape[0])   # after t
    xcols = ctx.xcols if ctx.xcols is not None else gemm16.cols(x2, x2)
    with side_ctx(side):
        dW1 = gemm16.wgrad(t, tcols, x2, xcols, W1.shape[0], W1.shape[1], slot1)
    _record(side, t, tparts, tcols, x2, xparts, xcols)
    dx = _f16_dgrad(t, tparts, w1t, p1, ctx.xshape, ctx.mbox)
    return dx, dW1, db1, dW2, None


class _FFNBf16Fn(torch.autograd.Function):
    """``_FFNFn`` for --precision bf16 on the same kernel's bf16 variant: the FFN-up epilogue adds
    the bias and writes gelu(u) and gelu'(u) in bf16; the FFN-down data gradient's epilogue
    multiplies by gelu'(u) and sums the FFN-up bias gradient (no bias_act pass either way)."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, mbox):
        x2 = gemm16.rows2(x)
        d, h = C().gemm_bf16_gelu(x2, cast_w(W1, torch.bfloat16), b1)
        y2 = gemm16.mm_bf16(h, cast_w(W2, torch.bfloat16))
        # the forward's batched W^T copies (one launch per forward) for the data gradients
        ctx.save_for_backward(x2, d, h, gemm16.bf16_wt(W1), gemm16.bf16_wt(W2))
        ctx.W, ctx.b1, ctx.mbox, ctx.xshape = (W1, W2), b1, mbox, x.shape
        return y2.view(*x.shape[:-1], y2.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, d, h, w1t, w2t = ctx.saved_tensors
        W1, W2 = ctx.W
        dy2 = gemm16.rows2(dy)
        dW2 = _wgrad(dy2, h, grad_slot(W2))
        t, db1 = C().gemm_bf16_dgelu(dy2, w2t, d, grad_slot(ctx.b1))
        dW1 = _wgrad(t, x2, grad_slot(W1))
        dx = _dgrad_bf16(t, None, ctx.xshape, ctx.mbox, w1t)
        return dx, dW1, db1, dW2, None


class _FFNBf16LibFn(torch.autograd.Function):
    """``_FFNBf16Fn`` with every product on hipBLASLt and the bias + GELU (and its backward with
    the bias gradient) as one bandwidth-bound pass each: in bf16 the library products plus the
    separate passes (u 70 + bias_gelu ~35 us; dgrad 65 + bias_gelu backward ~50) beat the
    hand-written kernel's fused GELU epilogues (185 / 152 us at the FFN shape, r5m)."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, mbox):
        x2 = gemm16.rows2(x)
        u = gemm16.mm_bf16(x2, cast_w(W1, torch.bfloat16))
        h = C().bias_act_fwd(u, b1, ACT_IDS['gelu'])
        y2 = gemm16.mm_bf16(h, cast_w(W2, torch.bfloat16))
        ctx.save_for_backward(x2, u, h, gemm16.bf16_wt(W1), gemm16.bf16_wt(W2))
        ctx.W, ctx.b1, ctx.mbox, ctx.xshape = (W1, W2), b1, mbox, x.shape
        return y2.view(*x.shape[:-1], y2.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, u, h, w1t, w2t = ctx.saved_tensors
        W1, W2 = ctx.W
        dy2 = gemm16.rows2(dy)
        dW2 = _wgrad(dy2, h, grad_slot(W2))
        dh = gemm16.mm_bf16(dy2, w2t)
        t, db1 = C().bias_act_bwd(dh, u, ctx.b1, None, ACT_IDS['gelu'], True, grad_slot(ctx.b1))
        dW1 = _wgrad(t, x2, grad_slot(W1))
        dx = _dgrad_bf16(t, None, ctx.xshape, ctx.mbox, w1t)
        return dx, dW1, db1, dW2, None


def _ffn_bf16_ok(x, W1, b1, W2):
    x2 = x.reshape(-1, x.shape[-1])
    return (b1 is not None and b1.dtype == torch.float32 and b1.is_contiguous() and
            gemm16.bf16_ok(x2, W1.shape[0], W1.shape[1]) and W2.shape[0] % 64 == 0 and
            cast_w(W1, torch.bfloat16).is_contiguous() and cast_w(W2, torch.bfloat16).is_contiguous())


def ffn_fusable(x, W1, b1, W2):
    """The fused FFN path applies: fp32 GPU activations on the fp16x3 GEMMs, or bf16 GPU
    activations (--precision bf16) on the bf16 variant."""
    if x.dtype == torch.bfloat16:
        return _ffn_bf16_ok(x, W1, b1, W2)
    return b1 is not None and gemm16.ok(x.reshape(-1, x.shape[-1]), W1.shape[0]) and W2.shape[0] % 64 == 0


def ffn(x, W1, b1, W2, res_grad=None):
    """gelu(x W1^T + b1) W2^T (the output bias / dropout / residual / LayerNorm follow)."""
    if x.dtype == torch.bfloat16:
        return (_FFNBf16LibFn if gemm16.bf16_lib() else _FFNBf16Fn).apply(x, W1, b1, W2, res_grad)
    return _FFNFn.apply(x, W1, b1, W2, res_grad)


# ----------------------------------------------------------------- fused Q/K/V projection
_ADJ = {}   # (data_ptr, shape, stride, dtype) of each tensor -> the view (built once per layout)


def _adjacent_view(ts):
    """If tensors ``ts`` are laid out back to back in one storage (FlatParamSpace
    guarantees it for Q/K/V), return a single [sum(rows), cols] view without copying.
    Views are cached by the tensors' addresses and shapes: the cached view holds its storage,
    so an address in the key cannot be reused by another allocation while the entry lives."""
    key = (tuple((t.data_ptr(), tuple(t.shape), t.stride(), t.dtype) for t in ts if t is not None)
           if ts[0] is not None else None)
    if key is not None and len(key) == len(ts):
        v = _ADJ.get(key)
        if v is not None:
            return v
    v = _adjacent_view_build(ts)
    if v is not None and key is not None and len(key) == len(ts):
        if len(_ADJ) >= 256:   # a model uses a few per layer; the bound caps what stale entries pin
            _ADJ.clear()
        _ADJ[key] = v
    return v


def _adjacent_view_build(ts):
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


def qkv_weight_view(wq, wk, wv):
    """The [3H, H] view of adjacent Q / K / V weights that linear3 multiplies by (None if the
    three are not laid out back to back)."""
    return _adjacent_view([wq, wk, wv])


def weight_pieces_scope(Ws, x):
    """Per-forward weight operands of the hand-written GEMMs for activations ``x`` [.., H]: every
    weight in ``Ws`` split into its fp16x3 pieces (fp32 runs, ``gemm16.weight_scope``) or
    transposed to bf16 (``--precision bf16``, ``gemm16.bf16_scope``) in one launch pair; a no-op
    context otherwise."""
    import contextlib
    if not torch.is_tensor(x) or not use_kernels(x):
        return contextlib.nullcontext()
    if x.dtype == torch.bfloat16:
        return gemm16.bf16_scope(Ws)   # W^T copies for the data gradients
    if x.dtype == torch.float32 and gemm16.enabled():
        return gemm16.weight_scope(Ws)
    return contextlib.nullcontext()


class _Linear3Fn(torch.autograd.Function):
    """y = x @ [Wq;Wk;Wv]^T + [bq;bk;bv] as ONE GEMM (N = 3H)."""

    @staticmethod
    def forward(ctx, x, wq, wk, wv, bq, bk, bv, mbox, bgrad=True):
        has_b = bq is not None
        ctx.bgrad = bgrad   # False: the bias gradient comes from the consumer (the fused attention)
        W = _adjacent_view([wq, wk, wv])
        if W is None:
            W = torch.cat([wq, wk, wv], 0)
        b = None
        if has_b:
            b = _adjacent_view([bq, bk, bv])
            if b is None:
                b = torch.cat([bq, bk, bv], 0)
        x2 = x.reshape(-1, x.shape[-1])
        ctx.params = (wq, wk, wv, bq, bk, bv)
        ctx.has_b, ctx.mbox, ctx.xshape = has_b, mbox, x.shape
        ctx.n = [wq.shape[0], wk.shape[0], wv.shape[0]]
        ctx.f16 = gemm16.ok(x2, W.shape[0])
        if ctx.f16:   # fp32 runs: the fp16x3 GEMM
            x2 = gemm16.rows2(x)
            ctx.xparts = gemm16.amax(x, x2)
            ctx.xcols = gemm16.cols_peek(x)
            xp = gemm16.take_pieces(x)   # the LayerNorm's pre-split copy of x, if it wrote one
            y, wt, ctx.wparts = gemm16.linear(x2 if xp is None else xp, ctx.xparts, W, b)
            ctx.save_for_backward(x2, wt)
            return y.view(*x.shape[:-1], y.shape[-1])
        Wc, bc = W, b
        if x.dtype != W.dtype:
            sh = [getattr(t, '_hx_bf16', None) for t in (wq, wk, wv)]
            Wc = _adjacent_view(sh) if all(t is not None for t in sh) else None
            Wc = Wc if Wc is not None else W.to(x.dtype)
            bc = cast_w(b, x.dtype) if has_b else None
        ctx.b16 = gemm16.bf16_ok(x2, W.shape[0], W.shape[1]) and Wc.is_contiguous()
        ctx.wt_b16 = None
        if ctx.b16:
            y = gemm16.mm_bf16(gemm16.rows2(x), Wc, bias=b if has_b else None)
            if ctx.needs_input_grad[0]:
                ctx.wt_b16 = gemm16.bf16_wt(W)   # the forward's batched W^T, for the data gradient
        else:
            y = torch.addmm(bc, x2, Wc.t()) if has_b else torch.mm(x2, Wc.t())
        ctx.save_for_backward(x2, Wc)
        return y.view(*x.shape[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, W = ctx.saved_tensors
        wq, wk, wv, bq, bk, bv = ctx.params
        n_out, n_in = sum(ctx.n), x2.shape[1]
        if ctx.f16:
            # W holds W^T's fp16 pieces here; dx after the side-stream weight gradient is queued
            dy2 = gemm16.rows2(dy)
            dys = gemm16.amax(dy, dy2)
            dcols = gemm16.cols(dy, dy2)
            xcols = ctx.xcols if ctx.xcols is not None else gemm16.cols(x2, x2)
            dx = None
            wg = lambda slot: gemm16.wgrad(dy2, dcols, x2, xcols, n_out, n_in, slot)
        else:
            dy2 = dy.reshape(-1, dy.shape[-1])
            dys = None
            if not ctx.needs_input_grad[0]:
                dx = None
            elif ctx.b16:
                dx = _dgrad_bf16(dy2, None, ctx.xshape, ctx.mbox, ctx.wt_b16)
            else:
                dx = _dgrad(dy2, W, ctx.xshape, ctx.mbox)
            wg = lambda slot: _wgrad(dy2, x2, slot)
        a, b_, _ = ctx.n
        # weight grads: ONE GEMM straight into the three adjacent flat slots when possible
        ws = [grad_slot(w) for w in (wq, wk, wv)]
        fused = _adjacent_view(ws) if all(t is not None for t in ws) else None
        has_b = ctx.has_b and ctx.bgrad
        bs = [grad_slot(t) for t in (bq, bk, bv)] if has_b else [None, None, None]
        fb = _adjacent_view(bs) if all(t is not None for t in bs) else None
        direct = fused is not None and (fb is not None or not has_b)
        side = side_begin(dy2.device, dy2.shape[0]) if direct else None
        with side_ctx(side):
            if fused is not None:
                wg(fused)
                gW = ws
            else:
                dW = wg(None)
                gW = [dW[:a], dW[a:a + b_], dW[a + b_:]]
                for k, t in enumerate(ws):
                    if t is not None:
                        t.copy_(gW[k])
                        gW[k] = t
            db = None
            if has_b:
                if use_kernels(dy2) and dy2.shape[-1] % 4 == 0:
                    db = C().colsum(dy2.contiguous(), None, fb)
                else:
                    db = dy2.float().sum(0)
        if ctx.f16:
            _record(side, dy2, x2, dys, ctx.xparts, dcols, xcols)
        else:
            _record(side, dy2, x2)
        if ctx.f16 and ctx.needs_input_grad[0]:
            dx = _f16_dgrad(dy2, dys, W, ctx.wparts, ctx.xshape, ctx.mbox)
        if not has_b:
            return (dx, gW[0], gW[1], gW[2], None, None, None, None, None)
        gb = bs if fb is not None else [db[:a], db[a:a + b_], db[a + b_:]]
        return (dx, gW[0], gW[1], gW[2], gb[0], gb[1], gb[2], None, None)


def linear3(x, wq, wk, wv, bq, bk, bv, res_grad=None, bias_grad=True):
    """The fused Q/K/V projection (``res_grad``: see ``ResidualGrad``).  ``bias_grad=False``: the
    bias is added in the GEMM epilogue but its gradient is produced by the consumer (``attention``
    with ``bias_grad=(bq, bk, bv)``: the column sums of dQKV from the attention backward's
    registers) -- this function then returns none for it."""
    return _Linear3Fn.apply(x, wq, wk, wv, bq, bk, bv, res_grad, bool(bias_grad))


# ----------------------------------------------------------------- attention core
def attention(qkv, mask_bias, num_heads, p, training, bias=None, bias_grad=None):
    """softmax(Q K^T / sqrt(d) + mask) -> dropout -> @ V  on the packed [B, S, 3H]
    projection; returns [B, S, H] (reference BertSelfAttention, :351-377).
    ``mask_bias`` is the additive [B, S] key mask ((1 - m) * -10000); ``bias`` the
    optional (bq, bk, bv) of a bias-less QKV projection, added inside the kernel
    (``HX_QKV_BIAS_EPILOGUE=0``);
    ``bias_grad`` the (bq, bk, bv) already in ``qkv`` (``linear3(..., bias_grad=False)``):
    only their gradient is produced here."""
    from .flash_attention import attention as _attention
    return _attention(qkv, mask_bias, num_heads, p if training else 0.0, bias, bias_grad)


# ----------------------------------------------------------------- MLM decoder + softmax-xent
class _DecoderXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, W, bias, labels):
        V, H = W.shape
        # the vocabulary padded to a multiple of 768 with zero weight rows (whole 192 / 256 tiles
        # of the hand-written GEMMs; the padding logits are exactly 0 and never read as logits)
        Vp = (V + 767) // 768 * 768
        ctx.f16 = gemm16.ok(h, 64) and h.is_contiguous() and H % 64 == 0
        ctx.b16 = False
        if ctx.f16:   # fp32 runs: the fp16x3 GEMM
            Wd = W.detach()
            if Wd.is_contiguous() and Wd.data_ptr() % 16 == 0:   # padding rows read as zero, no copy
                wf, wt, wrow, wcol = C().split_weight_f16([Wd], [Vp])[0]
            else:
                wf, wt, wrow, wcol = C().split_weight_f16([_padded_rows(W, Vp)])[0]
            full = gemm16.mm(h, gemm16.amax(h, h), wf, wrow)
            ctx.wpieces = (wt, wcol)
        elif gemm16.bf16_ok(h, 64, H) and h.is_contiguous():
            # --precision bf16 on the hand-written kernel (bf16 logits)
            ctx.b16 = True
            full = gemm16.mm_bf16(h, _padded_rows(cast_w(W, torch.bfloat16), Vp))
        else:
            full = torch.mm(h, cast_w(W, h.dtype).t())
        logits = full[:, :V]
        loss_rows = C().softmax_xent_(logits, bias, labels, -1)   # logits <- softmax - onehot
        count = (labels != -1).sum().to(torch.float32)
        loss = loss_rows.sum() / count
        ctx.save_for_backward(h, full, count)
        ctx.params = (W, bias)
        return loss

    @staticmethod
    def backward(ctx, g):
        if ctx.f16:
            return _decoder_backward_f16(ctx, g)
        h, dl_full, count = ctx.saved_tensors
        W, bias = ctx.params
        dl = dl_full[:, :W.shape[0]]
        # d loss / d logits = (softmax - onehot) * g / count.  The scale stays a
        # device scalar (no host sync) and is applied to the small operands -- the
        # bias column sum's result, dh (M x H) and h (M x H) -- never to the
        # M x V gradient itself (a 312 MB rewrite at B=128).
        scale = (g.float() / count).reshape(1)
        dbias = C().colsum(dl, scale, grad_slot(bias) if bias is not None else None)
        hs = h * scale.to(h.dtype)
        slot = grad_slot(W)
        if ctx.b16:
            # dl over the padded vocabulary (padding columns 0) against the padded W^T in bf16
            wt = C().weight_bf16_t([_padded_rows(W, dl_full.shape[1])])[0]
            dh = gemm16.mm_bf16(dl_full, wt).mul_(scale.to(dl.dtype))
        else:
            dh = torch.mm(dl, cast_w(W, dl.dtype)).mul_(scale.to(dl.dtype))
        side = side_begin(dl.device, dl.shape[0]) if slot is not None else None
        with side_ctx(side):
            if ctx.b16 and C().wgrad_bf16_ok(dl_full, hs):
                # over the padded vocabulary (whole 128-row tiles); rows past V are not stored
                out = slot if slot is not None else torch.empty(W.shape[0], hs.shape[1], device=dl.device)
                dW = C().wgrad_bf16(dl_full, hs, out)
            else:
                dW = _wgrad(dl, hs, slot)
        if side is not None:
            dl.record_stream(side)
            hs.record_stream(side)
        return dh, dW, dbias, None


_PAD = {}


def _padded_rows(W, rows):
    """W [V, H] copied into a cached zero-padded [rows, H] buffer of W's dtype (the padding rows
    stay 0)."""
    key = (W.device, rows, W.shape[1], W.dtype)
    buf = _PAD.get(key)
    if buf is None:
        buf = _PAD[key] = torch.zeros(rows, W.shape[1], device=W.device, dtype=W.dtype)
    buf[:W.shape[0]].copy_(W.detach())
    return buf


def _decoder_backward_f16(ctx, g):
    h, dl_full, count = ctx.saved_tensors
    Wt, bias = ctx.params
    wt, wparts = ctx.wpieces
    V = Wt.shape[0]
    dl = dl_full[:, :V]
    scale = (g.float() / count).reshape(1)
    dbias = C().colsum(dl, scale, grad_slot(bias) if bias is not None else None)
    # |softmax - onehot| <= 1: a constant bound is a valid max |dl| for the fp16 split
    one = gemm16.bound(dl_full.device)
    # dh = dl . W over the padded vocabulary (split-K slabs: 40 output tiles alone would idle the CUs)
    dh = gemm16.mm(dl_full, one, wt, wparts, ks=0).mul_(scale)
    hs = h * scale.to(h.dtype)
    slot = grad_slot(Wt)
    # per-column scales: dl's columns are the vocabulary (rare words' probabilities sit far below
    # the tensor's max), hs's the hidden features -- one column-max pass each
    dW = gemm16.wgrad(dl_full, gemm16.cols(dl_full, dl_full), hs, gemm16.cols(hs, hs), V, h.shape[1], slot)
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
