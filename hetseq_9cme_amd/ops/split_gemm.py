"""fp32 GEMMs on the bf16 matrix cores: split-plane emulation (``--fp32-gemm``).

gfx950 has no TF32/xf32; its f32-input MFMA runs at the f32 vector rate,
157 TF/s, 1/16 of the 2.5 PF/s bf16 MFMA rate.  The fp32 training path of
round 1 spent ~59 of its 68 ms per BERT-base step in library fp32 GEMMs at
~94 % of that rate -- fp32 MFMA was the ceiling.  This module breaks it while
keeping fp32-class results:

    x = x0 + x1 (+ x2) + r,  x_i bf16 (round-to-nearest), |r| <= 2^-17 |x| (2^-26 |x|)

and a product a.b is a sum of piece products, each exact in the MFMA's fp32
accumulator:

  ``bf16x3``: a0 b0 + a1 b0 + a0 b1                        (3 bf16 GEMM passes)
  ``bf16x6``: + a2 b0 + a1 b1 + a0 b2                      (6 passes, fp32-exact class)

Measured on MI355X against fp64 (``tools/bench_split_gemm.py``, BERT-base
shapes, max |err| / sum|a.b|): native fp32 MFMA 3.7-4.5e-7, bf16x6 4.4-5.5e-7,
bf16x3 0.7-1.5e-6 -- all three far from TF32 (~1e-3 relative per product).

Pass structure.  The planes of an operand are stored next to each other along
the GEMM's REDUCTION dimension, so one ordinary bf16 x bf16 -> fp32 GEMM with
K' = passes x K sums all the pass products.  Which piece sits in which plane
is fixed per role so the three GEMMs of a linear layer pair the right pieces:

  role                          layout              piece order
  layer input x (A of fwd,      [T, n, K]           P  (bf16x3: 0 1 0)
    B of wgrad)                                        (bf16x6: 0 1 0 2 1 0)
  output grad dy (A of dgrad,   [T, n, N]           Q  (bf16x3: 0 0 1)
    A of wgrad)                                        (bf16x6: 0 0 1 0 1 2)
  weight W, forward operand     [N, n, K]           Q
  weight W, dgrad operand       [n, N, K] stacked   P

  forward  y  = x' [T, nK] . W_Q'^T          pairs (P_j, Q_j)
  dgrad    dx = dy' [T, nN] . W_P'' [nN, K]  pairs (Q_j, P_j)
  wgrad    dW = dy'^T . x'  over nT rows     pairs (Q_j, P_j)   ([T, n, D] viewed as [nT, D])

Every pairs column is {(0,0), (1,0), (0,1)} (bf16x6: plus (2,0), (1,1), (0,2)).
The weight-gradient GEMM runs on a hand-written split-K kernel
(``csrc/kernels/wgrad_split.hip``) that stages each DISTINCT piece of a token
block once and runs all passes from registers (the stacked [nT, D] views would
stream dY_0 twice / X_0 three times); shapes it does not cover take the stacked
form through ``wgrad_bf16.hip`` or the library.
"""
import os

import torch

from ._ext import C, use_kernels

PIECES = {3: 2, 6: 3}
ORDER_P = {3: (0, 1, 0), 6: (0, 1, 0, 2, 1, 0)}
ORDER_Q = {3: (0, 0, 1), 6: (0, 0, 1, 0, 1, 2)}
MODES = {'native': 0, 'bf16x3': 3, 'bf16x6': 6, 'fp16x3': 0}   # fp16x3: ops/gemm16.py
# Prefix form (see ``prefix_mm``): the large operand holds each distinct piece once, in
# natural order, and the weight operand piece j repeated npc - j times.
ORDER_N = {3: (0, 1), 6: (0, 1, 2)}
ORDER_W_PREFIX = {3: (0, 0, 1), 6: (0, 0, 0, 1, 1, 2)}


# Below this many rows (tokens of the GEMM's M side) the split GEMMs lose to native f32
# MFMA (smaller grids, split overhead).  BERT-base at 32 x 128 = 4096 tokens: 19.7 ms/step on
# the bf16x6 path vs 21.2 ms native (round 2, after the NT-form data gradients and the LDS-DMA
# weight-gradient kernel; it was 22.6 vs 21.2 before them); NER fine-tuning batches (~1000
# tokens) still run faster native (10.8 vs 12.9 ms/update).  Both are fp32-exact class, so
# small GEMMs (MLM head on the masked rows, pooler, small batches) simply stay native.
MIN_ROWS = {3: 2048,
            6: int(os.environ.get('HETSEQ_SPLIT_MIN_ROWS_X6', '4096'))}


_SPLITK = True        # split-K slabs for deep, narrow library products (the MLM decoder's dgrad)
_WGRAD_GROUP = True   # two weight gradients over the same tokens in one launch
_PREFIX_GEMM = True   # prefix form for the deep 4H -> H library products


class _State(object):
    passes = 0
    piece_gemm = {'1': True, '0': False}.get(os.environ.get('HETSEQ_PIECE_GEMM', ''))   # see nt_ok
    addmm_out_ok = None   # does torch.addmm(bf16, bf16, out_dtype=fp32, out=acc) work in place?
    wp = None   # {(data_ptr, shape): (wf, wt)} of the running forward's batch split (weight_pieces_scope)


def set_fp32_gemm(mode):
    """'native' (fp32 MFMA through the libraries), 'bf16x3', 'bf16x6' or 'fp16x3' (three fp16
    piece products on fp32 operands split in the GEMM kernels: ops/gemm16.py)."""
    from . import gemm16
    if mode not in MODES:
        raise ValueError('--fp32-gemm must be one of {}'.format(sorted(MODES)))
    _State.passes = MODES[mode]
    gemm16.set_enabled(mode == 'fp16x3')


def fp32_gemm_mode():
    from . import gemm16
    if gemm16.enabled():
        return 'fp16x3'
    return {3: 'bf16x3', 6: 'bf16x6', 0: 'native'}[_State.passes]


def attention_split(x2):
    """Does the fp32 attention run its products on the bf16 matrix cores (attention_x6.hip) for
    the [rows, 3H] projection ``x2``: bf16x6 / bf16x3 whenever the linears split, fp16x3 from the
    same row count (the attention kernels stay bf16x6-class under every split mode)."""
    from . import gemm16
    if active(x2):
        return True
    rows = x2.numel() // max(1, x2.shape[-1])
    return gemm16.enabled() and x2.dtype == torch.float32 and use_kernels(x2) and rows >= MIN_ROWS[6]


def active(x, n_out=None):
    """Split emulation applies to fp32 GPU operands [rows, features] when a split mode is
    set and the GEMM is big enough to fill the chip on the bf16 path: at least
    ``MIN_ROWS`` rows, or a wide output (``n_out`` >= 8192, the MLM decoder's vocabulary)."""
    if not (_State.passes > 0 and x.dtype == torch.float32 and use_kernels(x)):
        return False
    rows = x.numel() // max(1, x.shape[-1])
    return rows >= MIN_ROWS[_State.passes] or (n_out is not None and n_out >= 8192 and rows >= 256)


def passes():
    return _State.passes


def planes(x2, order, stacked=False, rpad=0, dpad=0):
    """bf16 planes of the fp32 matrix ``x2`` [R, D]: [R, n*Dp] interleaved, or
    [n*Rp, Dp] stacked, rows / columns zero-padded to ``rpad`` / ``dpad``."""
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    return C().split_planes(x2, list(order), max(order) + 1, bool(stacked), int(rpad), int(dpad))


def forward(x2, W, rpad=0):
    """y = x2 @ W^T in fp32; returns (y, x planes for the backward).  ``rpad``: W's rows
    zero-padded to this count (y gets rpad columns, the padding ones exactly 0)."""
    n = _State.passes
    xs = planes(x2, ORDER_P[n])
    wq = planes(W, ORDER_Q[n], rpad=rpad)
    return torch.mm(xs, wq.t(), out_dtype=torch.float32), xs


def forward_planes(xs, W):
    """y = x @ W^T from x's planes (already split, e.g. by a fused producer)."""
    return torch.mm(xs, planes(W, ORDER_Q[_State.passes]).t(), out_dtype=torch.float32)


ACT_IDS = {'gelu': 0, 'tanh': 1, 'relu': 2, 'none': 3}


def act_planes(y, b, act, order=None):
    """Planes (order P, or ``order``) of act(y + b): the bias-activation epilogue writes the
    next GEMM's input pieces directly (csrc/kernels/elementwise.hip ``bias_act_planes_k``)."""
    n = _State.passes
    return C().bias_act_planes(y, b, None, ACT_IDS[act], list(order or ORDER_P[n]), PIECES[n], None)[0]


def act_grad_planes(dout, y, b, act, dbias_out=None, order=None):
    """(planes (order Q, or ``order``) of dout * act'(y + b), dbias) in one pass."""
    n = _State.passes
    return C().bias_act_planes(y, b, dout, ACT_IDS[act], list(order or ORDER_Q[n]), PIECES[n], dbias_out)


def grad_planes(dy2, dpad=0):
    return planes(dy2, ORDER_Q[_State.passes], dpad=dpad)


def weight_planes_t(W, rpad=0, order=None):
    """Transposed dgrad operand [K, n * Np] (order P, or ``order``, over W's rows, zero-padded
    to ``rpad``), or None when W's shape does not fit the transposing kernel (64-multiples)."""
    N, K = W.shape
    Np = max(N, rpad)
    if K % 64 or Np % 64 or W.stride(-1) != 1 or W.stride(0) % 4 or W.data_ptr() % 16:
        return None
    n = _State.passes
    return C().split_planes_t(W, list(order or ORDER_P[n]), PIECES[n], int(rpad))


def _splitk(m, n, k):
    """Reduction slabs for a product with few 256 x 256 output tiles and a deep reduction
    (1 = none): enough slabs for ~512 tiles, each slab >= 8192 deep and a multiple of 64."""
    tiles = ((m + 255) // 256) * ((n + 255) // 256)
    if tiles >= 64 or k < 65536 or not _SPLITK:
        return 1
    for s in (16, 12, 8, 4, 2):
        if tiles * s <= 768 and k % (64 * s) == 0 and k // s >= 8192:
            return s
    return 1


def dgrad(dys, W, acc=None, rpad=0):
    """dy @ W (fp32) from the dy planes; accumulated into ``acc`` (beta = 1) if given.
    ``rpad``: dy's planes were column-padded to this width (W's rows are padded to match).

    The weight operand is W^T's planes [K, n * Np], so the product runs in NT form (both
    operands contiguous along the reduction dimension, like the forward GEMM): 7-15 %
    faster than the NN product with W's stacked planes [n * Np, K] on MI355X
    (tools/probe/dgrad_layout_probe.py); other shapes keep the stacked form."""
    wt = weight_planes_t(W, rpad)
    wb = wt.t() if wt is not None else planes(W, ORDER_P[_State.passes], stacked=True, rpad=rpad)
    if acc is None:
        s = _splitk(dys.shape[0], wb.shape[1], wb.shape[0])
        if s > 1 and dys.is_contiguous():
            # narrow output, very deep reduction (the MLM decoder: 2560 x 768 from K' = 6 x 30720):
            # too few output tiles to fill the CUs, so the reduction is cut into s slabs run as
            # one strided batched GEMM, partial products summed after (1051 -> 580 us,
            # tools/probe/decoder_gemm_probe.py)
            kc = wb.shape[0] // s
            a = dys.view(dys.shape[0], s, kc).transpose(0, 1)
            return torch.bmm(a, wb.view(s, kc, wb.shape[1]), out_dtype=torch.float32).sum(0)
        return torch.mm(dys, wb, out_dtype=torch.float32)
    if _State.addmm_out_ok is not False:
        try:
            r = torch.addmm(acc, dys, wb, out_dtype=torch.float32, out=acc)
            _State.addmm_out_ok = True
            return r
        except (RuntimeError, TypeError):
            _State.addmm_out_ok = False
    return acc.add_(torch.mm(dys, wb, out_dtype=torch.float32))


# ---------------------------------------------------------------- pieces form (hand-written GEMMs)
# Operands stored as [rows, npc, D]: each DISTINCT piece once (npc = 2 for bf16x3, 3 for
# bf16x6) -- half the bytes of the pass-stacked planes for bf16x6, the fp32 size for bf16x3.
# The forward and data-gradient GEMMs run on csrc/kernels/gemm_split.hip (every piece
# fragment reused by all passes from registers), the weight gradient on wgrad_split.hip.

def npieces():
    return PIECES[_State.passes]


# Below this many rows the piece GEMMs' 256-row tiles leave CUs idle (4096 rows x N = 768: 64
# tiles for 256 CUs) and the library GEMMs on pass-stacked planes win: BERT-base at batch 32
# (4096 tokens) 24.4 ms/step on the piece GEMMs against 20.0 on the planes path; at batch 64
# (8192 tokens) the piece GEMMs win, 30.4 against 31.0 ms (profiles/r3_overlap_wgrad_ab.md).
PIECE_MIN_ROWS = int(os.environ.get('HX_PIECE_MIN_ROWS', '8192'))


def nt_ok(n_in, n_out, rows=None):
    """Use the hand-written piece GEMMs for a linear layer W [n_out, n_in] (fwd: N = n_out,
    K = n_in; dgrad: N = n_in, K = n_out) over ``rows`` tokens: the default under bf16x6 from
    ``PIECE_MIN_ROWS`` rows (csrc/kernels/gemm_split.hip, LDS-DMA pipeline, profiles/r3_*),
    opt-in for bf16x3 (``HETSEQ_PIECE_GEMM=1``) and off with ``HETSEQ_PIECE_GEMM=0``, where the
    library GEMMs on pass-stacked planes run instead."""
    on = _State.piece_gemm if _State.piece_gemm is not None else _State.passes == 6
    if rows is not None and rows < PIECE_MIN_ROWS and _State.piece_gemm is None:
        return False
    return on and n_out % 128 == 0 and n_in % 128 == 0


def producer_pieces(rows, H, ref):
    """Number of pieces a producer (LayerNorm / embedding forward) should write next to its fp32
    output [rows, H] on ``ref``'s device for a consuming piece-GEMM linear, or 0: the split path
    is on for this size (``active``'s rule) and the piece GEMMs take the shape (``nt_ok``)."""
    if not (_State.passes > 0 and use_kernels(ref) and rows >= MIN_ROWS[_State.passes] and nt_ok(H, 128, rows)):
        return 0
    return npieces()


def attach_pieces(out, pcs):
    """Hand ``pcs`` (pieces of ``out``, written by its producer) to the consumer linear."""
    if pcs is not None and pcs.numel():
        out._hx_pieces = pcs
        out._hx_pieces_ver = out._version
    return out


def input_pieces(x, x2):
    """Pieces of the linear input ``x`` (viewed as ``x2`` [rows, K]): the producer's, when it
    wrote them and ``x`` has not changed since, else split here."""
    pcs = getattr(x, '_hx_pieces', None)
    if pcs is not None and getattr(x, '_hx_pieces_ver', -1) == x._version and \
            pcs.shape == (x2.shape[0], npieces() * x2.shape[1]):
        return pcs
    return pieces(x2)


def pieces(x2):
    """[R, npc * D] bf16 pieces of the fp32 matrix ``x2`` [R, D] (piece p at column p * D)."""
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    n = npieces()
    return C().split_planes(x2, list(range(n)), n, False, 0, 0)


_B16_CACHE = {}


def b16(n):
    """Are the weight pieces that form the B operand of an n-column product stored in the B16
    layout [rows][K / 16][3][16] (csrc/kernels/gemm_split.hip, hx_gemm_split_weight_b16)?"""
    key = (n, _State.passes)
    v = _B16_CACHE.get(key)
    if v is None:
        v = _B16_CACHE[key] = bool(C().gemm_split_weight_b16(int(n), int(_State.passes)))
    return v


def _wmask(W):
    N, K = W.shape
    return (1 if b16(N) else 0) | (2 if b16(K) else 0)


def weight_pieces(W):
    """(wf [N, npc * K], wt [K, npc * N]): pieces of W [N, K] and of W^T, one pass; each in the
    layout its GEMM reads (``b16``: wf is the B operand of the N-column forward, wt of the
    K-column data gradient).  Inside ``weight_pieces_scope`` the batch split of the running
    forward is returned."""
    if _State.wp is not None:
        e = _State.wp.get((W.data_ptr(), tuple(W.shape)))
        if e is not None:
            return e
    return C().split_weight(W.contiguous(), npieces(), _wmask(W))


class weight_pieces_scope(object):
    """Split every weight in ``Ws`` in ONE launch (split.hip ``split_weight_many_k``) on entry;
    ``weight_pieces`` returns those pieces until exit.  Scoped to one forward: weights change
    between forwards (optimizer step) and a recompute under activation checkpointing runs
    outside the scope, so it splits again.  No-op for an empty list or outside bf16x3/x6."""

    def __init__(self, Ws):
        self.Ws = [W for W in Ws if W is not None]

    def __enter__(self):
        self.prev = _State.wp
        if self.Ws and _State.passes > 0 and len(self.Ws) <= 64 and \
                all(W.dim() == 2 and W.shape[0] % 64 == 0 and W.shape[1] % 64 == 0 and W.is_contiguous()
                    for W in self.Ws):
            outs = C().split_weight_many(self.Ws, npieces(), [_wmask(W) for W in self.Ws])
            _State.wp = {(W.data_ptr(), tuple(W.shape)): tuple(o) for W, o in zip(self.Ws, outs)}
        return self

    def __exit__(self, *exc):
        _State.wp = self.prev
        return False


def gemm(a, b, out=None, beta=False):
    """out (+)= sum over piece pairs of a_p . b_q^T, fp32 [M, N] (b = weight pieces from
    ``weight_pieces``, in the layout ``b16(N)`` says)."""
    return C().gemm_split(a, b, _State.passes, out, beta, 2 if b16(b.shape[0]) else 0)


def gemm_gelu(a, b, bias, deriv=False):
    """(u = a . b^T + bias, pieces of gelu(u)): the FFN-up GEMM with its GELU epilogue.
    ``deriv``: return gelu'(u) in place of u -- the only thing the backward needs, computed from
    the same erf as gelu(u), so the backward epilogue runs no erf / exp (gemm_dgelu(deriv=True))."""
    return C().gemm_split_gelu(a, b, _State.passes, bias, 2 if b16(b.shape[0]) else 0, 1 if deriv else 0)


def gemm_dgelu(a, b, u, bias, dbias_out, deriv=False):
    """(pieces of (a . b^T) * gelu'(u (+ bias)), d bias): the FFN-down data gradient with the
    GELU backward epilogue (``deriv``: ``u`` holds gelu'(u) from gemm_gelu(deriv=True))."""
    return C().gemm_split_dgelu(a, b, _State.passes, u, bias, dbias_out, 2 if b16(b.shape[0]) else 0,
                                1 if deriv else 0)


def dgrad_pieces(dys, wt, acc=None):
    """dy @ W from dy's pieces and W^T's pieces, accumulated into ``acc`` if given."""
    if acc is None:
        return gemm(dys, wt)
    return gemm(dys, wt, out=acc, beta=True)


def wgrad_pieces(dys, xs, n_out, n_in, slot):
    n = npieces()
    out = slot if slot is not None else torch.empty(n_out, n_in, device=dys.device)
    return C().wgrad_split(dys, [p * n_out for p in range(n)], xs, [p * n_in for p in range(n)], _State.passes,
                           n_out, n_in, out)


def wgrad_pieces_group(items):
    """Two weight gradients over the same tokens as ONE launch (wgrad_split.hip's grouped form):
    ``items`` = [(dys, xs, n_out, n_in, slot)] x 2, as for ``wgrad_pieces``.  Returns the two
    dW tensors, or None when the pair does not qualify (then run them one by one).
    (``_WGRAD_GROUP = False`` turns grouping off.)"""
    if _State.passes != 6 or not _WGRAD_GROUP:
        return None
    args, outs = [], []
    for dys, xs, n_out, n_in, slot in items:
        if not C().wgrad_split_ok(dys, xs, n_out, n_in):
            return None
        out = slot if slot is not None else torch.empty(n_out, n_in, device=dys.device)
        outs.append(out)
        args.append((dys, [0, n_out, 2 * n_out], xs, [0, n_in, 2 * n_in], n_out, n_in, out))
    return outs if C().wgrad_split_group(args) else None


def act_pieces(y, b, act):
    """Pieces of act(y + b) written by the bias-activation epilogue."""
    n = npieces()
    return C().bias_act_planes(y, b, None, ACT_IDS[act], list(range(n)), n, None)[0]


def act_grad_pieces(dout, y, b, act, dbias_out=None):
    """(pieces of dout * act'(y + b), dbias) in one pass."""
    n = npieces()
    return C().bias_act_planes(y, b, dout, ACT_IDS[act], list(range(n)), n, dbias_out)


def _piece_offsets(order, d):
    """Column offset of the first plane holding each distinct piece."""
    return [order.index(k) * d for k in range(len(set(order)))]


def wgrad(dys, xs, n_out, n_in, slot, dy_order=None, x_order=None):
    """dW [n_out, n_in] = sum over tokens and passes of dy-piece^T x-piece.  The
    split-piece kernel (csrc/kernels/wgrad_split.hip) stages each distinct piece once
    and runs all passes from registers; other shapes use the stacked-rows form.
    ``dy_order`` / ``x_order``: the operands' plane orders (default Q / P)."""
    n = _State.passes
    dy_order, x_order = dy_order or ORDER_Q[n], x_order or ORDER_P[n]
    if C().wgrad_split_ok(dys, xs, n_out, n_in):
        out = slot if slot is not None else torch.empty(n_out, n_in, device=dys.device)
        return C().wgrad_split(dys, _piece_offsets(dy_order, n_out), xs, _piece_offsets(x_order, n_in), n,
                               n_out, n_in, out)
    assert dy_order == ORDER_Q[n] and x_order == ORDER_P[n], 'stacked-rows wgrad needs the pass orders'
    from .fused import _wgrad
    return _wgrad(dys.view(-1, n_out), xs.view(-1, n_in), slot)


# ---------------------------------------------------------------- prefix form
def _prefix_on():
    return _PREFIX_GEMM


def prefix_ok(k, n_out):
    """The prefix form pays off for deep, narrow products (reduction k >= 2 x output
    width: the FFN-down forward and the FFN-up data gradient, k = 4H, n = H): half the plane
    bytes for the producer to write and the GEMM to read, against two extra passes over the
    fp32 output; measured 388 vs 420 us for the bare GEMMs at T=16384, k=3072, n=768 before
    the plane savings, slower for k = n (tools/probe/prefix_gemm_probe.py)."""
    return _prefix_on() and _State.passes > 0 and k >= 2 * n_out and k % 64 == 0 and n_out % 64 == 0


def prefix_mm(ap, wb, k, acc=None):
    """sum over piece pairs of A_a B_b from the prefix form: ``ap`` = the large operand's
    distinct pieces [R, npc * k] (natural order 0, 1, 2), ``wb`` = the weight operand
    [n * k, N] whose row blocks hold piece j repeated npc - j times (ORDER_W_PREFIX).
    Product j pairs the first npc - j pieces of A with B's piece j -- one library GEMM per
    piece of B over a column PREFIX of ``ap`` (no copy: lda = npc * k) -- accumulated with
    beta = 1 (into ``acc`` when given)."""
    npc = PIECES[_State.passes]
    c, off = acc, 0
    for j in range(npc):
        m = (npc - j) * k
        a, b = ap[:, :m], wb[off:off + m]
        off += m
        if c is None:
            c = torch.mm(a, b, out_dtype=torch.float32)
        elif _State.addmm_out_ok is not False:
            try:
                c = torch.addmm(c, a, b, out_dtype=torch.float32, out=c)
                _State.addmm_out_ok = True
            except (RuntimeError, TypeError):
                _State.addmm_out_ok = False
                c = c.add_(torch.mm(a, b, out_dtype=torch.float32))
        else:
            c = c.add_(torch.mm(a, b, out_dtype=torch.float32))
    return c


def forward_prefix(xp, W):
    """y = x @ W^T from x's natural-order pieces (prefix form)."""
    n = _State.passes
    return prefix_mm(xp, planes(W, ORDER_W_PREFIX[n]).t(), W.shape[1])


def dgrad_prefix(dyp, W, acc=None):
    """dy @ W from dy's natural-order pieces (prefix form), + ``acc`` if given; the weight
    operand is W^T's planes in ORDER_W_PREFIX (NT form)."""
    n = _State.passes
    wt = weight_planes_t(W, 0, ORDER_W_PREFIX[n])
    assert wt is not None, 'dgrad_prefix: W shape must be 64-aligned'
    return prefix_mm(dyp, wt.t(), W.shape[0], acc)
