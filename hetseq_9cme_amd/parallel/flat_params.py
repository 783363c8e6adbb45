"""Flat, bucket-ordered parameter / gradient storage.

The reference keeps 206 separate parameter and gradient tensors, lets DDP copy
gradients into 25 MB flat buckets and back, and runs Python
per-parameter loops for grad scaling, clipping and Adam (~1,850 launches per
step).

Here every trainable parameter is re-homed as a *view* into ONE contiguous
fp32 buffer and every ``.grad`` is a view into ONE contiguous gradient buffer
laid out identically.  Consequences:

* the gradient all-reduce buckets are plain contiguous slices of the flat
  gradient buffer -> RCCL reduces them in place, no pack/unpack copies;
* global L2 norm, clip, grad scaling and the optimizer update are single
  kernels over flat memory (one launch each, HBM-streaming);
* parameters whose storage must be adjacent for fused kernels (e.g. the
  Q/K/V projections -> one N=2304 GEMM) are placed back to back.

Layout order: parameter *groups* (module blocks) are laid out in REVERSE
forward order so that the first bucket to fill during backward is bucket 0;
inside a block forward order is kept.  Every tensor starts on a 64-element
(256 B) boundary so vector kernels can use 16-byte accesses.
"""
from collections import OrderedDict

import torch

ALIGN = 64


def _block_key(name):
    parts = name.split('.')
    # group encoder layers as one block; other params by their owning module
    for i, p in enumerate(parts):
        if p == 'layer' and i + 1 < len(parts) and parts[i + 1].isdigit():
            return '.'.join(parts[:i + 2])
    return '.'.join(parts[:-1])


class FlatParamSpace(object):
    """Owns the flat parameter and gradient buffers of a model."""

    def __init__(self, model, device=None, dtype=torch.float32, contiguous_groups=None,
                 reverse_blocks=True):
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        # de-duplicate tied params (named_parameters already does, keep first name)
        seen = set()
        uniq = []
        for n, p in named:
            if id(p) in seen:
                continue
            seen.add(id(p))
            uniq.append((n, p))
        name_to_param = OrderedDict(uniq)

        # build block order
        blocks = OrderedDict()
        for n, p in uniq:
            blocks.setdefault(_block_key(n), []).append(n)
        block_names = list(blocks.keys())
        if reverse_blocks:
            block_names = block_names[::-1]

        # contiguity constraints: reorder inside a block so each group is adjacent
        groups = contiguous_groups or []
        group_of = {}
        for g in groups:
            for n in g:
                group_of[n] = g
        order = []
        for b in block_names:
            placed = set()
            for n in blocks[b]:
                if n in placed:
                    continue
                g = group_of.get(n)
                if g is not None and all(x in name_to_param for x in g):
                    for x in g:
                        if x not in placed:
                            order.append(x)
                            placed.add(x)
                else:
                    order.append(n)
                    placed.add(n)
        self.names = order
        self.params = [name_to_param[n] for n in order]
        # flat index of each trainable parameter in ``model.parameters()`` order: the
        # order torch optimizers (and so reference checkpoints) index their state by
        self.model_order = [order.index(n) for n, _ in uniq]
        if device is None:
            device = self.params[0].device
        self.device = torch.device(device)
        self.dtype = dtype

        offsets, off = [], 0
        for p in self.params:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            offsets.append(off)
            off += p.numel()
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        self.offsets = offsets
        self.sizes = [p.numel() for p in self.params]

        self.param_flat = torch.zeros(self.numel, dtype=dtype, device=self.device)
        self.grad_flat = torch.zeros(self.numel, dtype=dtype, device=self.device)
        with torch.no_grad():
            for p, o in zip(self.params, offsets):
                view = self.param_flat[o:o + p.numel()].view_as(p)
                view.copy_(p.data.to(self.device, dtype))
                p.data = view
                p.grad = self.grad_flat[o:o + p.numel()].view_as(p)
        self.index_of = {id(p): i for i, p in enumerate(self.params)}
        # direct-write gradient slots (see ``claim``)
        self.slots = [self.grad_flat[o:o + p.numel()].view_as(p) for p, o in zip(self.params, offsets)]
        self.claimed = set()
        for i, p in enumerate(self.params):
            p._hx_flat = self
            p._hx_index = i

        # verify contiguity groups are adjacent (required for fused views)
        for g in groups:
            if not all(n in name_to_param for n in g):
                continue
            idx = [self.names.index(n) for n in g]
            for a, b in zip(idx[:-1], idx[1:]):
                assert b == a + 1 and self.offsets[b] == self.offsets[a] + self.sizes[a], \
                    'contiguous group {} could not be laid out adjacently'.format(g)

        self.param_bf16 = None

    # ------------------------------------------------------------------ bf16 compute copy
    def enable_bf16_shadow(self):
        """``--precision bf16``: a bf16 copy of the flat parameters, laid out
        identically, that the GEMMs read instead of casting the fp32 master
        weights on every use.  The fused Adam writes it as part of the update
        (``_Adam.bf16_shadow``); ``refresh_bf16`` re-syncs it after a load."""
        if self.param_bf16 is None:
            self.param_bf16 = torch.empty(self.numel, dtype=torch.bfloat16, device=self.device)
            for p, o in zip(self.params, self.offsets):
                p._hx_bf16 = self.param_bf16[o:o + p.numel()].view(p.shape)
        self.refresh_bf16()
        return self.param_bf16

    def refresh_bf16(self):
        if self.param_bf16 is not None:
            with torch.no_grad():
                self.param_bf16.copy_(self.param_flat)

    # ------------------------------------------------------------------
    def rebind_grads(self):
        """Re-attach ``.grad`` views (used after something set grads to None)."""
        for p, o in zip(self.params, self.offsets):
            g = p.grad
            if g is None or g.data_ptr() != self.grad_flat[o:o + 1].data_ptr():
                view = self.grad_flat[o:o + p.numel()].view_as(p)
                if g is not None:
                    view.copy_(g)
                p.grad = view

    def zero_grad(self):
        """Start a new step: grads become None (autograd will steal the slot views the
        fused backward kernels write into -- no memset, no AccumulateGrad add)."""
        for p in self.params:
            p.grad = None
        self.claimed.clear()

    def claim(self, p):
        """Return p's flat gradient slot if the caller may WRITE (overwrite) it as
        the first gradient contribution of this step, else None.  The backward that
        claims a slot must fully overwrite it and return it as the gradient; autograd
        then adopts the tensor as ``p.grad`` without copying."""
        i = p._hx_index
        if p.grad is not None or i in self.claimed:
            return None
        self.claimed.add(i)
        # a FRESH view object: autograd adopts a returned grad without copying only
        # if no other Python reference holds its TensorImpl
        o = self.offsets[i]
        return self.grad_flat[o:o + self.sizes[i]].view(p.shape)

    def is_claimed(self, p):
        return p._hx_index in self.claimed

    def adopt(self, i):
        """Make param i's .grad the flat slot (copy in a grad produced elsewhere;
        zero-fill if the param got no gradient this step)."""
        p = self.params[i]
        slot = self.slots[i]
        g = p.grad
        if g is None:
            slot.zero_()
            p.grad = slot
        elif g.data_ptr() != slot.data_ptr():
            slot.copy_(g)
            p.grad = slot

    def adopt_all(self):
        for i in range(len(self.params)):
            self.adopt(i)

    def param_range(self, i):
        return self.offsets[i], self.offsets[i] + self.sizes[i]

    def runs_for(self, used_mask):
        """Contiguous [start, end) element ranges covering the params whose
        ``used_mask`` entry is True (used by the optimizer to skip params that
        received no gradient, matching the reference's ``grad is None`` skip)."""
        runs = []
        start = None
        end = None
        for i, u in enumerate(used_mask):
            s, e = self.param_range(i)
            if u:
                if start is None:
                    start = s
                end = e
            else:
                if start is not None:
                    runs.append((start, end))
                    start = None
        if start is not None:
            runs.append((start, end))
        return runs

    def state_views(self, flat):
        """Per-parameter views of another flat buffer with this layout."""
        return [flat[o:o + n].view_as(p) for p, o, n in zip(self.params, self.offsets, self.sizes)]
