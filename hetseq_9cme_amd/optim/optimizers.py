"""Optimizers over the flat parameter space.

API parity with the reference wrapper (hetseq/optim.py:6-131): ``get_lr``,
``set_lr``, ``state_dict``, ``load_state_dict(sd, overrides)``, ``backward``,
``multiply_grads``, ``clip_grad_norm``, ``step``, ``zero_grad``; class names
``_Adam`` / ``_Adadelta`` (checkpoints record ``optimizer_name``).

Update rules (exactly the reference's, optim.py:162-231 / 263-304):
  Adam (fairseq "AdamW" variant, decoupled weight decay on ALL params):
      m = b1 m + (1-b1) g ;  v = b2 v + (1-b2) g^2
      p -= wd*lr*p                                   (if wd != 0)
      p -= lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps)
  Adadelta: the standard algorithm with L2 weight decay added to the grad.

MI355X-native implementation: parameters, gradients and optimizer moments
are flat fp32 buffers (``FlatParamSpace``).  ``multiply_grads`` and the clip
coefficient do not touch memory -- they update a *device* scalar ``gscale``
that the single fused update kernel applies on the fly; the global grad norm
is one reduction kernel over the flat gradient buffer.  One step therefore
costs two small reduction launches + one streaming update launch instead of
~1,850 launches, and never blocks the host.
On CPU tensors the same math runs through torch ops (reference/oracle path).
"""
import math

import torch

from .. import ops


class _Optimizer(object):
    """Common machinery: flat space, lazy grad scale, LR, state_dict format."""

    def __init__(self, args, flat):
        self.args = args
        self.flat = flat
        self.device = flat.device
        self._lr = float(args.lr[0])
        # device-resident scalars: [gscale] ; grad norm result
        self._gscale = torch.ones(1, dtype=torch.float32, device=self.device)
        self._gscale_host = 1.0          # host multiplier folded on next use
        self._grad_norm = torch.zeros(1, dtype=torch.float32, device=self.device)
        self._clipped = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.used_mask = [True] * len(flat.params)
        self.param_groups = [dict(self.optimizer_config)]
        self.param_groups[0]['lr'] = self._lr
        self.use_kernels = self.device.type == 'cuda' and getattr(args, 'fused_kernels', True)

    # --- LR -----------------------------------------------------------
    def get_lr(self):
        return self._lr

    def set_lr(self, lr):
        self._lr = float(lr)
        for g in self.param_groups:
            g['lr'] = self._lr

    @property
    def params(self):
        return list(self.flat.params)

    # --- grads --------------------------------------------------------
    phase_hook = None   # set by the controller under --profile-phases
    bf16_shadow = None  # bf16 copy of the flat params kept in sync by step() (--precision bf16)
    # Graph-captured steps (utils/train_graph.py): a device fp32 buffer the update kernels read
    # their per-update hyper-parameters from (2 per run for Adam: step size, wd * lr; 1 for
    # Adadelta: lr), so a replayed graph applies the current schedule.  ``_hp_vals`` holds the
    # values of the latest step (also the ones a capture pass computed but could not write).
    device_hparams = None
    _hp_vals = None
    _runs_sig = None

    def _hp_slice(self, r, width):
        hp = self.device_hparams
        return None if hp is None else hp[width * r:width * (r + 1)]

    def _write_hparams(self):
        """Write ``_hp_vals`` into ``device_hparams`` (small fills; skipped while capturing,
        where they would be frozen into the graph)."""
        hp = self.device_hparams
        if hp is None or self._hp_vals is None or torch.cuda.is_current_stream_capturing():
            return
        for k, v in enumerate(self._hp_vals):
            hp[k].fill_(v)

    def backward(self, loss):
        if self.phase_hook is not None:
            self.phase_hook('backward')
        loss.backward()

    def zero_grad(self):
        self.flat.zero_grad()
        self._gscale.fill_(1.0)
        self._gscale_host = 1.0

    def multiply_grads(self, c):
        """Multiply grads by ``c`` (python number or 0-d/1-elem device tensor).
        Lazy: folded into the scale applied by the fused kernels."""
        if torch.is_tensor(c):
            self._gscale.mul_(c.to(self._gscale.dtype).reshape(1))
        else:
            self._gscale_host *= float(c)

    def _fold_host_scale(self):
        if self._gscale_host != 1.0:
            self._gscale.mul_(self._gscale_host)
            self._gscale_host = 1.0

    def scaled_grad_flat(self):
        """The flat gradient with every pending multiply/clip applied (a new
        tensor) -- what a custom (non-fused) optimizer's ``step`` consumes."""
        self._fold_host_scale()
        return self.flat.grad_flat * self._gscale

    def clip_grad_norm(self, max_norm):
        """Global L2 norm of the (scaled) grads; clip by folding the coefficient
        into ``gscale``.  Returns the pre-clip norm as a 1-element DEVICE tensor
        (read lazily by the meters)."""
        self._fold_host_scale()
        g = self.flat.grad_flat
        if self.use_kernels:
            ops.flat_grad_norm_clip(g, self._gscale, self._grad_norm, self._clipped, float(max_norm))
        else:
            norm = g.float().norm(2) * self._gscale.abs()
            self._grad_norm.copy_(norm.reshape(1))
            if max_norm > 0:
                coef = (max_norm / (norm + 1e-6)).clamp(max=1.0)
                self._clipped.copy_((norm > max_norm).float().reshape(1))
                self._gscale.mul_(coef.reshape(1))
            else:
                self._clipped.zero_()
        return self._grad_norm

    @property
    def clipped(self):
        return self._clipped

    # --- state dict (torch-optimizer format, reference-compatible) ------
    # Torch optimizers number their state by position in ``model.parameters()``
    # (requires_grad only, tied weights once) -- the reference builds its Adam over
    # exactly that list (hetseq/controller.py:92-96).  The flat layout orders
    # parameters differently (reverse blocks, fused groups), so state is emitted and
    # consumed through ``flat.model_order`` (position -> flat index).
    # ``param_order`` tags the layout: 'model' (this format; also what a torch optimizer over
    # model.parameters() -- the reference's -- writes, untagged).  Round-1 files of this framework
    # were numbered by FLAT index and carry no tag: the checkpoint loader recognises them by their
    # framework-specific args and passes ``legacy_flat_order=True`` (see Controller.load_checkpoint).
    STATE_ORDER = 'model'

    def state_dict(self):
        state = {}
        for pos, i in enumerate(self.flat.model_order):
            s = self._param_state(i)
            if s is not None:
                state[pos] = s
        groups = []
        for g in self.param_groups:
            gg = {k: v for k, v in g.items()}
            gg['params'] = list(range(len(self.flat.params)))
            groups.append(gg)
        return {'state': state, 'param_groups': groups, 'param_order': self.STATE_ORDER}

    def load_state_dict(self, state_dict, optimizer_overrides=None, legacy_flat_order=False):
        """``legacy_flat_order``: the state is numbered by flat index (an untagged file written
        by this framework before the state-order tag existed) and is remapped accordingly."""
        order = state_dict.get('param_order', 'flat' if legacy_flat_order else 'model')
        if order not in ('model', 'flat'):
            raise ValueError('unknown optimizer state order {!r}'.format(order))
        groups = state_dict['param_groups']
        saved = groups[0]
        for k, v in saved.items():
            if k != 'params':
                self.param_groups[0][k] = v
        if optimizer_overrides:
            self.param_groups[0].update(optimizer_overrides)
        self._apply_group_config()
        saved_ids = list(saved['params'])
        if len(saved_ids) != len(self.flat.params):
            raise ValueError('loaded state dict has a different number of parameters')
        for idx, s in state_dict['state'].items():
            pos = saved_ids.index(idx) if idx in saved_ids else int(idx)
            i = pos if order == 'flat' else self.flat.model_order[pos]
            shape = self.flat.params[i].shape
            for k, v in s.items():
                if torch.is_tensor(v) and v.dim() > 0 and v.numel() != shape.numel():
                    raise ValueError('optimizer state {!r} of parameter {} ({}) has shape {}, expected {}'.format(
                        k, pos, self.flat.names[i], tuple(v.shape), tuple(shape)))
            self._load_param_state(i, s)
        self._lr = self.param_groups[0]['lr']

    def _apply_group_config(self):
        pass

    def _param_state(self, i):
        raise NotImplementedError

    def _load_param_state(self, i, s):
        raise NotImplementedError


class _Adam(_Optimizer):
    """Fused AdamW-style Adam over flat fp32 buffers."""

    def __init__(self, args, flat):
        self.args = args
        super().__init__(args, flat)
        self.exp_avg = torch.zeros_like(flat.param_flat)
        self.exp_avg_sq = torch.zeros_like(flat.param_flat)
        self.steps = [0] * len(flat.params)
        self.amsgrad = False
        self.bf16_shadow = None   # optional bf16 copy of params written by the update

    @property
    def optimizer_config(self):
        return {
            'lr': float(self.args.lr[0]),
            'betas': eval(self.args.adam_betas) if isinstance(self.args.adam_betas, str)
            else tuple(self.args.adam_betas),
            'eps': float(self.args.adam_eps),
            'weight_decay': float(self.args.weight_decay),
            'amsgrad': False,
        }

    # --find-unused-parameters under data parallelism: the controller sets this, per update, to
    # the all-reduced used flags (f64 device slice of the stats vector, > 0 = some rank used the
    # parameter).  ``step`` then skips unused parameters and advances the per-parameter step
    # counters ON DEVICE (``_steps_dev``) -- no host read of the flags.
    device_used = None
    _steps_dev = None
    _mask_table = None
    _masked = False     # the latest update took the masked path
    _lr_dev = None      # f64 [1]: the masked update's lr (a replayed graph reads the current one)

    def _write_hparams(self):
        super()._write_hparams()
        if self._masked and self._lr_dev is not None and not torch.cuda.is_current_stream_capturing():
            self._lr_dev.fill_(self._lr)

    def _device_steps(self):
        if self._steps_dev is None:
            self._steps_dev = torch.tensor(self.steps, dtype=torch.int32, device=self.device)
            self._mask_hp = torch.zeros(2 * len(self.steps), dtype=torch.float32, device=self.device)
        return self._steps_dev

    def _pull_steps(self):
        """Device step counters -> host list (one sync; checkpointing / switching paths)."""
        if self._steps_dev is not None:
            self.steps = [int(t) for t in self._steps_dev.tolist()]
            self._steps_dev = None

    def _masked_table(self):
        """(param, start, end) rows, one per <= chunk-float slice of one parameter (ends rounded
        up to 4 floats; the flat layout's 64-float alignment keeps that inside the padding)."""
        if self._mask_table is None:
            chunk = ops.C().adam_mask_chunk()
            rows = []
            for i in range(len(self.flat.params)):
                s, e = self.flat.param_range(i)
                e = (e + 3) // 4 * 4
                for a in range(s, e, chunk):
                    rows.append((i, a, min(e, a + chunk)))
            self._mask_table = torch.tensor(rows, dtype=torch.int64, device=self.device).reshape(-1, 3)
        return self._mask_table

    def step(self, closure=None):
        g = self.param_groups[0]
        beta1, beta2 = g['betas']
        eps, wd, lr = g['eps'], g['weight_decay'], self._lr
        self._fold_host_scale()
        self._masked = False
        if self.device_used is not None:
            used, self.device_used = self.device_used, None
            if self.use_kernels:
                self._masked = True
                self._host_step()
                ops.C().adam_masked(self.flat.param_flat, self.flat.grad_flat, self.exp_avg, self.exp_avg_sq,
                                    self.bf16_shadow, self._gscale, self._masked_table(),
                                    used.reshape(-1).to(torch.float64).contiguous(), self._device_steps(),
                                    self._mask_hp, float(lr), float(beta1), float(beta2), float(eps), float(wd),
                                    lr_dev=self._lr_dev)
                return
            self.used_mask = [bool(u > 0) for u in used.reshape(-1).tolist()]   # CPU reference path
        runs = self._host_step()
        for r, (start, end, t) in enumerate(runs):
            bc1 = 1 - beta1 ** t
            bc2 = 1 - beta2 ** t
            step_size = lr * math.sqrt(bc2) / bc1
            if self.use_kernels:
                ops.fused_adam(self.flat.param_flat, self.flat.grad_flat, self.exp_avg,
                               self.exp_avg_sq, self._gscale, start, end,
                               float(beta1), float(beta2), float(eps), float(step_size),
                               float(wd * lr), self.bf16_shadow, self._hp_slice(r, 2))
            else:
                p = self.flat.param_flat[start:end]
                gr = self.flat.grad_flat[start:end].float() * self._gscale
                m = self.exp_avg[start:end]
                v = self.exp_avg_sq[start:end]
                m.mul_(beta1).add_(gr, alpha=1 - beta1)
                v.mul_(beta2).addcmul_(gr, gr, value=1 - beta2)
                denom = v.sqrt().add_(eps)
                if wd != 0:
                    p.add_(p, alpha=-wd * lr)
                p.addcdiv_(m, denom, value=-step_size)
                if self.bf16_shadow is not None:
                    self.bf16_shadow[start:end].copy_(p)

    def _host_step(self):
        """Host half of an update: advance the step counters, compute this update's
        hyper-parameters and (graph mode) write them to the device buffer.  A replayed
        graph calls only this; ``step`` calls it and then launches the kernels.  The masked
        (``device_used``) update advances its counters on the device: its host half is only
        the learning rate, which a graph-captured update reads from ``_lr_dev``."""
        if self._masked:
            if self._lr_dev is None:   # allocated by the first (eager) masked update, never in a capture
                self._lr_dev = torch.zeros(1, dtype=torch.float64, device=self.device)
            self._hp_vals = []
            self._runs_sig = ('masked',)
            self._write_hparams()
            return []
        self._pull_steps()
        g = self.param_groups[0]
        beta1, beta2 = g['betas']
        lr, wd = self._lr, g['weight_decay']
        runs = self._runs_by_step()
        vals = []
        for (_, _, t) in runs:
            vals += [lr * math.sqrt(1 - beta2 ** t) / (1 - beta1 ** t), wd * lr]
        self._hp_vals = vals
        self._runs_sig = tuple((a, b) for a, b, _ in runs)
        self._write_hparams()
        return runs

    def _runs_by_step(self):
        """Advance per-param step counters for used params and return
        contiguous (start, end, step) runs sharing one step count."""
        runs = []
        cur = None
        for i, used in enumerate(self.used_mask):
            s, e = self.flat.param_range(i)
            if used:
                self.steps[i] += 1
                t = self.steps[i]
                if cur is not None and cur[2] == t:
                    cur[1] = e
                else:
                    if cur is not None:
                        runs.append(tuple(cur))
                    cur = [s, e, t]
            else:
                if cur is not None:
                    runs.append(tuple(cur))
                    cur = None
        if cur is not None:
            runs.append(tuple(cur))
        return runs

    def _param_state(self, i):
        self._pull_steps()
        if self.steps[i] == 0:
            return None
        s, e = self.flat.param_range(i)
        shape = self.flat.params[i].shape
        return {
            'step': self.steps[i],
            'exp_avg': self.exp_avg[s:e].view(shape),
            'exp_avg_sq': self.exp_avg_sq[s:e].view(shape),
        }

    def _load_param_state(self, i, st):
        self._pull_steps()
        s, e = self.flat.param_range(i)
        self.steps[i] = int(st['step'])
        self.exp_avg[s:e].copy_(st['exp_avg'].reshape(-1).to(self.exp_avg))
        self.exp_avg_sq[s:e].copy_(st['exp_avg_sq'].reshape(-1).to(self.exp_avg_sq))


class _Adadelta(_Optimizer):
    """Fused Adadelta (MNIST task) over flat fp32 buffers."""

    def __init__(self, args, flat):
        self.args = args
        super().__init__(args, flat)
        self.square_avg = torch.zeros_like(flat.param_flat)
        self.acc_delta = torch.zeros_like(flat.param_flat)
        self.steps = [0] * len(flat.params)

    @property
    def optimizer_config(self):
        return {
            'lr': float(self.args.lr[0]),
            'rho': float(self.args.adadelta_rho),
            'eps': float(self.args.adadelta_eps),
            'weight_decay': float(self.args.dadelta_weight_decay),
        }

    def step(self, closure=None):
        g = self.param_groups[0]
        rho, eps, wd, lr = g['rho'], g['eps'], g['weight_decay'], self._lr
        self._fold_host_scale()
        runs = self._host_step()
        for (start, end) in runs:
            if self.use_kernels:
                ops.fused_adadelta(self.flat.param_flat, self.flat.grad_flat, self.square_avg,
                                   self.acc_delta, self._gscale, start, end,
                                   float(lr), float(rho), float(eps), float(wd), self._hp_slice(0, 1))
            else:
                p = self.flat.param_flat[start:end]
                gr = self.flat.grad_flat[start:end] * self._gscale
                sq = self.square_avg[start:end]
                acc = self.acc_delta[start:end]
                if wd != 0:
                    gr = gr.add(p, alpha=wd)
                sq.mul_(rho).addcmul_(gr, gr, value=1 - rho)
                std = sq.add(eps).sqrt_()
                delta = acc.add(eps).sqrt_().div_(std).mul_(gr)
                p.add_(delta, alpha=-lr)
                acc.mul_(rho).addcmul_(delta, delta, value=1 - rho)

        if self.bf16_shadow is not None:
            self.flat.refresh_bf16()

    def _host_step(self):
        for i, used in enumerate(self.used_mask):
            if used:
                self.steps[i] += 1
        runs = self.flat.runs_for(self.used_mask)
        self._hp_vals = [self._lr]
        self._runs_sig = tuple(runs)
        self._write_hparams()
        return runs

    def _param_state(self, i):
        if self.steps[i] == 0:
            return None
        s, e = self.flat.param_range(i)
        shape = self.flat.params[i].shape
        return {'step': self.steps[i], 'square_avg': self.square_avg[s:e].view(shape),
                'acc_delta': self.acc_delta[s:e].view(shape)}

    def _load_param_state(self, i, st):
        s, e = self.flat.param_range(i)
        self.steps[i] = int(st['step'])
        self.square_avg[s:e].copy_(st['square_avg'].reshape(-1).to(self.square_avg))
        self.acc_delta[s:e].copy_(st['acc_delta'].reshape(-1).to(self.acc_delta))


OPTIMIZER_REGISTRY = {'adam': _Adam, 'adadelta': _Adadelta}


def register_optimizer(name):
    """Class decorator adding an ``_Optimizer`` subclass to ``--optimizer`` choices.
    Optional ``add_args(group)`` static method declares its flags."""
    def deco(cls):
        if name in OPTIMIZER_REGISTRY and OPTIMIZER_REGISTRY[name] is not cls:
            raise ValueError('optimizer {} already registered'.format(name))
        OPTIMIZER_REGISTRY[name] = cls
        return cls
    return deco


def build_optimizer(args, flat):
    if args.optimizer not in OPTIMIZER_REGISTRY:
        raise ValueError('unsupported optimizer - {}'.format(args.optimizer))
    return OPTIMIZER_REGISTRY[args.optimizer](args, flat)
