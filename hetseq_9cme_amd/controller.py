"""Controller: the synchronous data-parallel training engine.

API parity with the reference Controller (hetseq/controller.py:31-440):
``train_step(samples)``, ``get_train_iterator``, ``save_checkpoint``,
``load_checkpoint``, ``lr_step``, ``lr_step_update``, ``get_lr``, ``get_model``,
``get_meter``, ``get_num_updates``, ``set_num_updates``; the same meters
(train_loss, train_nll_loss, valid_*, wps, ups, wpb, bsz, gnorm, clip, wall,
train_wall) and the same update arithmetic:

  per micro-batch: forward/backward (``no_sync`` except on the last one),
  dummy batch with zeroed loss when this rank's shard ran out;
  stats: fast path = SUM all-reduce of [sample_size, nsentences, loss, nll_loss,
  ntokens, ooms] then loss /= sample_size*ln2; slow path = all_gather_list of the
  logging outputs + cross-rank grad-norm consistency assertion;
  grads *= W / sample_size; clip to --clip-norm; optimizer step; num_updates += 1.

MI355X-native engine underneath:
  * parameters/grads live in one flat fp32 buffer (``FlatParamSpace``);
  * DDP is replaced by ``GradReducer`` (in-place RCCL all-reduce of contiguous
    grad-buffer buckets, launched in backward as buckets fill);
  * grad scaling and clipping are folded into device scalars; norm, clip and
    Adam are one reduction + one fused update kernel (no host sync);
  * the stats vector is built and all-reduced on device; meters read it lazily
    (only when a log line is printed);
  * batches arrive already staged on the HIP copy stream (``DeviceBatch``).
"""
import contextlib
import math
import os
import threading
from collections import OrderedDict

import torch

from . import checkpoint_utils, ops
from .ops import gemm_tuning
from .options import comm_cus, graph_train_step_enabled
from .data.prefetch import unwrap
from .optim import build_lr_scheduler, build_optimizer
from .parallel import distributed as dist_utils
from .parallel.flat_params import FlatParamSpace
from .parallel.reducer import GradReducer, TransportErrorMonitor
from .utils.meters import AverageMeter, StopwatchMeter, TimeMeter
from .utils.phase_timer import PhaseTimer
from .utils.misc import ensure_train, move_to_device

LN2 = math.log(2)

# flags this framework's parser has always added and the reference's never did (options.py)
_OWN_FLAGS = ('fused_kernels', 'allreduce_impl', 'precision', 'overlap_wgrad', 'gemm_tuning')


def state_order_ambiguous(optim_state, ck_args):
    """Is an optimizer state's parameter order unknowable?  States are numbered in
    model.parameters() order; files since the state-order tag say so ('param_order'), and so do
    untagged ones from the reference / torch optimizers (no flags of this framework in their
    args) and from this framework after --fp32-gemm appeared (which came after the switch to
    model order).  Only untagged files of this framework's earliest builds (own flags, no
    ``fp32_gemm``) may be numbered by flat index, and nothing in them tells which: refuse those."""
    if 'param_order' in optim_state or ck_args is None:
        return False
    own = any(hasattr(ck_args, f) for f in _OWN_FLAGS)
    return own and not hasattr(ck_args, 'fp32_gemm')


class Controller(object):
    def __init__(self, args, task, model, criterion=None, dummy_batch=None, oom_batch=None):
        self.args = args
        self.task = task
        self.cuda = torch.cuda.is_available() and not getattr(args, 'cpu', False)
        self.device = torch.device('cuda', torch.cuda.current_device()) if self.cuda else torch.device('cpu')
        if not getattr(args, 'fused_kernels', True):
            ops.set_fused(False)      # A/B mode: plain torch ops on the GPU
        ops.set_fp32_gemm(getattr(args, 'fp32_gemm', 'native'))
        ow = getattr(args, 'overlap_wgrad', 'auto')
        # 'auto' threshold: products of >= 8192 token rows; >= 4096 for hidden sizes >= 1024, whose
        # wider products pay for the overlap already there (BERT-large seq 128 b32 44.34-44.40 vs
        # 45.38-45.55 ms/step, seq 512 b8 48.80-49.03 vs 49.35-49.36; BERT-base at 4096 rows is
        # bimodal, 12.6 or 13.9 vs 13.1: profiles/r6ae_side_stream_low_priority_ab.txt)
        hidden = getattr(getattr(model, 'config', None), 'hidden_size', 0) or 0
        ops.set_side_stream({True: 'on', False: 'off', None: 'auto'}.get(ow, ow),
                            auto_rows=4096 if hidden >= 1024 else None)
        if getattr(args, 'debug_kernels', False) and self.cuda:
            ops.C().set_debug(True)   # validation inside the bindings (see csrc/bindings.cpp)
        if self.cuda:
            gemm_tuning.configure(getattr(args, 'gemm_tuning', 'table'), getattr(args, 'gemm_tuning_file', None))
        model = model.to(self.device)
        if getattr(args, 'precision', 'fp32') == 'bf16' and hasattr(model, 'set_compute_dtype'):
            model.set_compute_dtype(torch.bfloat16)
        self._model = model
        self.world_size = args.distributed_world_size
        groups = model.flat_contiguous_groups() if hasattr(model, 'flat_contiguous_groups') else None
        self.flat = FlatParamSpace(model, self.device, contiguous_groups=groups)
        if getattr(args, 'precision', 'fp32') == 'bf16' and self.cuda:
            self.flat.enable_bf16_shadow()
        force = bool(getattr(args, 'force_reducer', False))
        use_reducer = (self.world_size > 1 or force) and not getattr(args, 'use_bmuf', False)
        self.reducer = GradReducer(self.flat, bucket_cap_mb=args.bucket_cap_mb,
                                   find_unused_parameters=getattr(args, 'find_unused_parameters', False),
                                   broadcast_params=use_reducer,
                                   bucket_peer_mb=getattr(args, 'bucket_peer_mb', 0.0), force=force)
        ncus = comm_cus(args) if self.cuda else 0
        self.comm_cus = ncus if use_reducer else 0
        if use_reducer and ncus > 0:
            # while its buckets are in flight the plans leave these CUs to the all-reduce
            self.reducer.set_comm_cus(ncus)
        if not use_reducer:
            self.reducer.enabled = False
        elif getattr(args, 'allreduce_impl', 'rccl') == 'xgmi':
            self.reducer.use_xgmi(blocks=getattr(args, 'xgmi_blocks', 64),
                                  timeout_s=float(getattr(args, 'distributed_timeout', 1800)),
                                  comm_cus=ncus)
        self._dummy_batch = dummy_batch
        self._oom_batch = oom_batch or dummy_batch
        self._lr_scheduler = None
        self._num_updates = 0
        self._optim_history = None
        self._optimizer = None
        self._prev_grad_norm = None
        self.fast_stat_sync = args.fast_stat_sync
        self._save_thread = None
        self._transport_monitor = TransportErrorMonitor(lag=2)
        self._graph_step = None
        if graph_train_step_enabled(args) and self.cuda:
            from .utils.train_graph import GraphedTrainStep
            self._graph_step = GraphedTrainStep(self)
        self._profile_phases = bool(getattr(args, 'profile_phases', False))
        self.phases = PhaseTimer(self._profile_phases, cuda=self.cuda)
        self.init_meters(args)

    # ------------------------------------------------------------------ meters
    def init_meters(self, args):
        self.meters = OrderedDict()
        self.meters['train_loss'] = AverageMeter()
        self.meters['train_nll_loss'] = AverageMeter()
        self.meters['valid_loss'] = AverageMeter()
        self.meters['valid_nll_loss'] = AverageMeter()
        self.meters['wps'] = TimeMeter()
        self.meters['ups'] = TimeMeter()
        self.meters['wpb'] = AverageMeter()
        self.meters['bsz'] = AverageMeter()
        self.meters['gnorm'] = AverageMeter()
        self.meters['clip'] = AverageMeter()
        self.meters['wall'] = TimeMeter()
        self.meters['train_wall'] = StopwatchMeter()

    # ------------------------------------------------------------------ lazily built parts
    @property
    def model(self):
        return self._model

    @property
    def optimizer(self):
        if self._optimizer is None:
            self._build_optimizer()
        return self._optimizer

    @property
    def lr_scheduler(self):
        if self._lr_scheduler is None:
            self._build_optimizer()
        return self._lr_scheduler

    def _build_optimizer(self):
        self._optimizer = build_optimizer(self.args, self.flat)
        self._optimizer.phase_hook = self.phases.begin if self._profile_phases else None
        if self.flat.param_bf16 is not None:
            self._optimizer.bf16_shadow = self.flat.param_bf16   # the fused update rewrites it
        self._lr_scheduler = build_lr_scheduler(self.args, self._optimizer)
        self._lr_scheduler.step_update(0)

    # ------------------------------------------------------------------ checkpoints
    def check_transport_all(self):
        """Collective-consistent check of every recorded update's xGMI error word: the
        words were summed by the stats all-reduce, so every rank reads the same values and all
        raise together -- before persisting weights and at the end of training, where the lagged
        per-step check has not yet looked at the last updates."""
        self._transport_monitor.check(force=True)

    def save_checkpoint(self, filename, extra_state, copies=()):
        self.check_transport_all()   # never persist weights updated from timed-out reductions
        if dist_utils.is_master(self.args):
            extra_state['train_meters'] = checkpoint_utils.meters_state(self.meters)
            state = checkpoint_utils.build_state(
                self.args, self.get_model().state_dict(), self.optimizer, self.lr_scheduler,
                self.get_num_updates(), self._optim_history, extra_state)
            if getattr(self.args, 'async_save', False):
                self.wait_for_save()
                self._save_thread = threading.Thread(target=checkpoint_utils.torch_persistent_save,
                                                     args=(state, filename, list(copies)), daemon=True)
                self._save_thread.start()
            else:
                checkpoint_utils.torch_persistent_save(state, filename, copies)

    def wait_for_save(self):
        if self._save_thread is not None:
            self._save_thread.join()
            self._save_thread = None

    def load_checkpoint(self, filename, reset_optimizer=False, reset_lr_scheduler=False, optimizer_overrides=None,
                        reset_meters=False):
        extra_state, self._optim_history, last_optim_state = None, [], None
        if os.path.exists(filename):
            state = checkpoint_utils.load_checkpoint_to_cpu(filename)
            try:
                self.get_model().load_state_dict(state['model'], strict=True)
            except Exception as e:
                raise Exception('Cannot load model parameters from checkpoint {}; '
                                'please ensure that the architectures match.'.format(filename)) from e
            extra_state = state['extra_state']
            self._optim_history = state['optimizer_history']
            last_optim_state = state.get('last_optimizer_state', None)
        if last_optim_state is not None and not reset_optimizer:
            self._build_optimizer()
            last_optim = self._optim_history[-1]
            assert last_optim['optimizer_name'] == self.optimizer.__class__.__name__, \
                'Optimizer does not match; please reset the optimizer (--reset-optimizer).'
            if not reset_lr_scheduler:
                self.lr_scheduler.load_state_dict(last_optim['lr_scheduler_state'])
            ck_args = state.get('args') if os.path.exists(filename) else None
            if state_order_ambiguous(last_optim_state, ck_args):
                raise RuntimeError(
                    'optimizer state of {} carries no state-order tag and was written by an early build of this '
                    'framework whose state may be numbered by flat index; resume it with --reset-optimizer'.format(
                        filename))
            self.optimizer.load_state_dict(last_optim_state, optimizer_overrides)
            self.set_num_updates(last_optim['num_updates'])
        if extra_state is not None and 'train_iterator' in extra_state:
            epoch = extra_state['train_iterator']['epoch']
            print('| loaded checkpoint {} (epoch {} @ {} updates)'.format(filename, epoch, self.get_num_updates()))
            self.lr_step(epoch)
            if 'train_meters' in extra_state and not reset_meters:
                checkpoint_utils.load_meters_state(self.meters, extra_state['train_meters'])
                del extra_state['train_meters']
                for meter in self.meters.values():
                    if isinstance(meter, TimeMeter):
                        meter.reset()
        elif extra_state is not None:
            print('| loaded checkpoint {} without iterator state (reference-format file)'.format(filename))
        else:
            print('| no existing checkpoint found {}'.format(filename))
        self.flat.refresh_bf16()
        return extra_state

    def get_train_iterator(self, epoch, combine=True, load_dataset=True):
        if load_dataset:
            print('| loading train data for epoch {}'.format(epoch))
            self.task.load_dataset(self.args.train_subset)
        self.task.configure_model(self.get_model())
        return self.task.get_batch_iterator(
            dataset=self.task.dataset(self.args.train_subset),
            max_tokens=self.args.max_tokens,
            max_sentences=self.args.max_sentences,
            max_positions=None,
            ignore_invalid_inputs=True,
            required_batch_size_multiple=self.args.required_batch_size_multiple,
            seed=self.args.seed,
            num_shards=self.args.distributed_world_size,
            shard_id=self.args.distributed_rank,
            num_workers=self.args.num_workers,
            epoch=epoch,
            device=self.device if self.cuda else None,
        )

    # ------------------------------------------------------------------ the step
    def _maybe_no_sync(self, i, n):
        if self.reducer.enabled and i < n - 1:
            return self.reducer.no_sync()
        return contextlib.nullcontext()

    def train_step(self, samples, dummy_batch=False, raise_oom=False):
        """Forward, backward and parameter update for one group of micro-batches."""
        if self._graph_step is not None and not dummy_batch:
            out = self._graph_step(samples)      # HIP-graph replay of a captured update
            if out is not NotImplemented:
                return out
        return self._train_step(samples, dummy_batch)

    def _train_step(self, samples, dummy_batch=False):
        capturing = self.cuda and torch.cuda.is_current_stream_capturing()
        ph = self.phases.begin
        ph('prep')
        self._transport_monitor.check()   # xGMI timeouts of update n-2, on every rank alike
        self._set_seed()
        model = self.model
        ensure_train(model)
        self.zero_grad()
        if not dummy_batch:
            self.meters['train_wall'].start()

        logging_outputs, sample_sizes, ooms = [], [], 0
        n_params = len(self.flat.params)
        step_used = [False] * n_params
        acc_ss, acc_ns, acc_nt = 0.0, 0.0, 0.0
        acc_loss, acc_nll = None, None
        sample_size, logging_output = 0, {}
        for i, sample in enumerate(samples):
            ph('sample')
            sample = self._prepare_sample(sample)
            if sample is None:
                if self._dummy_batch is None:
                    raise RuntimeError('first batch of the run is empty: no dummy batch available')
                sample = self._prepare_sample(self._dummy_batch)
                ignore_grad = True
            else:
                ignore_grad = False
                if self._dummy_batch is None:
                    self._dummy_batch = sample
            try:
                with self._maybe_no_sync(i, len(samples)):
                    self.reducer.prepare_for_backward()
                    ph('forward')     # optimizer.backward() opens 'backward'
                    loss, sample_size, logging_output = self.task.train_step(sample, model, self.optimizer,
                                                                             ignore_grad)
                    self.reducer.after_backward()
                    for k, u in enumerate(self.reducer.used):
                        if u:
                            step_used[k] = True
                ph('stats')
                if not ignore_grad:
                    logging_outputs.append(logging_output)
                    sample_sizes.append(sample_size)
                    if self.fast_stat_sync:
                        acc_ss += sample_size
                        acc_ns += logging_output.get('nsentences', 0.0)
                        acc_nt += logging_output.get('ntokens', 0.0)
                        l = logging_output.get('loss', 0.0)
                        nl = logging_output.get('nll_loss', 0.0)
                        acc_loss = l.double() if acc_loss is None else acc_loss + l.double()
                        acc_nll = nl.double() if acc_nll is None else acc_nll + nl.double()
            except RuntimeError as e:
                if 'out of memory' in str(e):
                    raise RuntimeError('ran out of memory with exception: {}'.format(e))
                raise e

        if dummy_batch:
            return None

        W = self.args.distributed_world_size
        size_for_norm = sample_size
        if self.fast_stat_sync:
            # [sample_size, nsentences, loss, nll_loss, ntokens, ooms] (+ xGMI error word)
            err = self.reducer.transport_error_async() if self.reducer.enabled else None
            fields = [acc_ss, acc_ns, 0.0, 0.0, acc_nt, float(ooms)] + ([0.0] if err is not None else [])
            # --find-unused-parameters: the local used flags (host-known) ride in the same
            # all-reduce; the optimizer consumes the summed flags on device (no host read)
            used_at = None
            if hasattr(self.optimizer, 'device_used'):
                self.optimizer.device_used = None   # never a previous update's flags
            if self.reducer.enabled and self.reducer.find_unused and hasattr(self.optimizer, 'device_used'):
                used_at = len(fields)
                fields += [1.0 if u else 0.0 for u in step_used]
            if capturing:
                # no host->device copy inside a graph (it would keep reading a freed pinned
                # buffer): the per-shape constants become fill nodes, one per run of equal values
                # (the used flags of a captured shape are the same on every replay)
                vec = torch.empty(len(fields), dtype=torch.float64, device=self.device)
                k = 0
                while k < len(fields):
                    e = k + 1
                    while e < len(fields) and fields[e] == fields[k]:
                        e += 1
                    vec[k:e].fill_(fields[k])
                    k = e
            else:
                host = torch.tensor(fields, dtype=torch.float64)
                vec = host.pin_memory().to(self.device, non_blocking=True) if self.cuda else host
            if acc_loss is not None:
                vec[2:4] = torch.stack([acc_loss.reshape(()), acc_nll.reshape(())]).to(vec.device)
            if err is not None:
                vec[6:7] = err
            if self._sync_stats():
                dist_utils.all_reduce(vec)
            if err is not None:
                self._transport_monitor.record(self._num_updates + 1, vec[6:7])
            if used_at is not None:
                self.optimizer.device_used = vec[used_at:used_at + len(step_used)]
            vec[2:4].div_(vec[0:1] * LN2)
            logging_output = {'sample_size': vec[0], 'nsentences': vec[1], 'loss': vec[2], 'nll_loss': vec[3],
                              'ntokens': vec[4], 'ooms': vec[5]}
            size_for_norm = vec[0] if self._sync_stats() else acc_ss
        elif self._sync_stats():
            err = self.reducer.transport_error_async() if self.reducer.enabled else None
            gathered = dist_utils.all_gather_list(
                [[{k: (v.item() if torch.is_tensor(v) else v) for k, v in lo.items()} for lo in logging_outputs],
                 sample_sizes, ooms,
                 (self._prev_grad_norm.item() if torch.is_tensor(self._prev_grad_norm) else self._prev_grad_norm),
                 int(err.item()) if err is not None else 0])
            prev_norms = [g[3] for g in gathered]
            ooms = sum(g[2] for g in gathered)
            if any(g[4] for g in gathered):   # every rank sees every rank's word: all raise together
                raise RuntimeError('xGMI all-reduce: a peer did not arrive within the timeout during update {} '
                                   '(error words per rank: {})'.format(self._num_updates + 1,
                                                                      [g[4] for g in gathered]))
            if not getattr(self.args, 'use_bmuf', False):
                assert (all(n == prev_norms[0] for n in prev_norms)
                        or all(n is None or math.isnan(n) or math.isinf(n) for n in prev_norms)), \
                    'Fatal error: gradients are inconsistent between workers'

        if not all(k in logging_output for k in ['ntokens', 'nsentences']):
            raise Exception('Please update the {}.aggregate_logging_outputs() method to return ntokens and '
                            'nsentences'.format(self.task.__class__.__name__))

        ph('optimizer')
        opt = self.optimizer
        # DDP averages gradients over ranks; the reducer SUMs, so its 1/W is folded here
        pre = self.reducer.grad_prescale if self.reducer.enabled else 1.0
        try:
            if torch.is_tensor(size_for_norm):
                scale = torch.where(size_for_norm > 0, (W * pre) / size_for_norm.clamp(min=1e-30),
                                    torch.full_like(size_for_norm, pre)).float()
                opt.multiply_grads(scale)
            elif size_for_norm > 0:
                opt.multiply_grads(W * pre / float(size_for_norm))
            elif pre != 1.0:
                opt.multiply_grads(pre)
            grad_norm = opt.clip_grad_norm(self.args.clip_norm)
            self._prev_grad_norm = grad_norm
            # skip only params no rank used (locally unused ones got the reduced gradient); on the
            # fast-stat-sync path the flags were all-reduced with the stats (opt.device_used)
            if getattr(opt, 'device_used', None) is None:
                opt.used_mask = self.reducer.global_used(step_used)
            opt.step()
            ph('meters')
            self.set_num_updates(self.get_num_updates() + 1)
            self.task.update_step(self._num_updates)
            if capturing:   # host meters: updated after every replay (utils/train_graph.py)
                self._captured_meter_args = (logging_output, size_for_norm if self.fast_stat_sync else sample_size,
                                             grad_norm, opt.clipped if self.args.clip_norm > 0 else 0.)
                return logging_output
            self._update_meters(logging_output, size_for_norm if self.fast_stat_sync else sample_size, grad_norm,
                                opt.clipped if self.args.clip_norm > 0 else 0.)
        except OverflowError as e:
            print('| WARNING: overflow detected, ' + str(e))
            if hasattr(opt, 'device_used'):
                opt.device_used = None
            self.zero_grad()
            logging_output = None

        self.meters['train_wall'].stop()
        self.phases.end_step()
        if logging_output is not None and 'sample_size' not in logging_output:
            logging_output['sample_size'] = sample_size
        return logging_output

    def _update_meters(self, logging_output, weight, grad_norm, clipped):
        """Per-update meters (reference controller.py:354-367); device values stay lazy.
        ``weight``: the all-reduced sample size on the fast path (reference: sample_size =
        vec[0] after the stats all-reduce, controller.py:300-306), the local one otherwise."""
        ntokens = logging_output.get('ntokens', 0)
        nsentences = logging_output.get('nsentences', 0)
        self.meters['wps'].update(ntokens)
        self.meters['ups'].update(1.)
        self.meters['wpb'].update(ntokens)
        self.meters['bsz'].update(nsentences)
        self.meters['gnorm'].update(grad_norm)
        self.meters['clip'].update(clipped)
        self.meters['train_loss'].update(logging_output.get('loss', 0), weight)
        if 'train_acc' in self.meters:
            self.meters['train_acc'].update(logging_output.get('acc', 0), weight)

    # ------------------------------------------------------------------ phase timing
    @property
    def phase_times(self):
        """Host seconds per phase accumulated so far (``--profile-phases``)."""
        return self.phases.host

    def phase_report(self, reset=True):
        """{'host': {...}, 'device': {...}, 'steps': n} -- see utils/phase_timer.py."""
        return self.phases.report(reset)

    # ------------------------------------------------------------------ misc API
    def zero_grad(self):
        self.optimizer.zero_grad()

    def clear_buffered_stats(self):
        pass

    def lr_step(self, epoch, val_loss=None):
        self.lr_scheduler.step(epoch, val_loss)
        return self.lr_step_update()

    def lr_step_update(self):
        return self.lr_scheduler.step_update(self.get_num_updates())

    def get_lr(self):
        return self.optimizer.get_lr()

    def get_model(self):
        return self._model

    def get_meter(self, name):
        return self.meters.get(name, None)

    def get_num_updates(self):
        return self._num_updates

    def set_num_updates(self, num_updates):
        self._num_updates = num_updates
        self.lr_step_update()

    def _prepare_sample(self, sample):
        if sample is None:
            return None
        sample = unwrap(sample)
        if sample is None or len(sample) == 0:
            return None
        if self.cuda:
            sample = move_to_device(sample, self.device)
        return sample

    def _set_seed(self):
        seed = self.args.seed + self.get_num_updates()
        if not (self.cuda and torch.cuda.is_current_stream_capturing()):   # (graph mode: set before capture)
            torch.manual_seed(seed)
            if self.cuda:
                torch.cuda.manual_seed(seed)
        ops.set_step_seed(seed)

    def _sync_stats(self):
        return self.args.distributed_world_size > 1

    def param_checksum(self):
        """Debug/race check: cheap checksum of the flat parameter buffer."""
        p = self.flat.param_flat
        w = torch.arange(1, 1 + min(p.numel(), 1 << 20), device=p.device, dtype=torch.float64)
        return float((p[:w.numel()].double() * w).sum().item() + p.double().sum().item())
