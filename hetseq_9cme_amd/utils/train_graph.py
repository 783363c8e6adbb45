"""HIP-graph replay of whole training updates (``--graph-train-step``).

Small-batch fine-tuning is host-bound: a BERT-base NER update at batch 32 launches ~180
kernels through ~100 autograd nodes, ~9 ms of Python/launch work against ~4.3 ms of GPU
kernels (profiles/r2_ner_*).  The reference has no answer to this (its loop is eager
PyTorch, hetseq/controller.py:222-377); on MI355X the answer is to capture the update --
forward, backward, stats, grad-norm / clip and the fused optimizer -- once per input shape
and replay it as ONE graph launch.

What makes an update replayable (everything else in the step is already free of host
synchronisation, see controller.py):

* dropout keys are read by the kernels from a device tensor (ops/rng.py) that is refilled
  before each replay, while the per-call-site stream ids are identical every update and
  stay baked into the graph;
* the optimizer's per-update hyper-parameters (Adam step size with bias correction and the
  scheduled LR, wd * lr; Adadelta lr) come from a device buffer (``device_hparams``) the
  host refills before each replay; step counters advance on the host as usual;
* the per-shape constants of the stats vector become fill nodes instead of a copy from a
  temporary pinned buffer; host meters are updated after each replay from the graph's
  static output tensors.

* with the gradient reducer on (world > 1, or ``--force-reducer``), the bucket all-reduces
  the backward hooks launch -- RCCL collectives on the side / comm streams, or the xGMI kernel
  -- and the stats all-reduce are captured as graph nodes; the per-parameter used flags of
  ``--find-unused-parameters`` are host-known at capture time and identical on every replay of
  the shape, so they ride in the stats vector as fill nodes (reference DDP setting of the NER
  runs: hetseq/controller.py:79-87, run_bert_fine_tuning_ner.sh:36).

Scope: one micro-batch per update, fp32 or bf16; with the reducer, an RCCL (``nccl``) process
group (gloo collectives are host-driven and cannot be captured).  Each distinct input shape is
warmed up eagerly ``warmup`` times, then captured into a graph that shares one memory pool with
the others (``max_graphs`` shapes at most; later new shapes, and anything else out of scope,
run eagerly).
"""
import collections

import torch

from ..ops.rng import get_rng


def _tensors(sample):
    if torch.is_tensor(sample):
        return [sample]
    if isinstance(sample, dict):
        return [t for k in sorted(sample) for t in _tensors(sample[k])]
    if isinstance(sample, (list, tuple)):
        return [t for x in sample for t in _tensors(x)]
    return []


def _clone_structure(sample):
    if torch.is_tensor(sample):
        return sample.clone()
    if isinstance(sample, dict):
        return {k: _clone_structure(v) for k, v in sample.items()}
    if isinstance(sample, (list, tuple)):
        return type(sample)(_clone_structure(x) for x in sample)
    return sample


def _capturable_group(c):
    """The reducer's collectives (and the stats all-reduce) can be captured: an RCCL group."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return False
    try:
        return dist.get_backend(c.reducer.group) == 'nccl'
    except Exception:
        return False


class _Entry(object):
    __slots__ = ('graph', 'static', 'out', 'meter_args', 'runs_sig')


class GraphedTrainStep(object):
    def __init__(self, controller, warmup=2, max_graphs=16, max_runs=None):
        self.ctrl = controller
        # one (step size, wd * lr) pair per optimizer run; a run covers >= 1 parameter, so the
        # parameter count bounds it (a fragmented --find-unused-parameters mask cannot overflow)
        if max_runs is None:
            max_runs = max(64, len(controller.flat.params))
        self.warmup = warmup
        self.max_graphs = max_graphs
        self.graphs = {}
        self.seen = collections.Counter()
        self.pool = None
        self.hparams = torch.zeros(2 * max_runs, dtype=torch.float32, device=controller.device)
        self.replays = 0
        self.captures = 0

    # ------------------------------------------------------------------ eligibility
    def _eligible(self, samples):
        c = self.ctrl
        if len(samples) != 1 or samples[0] is None or c._profile_phases:
            return False
        if c.reducer.enabled and not _capturable_group(c):
            return False
        # the xGMI all-reduce numbers its rounds from a host counter passed as a kernel argument
        # (xgmi_allreduce.hip): a captured launch would replay the capture-time round, its peer
        # waits would pass at once and ranks could read half-reduced buckets -- RCCL only
        if c.reducer.enabled and getattr(c.reducer, 'xgmi', None) is not None:
            return False
        # the slow stats path (all_gather_list + .item(), the used-flag .tolist()) synchronises
        # with the host and cannot be captured: with synced stats the update must use the fast path
        if c.reducer.enabled and c._sync_stats() and not c.fast_stat_sync:
            return False
        return not getattr(c.args, 'use_bmuf', False)

    def _key(self, sample):
        ts = _tensors(sample)
        if not ts or any(not t.is_cuda for t in ts):
            return None
        return tuple((tuple(t.shape), t.dtype) for t in ts)

    # ------------------------------------------------------------------ step
    def __call__(self, samples):
        if not self._eligible(samples):
            return NotImplemented
        c = self.ctrl
        sample = c._prepare_sample(samples[0])
        if sample is None:
            return NotImplemented
        key = self._key(sample)
        if key is None:
            return NotImplemented
        ent = self.graphs.get(key)
        if ent is None:
            self.seen[key] += 1
            if self.seen[key] <= self.warmup or len(self.graphs) >= self.max_graphs:
                return c._train_step([sample])
            return self._capture_and_run(key, sample)
        return self._replay(ent, sample)

    def _set_device_keys(self):
        rng = get_rng()
        t = rng.seed_tensor(self.ctrl.device)
        t.fill_(rng.seed)
        rng._dev[t.device.index][1] = rng.seed

    def _capture_and_run(self, key, sample):
        c = self.ctrl
        opt = c.optimizer
        ent = _Entry()
        ent.static = _clone_structure(sample)
        rng = get_rng()
        rng.seed_tensor(c.device)          # the key tensor must exist outside the graph pool
        opt.device_hparams = self.hparams
        c._set_seed()                      # torch's generators cannot be re-seeded inside a capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        rng.external = True
        try:
            # thread-local capture: the RCCL process group's watchdog thread keeps querying its
            # events during the capture; under the default global mode those queries fail
            # ('operation not permitted when stream is capturing') and the watchdog aborts the
            # process (seen once in test_graph_step_with_rccl_reducer_ner)
            with torch.cuda.graph(g, pool=self.pool, capture_error_mode='thread_local'):
                ent.out = c._train_step([ent.static])
        except Exception:
            # a failed capture must not leave the optimizer pointed at the graph's buffer:
            # this shape runs eagerly from now on
            opt.device_hparams = None
            self.seen[key] = -(1 << 30)
            raise
        finally:
            rng.external = False
        self.pool = g.pool()
        ent.graph = g
        ent.meter_args = c._captured_meter_args
        ent.runs_sig = opt._runs_sig
        if len(opt._hp_vals) > self.hparams.numel():
            raise RuntimeError('graph-captured update: {} optimizer runs exceed the hyper-parameter buffer'
                               .format(len(opt._runs_sig)))
        self.graphs[key] = ent
        self.captures += 1
        # the capture pass performed this update's host half (seed, step counters, num_updates,
        # hyper-parameters) without running anything on the device: write the device-side
        # inputs it could not, then run the update
        self._set_device_keys()
        opt._write_hparams()
        c.meters['train_wall'].start()
        g.replay()
        return self._after(ent)

    def _replay(self, ent, sample):
        c = self.ctrl
        opt = c.optimizer
        for dst, src in zip(_tensors(ent.static), _tensors(sample)):
            dst.copy_(src, non_blocking=True)
        c._set_seed()
        self._set_device_keys()
        opt._host_step()                     # step counters + this update's hyper-parameters
        if opt._runs_sig != ent.runs_sig:
            raise RuntimeError('graph-captured update: the optimizer ran different parameter ranges than at '
                               'capture time ({} vs {}); disable --graph-train-step for this model'
                               .format(opt._runs_sig, ent.runs_sig))
        c.meters['train_wall'].start()
        ent.graph.replay()
        c.set_num_updates(c.get_num_updates() + 1)
        c.task.update_step(c.get_num_updates())
        self.replays += 1
        return self._after(ent)

    def _after(self, ent):
        # the returned tensors are the graph's static outputs: the next replay overwrites
        # them (the meters consume them on the stream first, so the train loop is unaffected)
        c = self.ctrl
        c._update_meters(*ent.meter_args)
        c.meters['train_wall'].stop()
        return dict(ent.out)
