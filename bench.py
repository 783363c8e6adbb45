"""Headline benchmark: BERT-base phase-1 (seq 128) pre-training throughput.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.  For N > 1 it runs one
rank per GPU over RCCL either under ``torch.distributed.run`` (RANK / WORLD_SIZE in the env)
or, launched plainly, by spawning its N rank processes itself on a 127.0.0.1 rendezvous
before anything touches the GPU (``launch_ranks``; the reference's single-node self-spawn,
hetseq/train.py:233-243).  A world that is not N, or a communicator that did not reduce over
N ranks, exits non-zero.  Runs the real
framework path -- synthetic NVIDIA-schema HDF5 shards -> native reader -> pinned
staging on the HIP copy stream -> Controller.train_step (fused HIP kernels,
hand-written fp16x3 GEMMs for every BERT linear and the MLM decoder, flat-buffer
RCCL / xGMI reducer, fused norm/clip/Adam) -- with
random-init BERT-base weights (no network: no corpus, no checkpoint).

Config = BASELINE.json's: BERT-base (L12 H768 A12 V30522), seq 128, 20 masked
positions per sequence, per-GPU batch 128 (weak scaling: global batch 128*N),
Adam lr 1e-4 + warmup 10000 + wd 0.01, clip 25, fast stat sync, fp32-class compute
(the reference's precision; ``--fp32-gemm fp16x3`` = fp32 GEMMs as three fp16 piece
products of power-of-two-scaled operands, ops/gemm16.py; parity vs native fp32 over 300
updates in profiles/).  W untimed warm-up steps, then exactly K timed steps
bracketed by barrier + device synchronize; the max over ranks is reported.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = ('sec/step + samples/sec BERT-base phase-1 seq128 bs=128 at 1/2/4/8 MI355X; speedup vs 1 GPU')
# reference samples/s (README.md:65-68 via BASELINE.md): published 4 GPUs = 49.2, 8 GPUs = 95.2;
# 1/2 GPUs unpublished -> the 4-GPU row's per-GPU rate (12.3 seq/s) times N.
REF_SAMPLES_PER_SEC = {1: 12.3, 2: 24.6, 4: 49.2, 8: 95.2}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=128, help='per-GPU sequences per step')
    ap.add_argument('--seq', type=int, default=128)
    ap.add_argument('--max-pred', type=int, default=20)
    ap.add_argument('--precision', default='fp32', choices=['fp32', 'bf16'])
    ap.add_argument('--fp32-gemm', default='fp16x3', choices=['fp16x3', 'native'],
                    help='fp32 GEMMs: fp16x3 (default, fp32 class: ops/gemm16.py) or native f32 MFMA '
                         '(ops/fp32_mode.py)')
    ap.add_argument('--model', default='base', choices=['base', 'large', 'tiny'])
    ap.add_argument('--no-fused', action='store_true', help='torch-op baseline (A/B only)')
    ap.add_argument('--data-dir', default=None)
    ap.add_argument('--update-freq', type=int, default=1)
    ap.add_argument('--num-workers', type=int, default=4, help='batch loader threads')
    ap.add_argument('--allreduce-impl', default='rccl', choices=['rccl', 'xgmi'],
                    help='gradient all-reduce transport for N > 1 (RCCL, or the hand-written xGMI kernel)')
    ap.add_argument('--bucket-cap-mb', type=int, default=25)
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'],
                    help='process-group backend (gloo only for rehearsals, e.g. with --same-device)')
    ap.add_argument('--same-device', action='store_true',
                    help='rehearsal on a 1-GPU box: every rank uses GPU 0 (numbers are not per-GPU)')
    ap.add_argument('--gemm-tuning', default='table', choices=['off', 'table', 'online', 'retune'])
    ap.add_argument('--gemm-tuning-file', default=None)
    ap.add_argument('--overlap-wgrad', dest='overlap_wgrad', action='store_const', const='on', default='auto',
                    help='every weight-gradient GEMM on a side HIP stream (default auto: the side stream from '
                         '8192 token rows, the compute stream below; profiles/r6e_overlap_ab.txt)')
    ap.add_argument('--no-overlap-wgrad', dest='overlap_wgrad', action='store_const', const='off')
    ap.add_argument('--graph-train-step', action='store_true',
                    help='capture each whole update (forward, backward, all-reduce, optimizer) in a HIP graph '
                         'and replay it (utils/train_graph.py)')
    ap.add_argument('--profile-phases', action='store_true',
                    help='extra untimed steps reporting host time per step phase (stderr)')
    ap.add_argument('--sync-debug', action='store_true',
                    help='warn on every host<->device synchronisation during the extra steps')
    ap.add_argument('--nodes', default=None,
                    help='heterogeneous launch (BASELINE config 3), e.g. 5,3: one launcher process per "node" '
                         'spawns its GPU count of ranks like train.py mode (a) (--distributed-gpus g_n '
                         '--distributed-rank r_n), all meeting over one tcp:// rendezvous; every GPU stays '
                         'visible (device = node offset + local index)')
    ap.add_argument('--node-launcher', action='store_true', help=argparse.SUPPRESS)
    ap.add_argument('--node-gpus', type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument('--node-rank', type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument('--device-offset', type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument('--comm-load', default=None,
                    help='diagnostic A/B (untimed by the driver): CUS:US:LDSKB[:mask] -- before every step, a '
                         'stand-in comm kernel of CUS workgroups (LDSKB KiB of LDS each, so no GEMM workgroup fits '
                         'beside one) spins for US microseconds beside the step on its own stream, its workgroups '
                         'dealt over the XCDs like an RCCL kernel\'s ("mask": confined to CUs 0..CUS-1 by a CU-masked '
                         'stream instead) (tools/probe/comm_contention_probe.sh)')
    ap.add_argument('--comm-cus', default='0',
                    help='CUs left to the overlapped gradient all-reduce for N > 1 (train.py --comm-cus; '
                         'default 0 = no reservation and no RCCL channel cap)')
    ap.add_argument('--comm-probe-steps', type=int, default=5,
                    help='N > 1: untimed steps AFTER the timed region with the gradient collectives off, for '
                         'exposed_comm_ms (0 = skip)')
    ap.add_argument('--reserve-cus', type=int, default=0,
                    help='CUs the GEMM / weight-gradient plans leave to a concurrent comm kernel (--comm-cus)')
    ap.add_argument('--world', type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument('--init-method', default=None, help=argparse.SUPPRESS)
    ap.add_argument('--nodes-meta', default=None, help=argparse.SUPPRESS)
    return ap.parse_args()


def _bus_id(dev):
    try:
        return int(torch.cuda.get_device_properties(dev).pci_bus_id)
    except Exception:
        return -1


def allreduce_busbw(ctrl, world, reps=3):
    """Bus bandwidth (GB/s) of the gradient all-reduce alone: every reducer bucket (slices of
    the flat gradient buffer, the reducer's sizes and order) all-reduced ``reps`` times on the
    compute stream, timed between barriers; None without a reducer.  Runs after the timed
    region and leaves the gradients summed over ranks (the next step overwrites them)."""
    red = getattr(ctrl, 'reducer', None)
    if red is None or not red.enabled or world < 2:
        return None
    g = ctrl.flat.grad_flat
    sizes = [(s, e) for (s, e, _) in red.buckets]
    nbytes = sum(e - s for s, e in sizes) * g.element_size()
    for s, e in sizes:   # warm-up
        torch.distributed.all_reduce(g[s:e], group=red.group)
    torch.cuda.synchronize()
    torch.distributed.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        for s, e in sizes:
            torch.distributed.all_reduce(g[s:e], group=red.group)
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device='cuda')
    torch.distributed.all_reduce(dt, op=torch.distributed.ReduceOp.MAX)
    t = float(dt.item()) / reps
    return round(2.0 * (world - 1) / world * nbytes / t / 1e9, 1)


def launch_nodes(a):
    """Parent of a --nodes run: one launcher subprocess per "node" (the per-node qsub/ssh scripts
    of the reference, STORE_RUN_FILE/Train_mnist/node8gpu32_het/run.sh:3-10); returns the exit code."""
    import random
    import subprocess
    counts = [int(x) for x in a.nodes.split(',')]
    world = sum(counts)
    port = random.randint(20000, 30000)
    rest = [x for x in sys.argv[1:]]
    i = rest.index('--nodes')
    del rest[i:i + 2]
    procs, base = [], 0
    for g in counts:
        cmd = [sys.executable, os.path.abspath(__file__)] + rest + [
            '--node-launcher', '--node-gpus', str(g), '--node-rank', str(base), '--device-offset', str(base),
            '--world', str(world), '--init-method', 'tcp://127.0.0.1:{}'.format(port), '--gpus', str(world),
            '--nodes-meta', ','.join(str(c) for c in counts)]
        procs.append(subprocess.Popen(cmd))
        base += g
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


def launch_ranks(a):
    """Parent of a plain ``bench.py --gpus N`` (N > 1, no RANK in the env): N rank processes with
    the env a ``torch.distributed.run`` launch would give them (RANK = LOCAL_RANK = device index,
    WORLD_SIZE = N, MASTER_ADDR 127.0.0.1 and a free port).  This process never touches the GPU.
    When one rank fails the others (stuck in a collective) are terminated; returns the exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus), LOCAL_WORLD_SIZE=str(a.gpus),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print('bench: a rank exited with {}; stopping the others'.format(code), file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
    return rc


def node_worker(i, a):
    """One rank of a --nodes launch: rank = node base + i, device = node offset + i."""
    os.environ.update(RANK=str(a.node_rank + i), LOCAL_RANK=str(i), WORLD_SIZE=str(a.world))
    rc = run(a, a.node_rank + i, a.world, 0 if a.same_device else a.device_offset + i, a.init_method)
    if rc:
        sys.exit(rc)


def main():
    a = parse()
    if a.nodes and not a.node_launcher and 'RANK' not in os.environ:
        sys.exit(launch_nodes(a))
    if a.node_launcher:
        import torch.multiprocessing as mp
        mp.spawn(node_worker, args=(a,), nprocs=a.node_gpus, join=True)
        return
    if a.gpus > 1 and 'RANK' not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    if world != a.gpus:
        # e.g. torch.distributed.run with a different --nproc-per-node: never report an N-GPU
        # number from another world size
        print('bench: --gpus {} but the launch gives WORLD_SIZE {}'.format(a.gpus, world), file=sys.stderr)
        sys.exit(2)
    sys.exit(run(a, rank, world, 0 if a.same_device else local_rank, 'env://'))


def run(a, rank, world, dev_index, init_method):
    if a.no_fused:
        os.environ['HETSEQ_NO_FUSED'] = '1'
    from hetseq_9cme_amd import options
    from hetseq_9cme_amd.controller import Controller
    from hetseq_9cme_amd.data import iterators
    from hetseq_9cme_amd.data.synthetic import (BERT_BASE, BERT_LARGE, BERT_TINY, write_bert_config,
                                                write_synthetic_bert_shards)
    from hetseq_9cme_amd.parallel import distributed as dist_utils
    from hetseq_9cme_amd import tasks

    print('bench: rank {}/{} on device {} ({})'.format(rank, world, dev_index, init_method), file=sys.stderr,
          flush=True)
    if not torch.cuda.is_available():
        print('bench: rank {} sees no GPU'.format(rank), file=sys.stderr, flush=True)
        return 4
    torch.cuda.set_device(dev_index)

    cfg = {'base': BERT_BASE, 'large': BERT_LARGE, 'tiny': BERT_TINY}[a.model]
    data_dir = a.data_dir or os.path.join(tempfile.gettempdir(), 'hx_bench_s{}_p{}_n{}'.format(
        a.seq, a.max_pred, (a.warmup + a.steps + 2) * a.batch * a.update_freq * world))
    cfg_path = os.path.join(data_dir, 'bert_config.json')
    n_total = (a.warmup + a.steps + 2) * a.batch * a.update_freq * world
    per_file = 8192
    n_files = (n_total + per_file - 1) // per_file
    if rank == 0 and not os.path.exists(os.path.join(data_dir, 'READY')):
        os.makedirs(data_dir, exist_ok=True)
        write_synthetic_bert_shards(data_dir, n_files=n_files, samples_per_file=per_file, seq_len=a.seq,
                                    max_pred=a.max_pred, vocab_size=cfg['vocab_size'], seed=1234, split='train')
        write_bert_config(cfg_path, **cfg)
        open(os.path.join(data_dir, 'READY'), 'w').close()

    argv = ['--task', 'bert', '--data', data_dir, '--config_file', cfg_path, '--max-sentences', str(a.batch),
            '--fast-stat-sync', '--lr', '1e-4', '--warmup-updates', '10000', '--weight-decay', '0.01',
            '--total-num-update', '1000000', '--clip-norm', '25', '--num-workers', str(a.num_workers), '--log-format', 'none',
            '--disable-validation', '--no-save', '--precision', a.precision, '--fp32-gemm', a.fp32_gemm,
            '--distributed-world-size', str(world),
            '--update-freq', str(a.update_freq), '--gemm-tuning', a.gemm_tuning,
            '--allreduce-impl', a.allreduce_impl, '--bucket-cap-mb', str(a.bucket_cap_mb),
            '--comm-cus', str(a.comm_cus)]
    if a.profile_phases:
        argv += ['--profile-phases']
    if a.graph_train_step:
        argv += ['--graph-train-step']
    if a.overlap_wgrad != 'auto':
        argv += ['--overlap-wgrad' if a.overlap_wgrad == 'on' else '--no-overlap-wgrad']
    if a.gemm_tuning_file:
        argv += ['--gemm-tuning-file', a.gemm_tuning_file]
    args = options.parse_training_args(argv)
    args.device_id = dev_index
    args.distributed_backend = a.backend
    if world > 1:
        args.distributed_init_method = init_method
        args.distributed_rank = rank
        dist_utils.distributed_init(args)
        torch.distributed.barrier()
    else:
        args.distributed_rank = 0
    while not os.path.exists(os.path.join(data_dir, 'READY')):
        time.sleep(0.5)

    torch.manual_seed(args.seed)
    task = tasks.setup_task(args)
    model = task.build_model(args)
    ctrl = Controller(args, task, model)
    epoch_itr = ctrl.get_train_iterator(epoch=0, load_dataset=True)
    ctrl.lr_step(epoch_itr.epoch)
    itr = iterators.GroupedIterator(epoch_itr.next_epoch_itr(shuffle=True), a.update_freq)

    load = None
    if a.comm_load:
        from hetseq_9cme_amd.ops._ext import C as _C
        f = a.comm_load.split(':')
        cus, us, kb = int(f[0]), float(f[1]), float(f[2])
        if len(f) > 3 and f[3] == 'mask':
            st = _C().cu_masked_stream(0, cus)
        else:
            _load_stream = torch.cuda.Stream()
            st = _load_stream.cuda_stream
        load = (_C(), st, cus, us, int(kb * 1024), torch.zeros(256, dtype=torch.int32, device='cuda'))
    if a.reserve_cus:
        from hetseq_9cme_amd import ops as _ops
        _ops.set_reserved_cus(a.reserve_cus)

    prio = None
    if os.environ.get('HX_COMPUTE_PRIO') == '1':
        # experiment: the step on a high-priority stream (the weight-gradient side stream stays at
        # normal priority), so the dispatcher serves the critical path first when CUs free up
        torch.cuda.synchronize()
        prio = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
        print('bench: compute stream priority {}'.format(prio.priority), file=sys.stderr, flush=True)

    def step():
        samples = next(itr)
        if load is not None:
            c, st, n, us, lds, sink = load
            c.spin(n, us, lds, sink, st)
        if prio is not None:
            with torch.cuda.stream(prio):
                return ctrl.train_step(samples)
        return ctrl.train_step(samples)

    for _ in range(a.warmup):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    t_enq = time.perf_counter()   # the host's last launch: close to the end => the host bounds the step
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    host_ms = (t_enq - t0) / a.steps * 1000.0
    loss = float(out['loss']) if out is not None else float('nan')
    # every rank's time and a count of the ranks the communicator really reduced over
    per_rank = [elapsed]
    ranks_seen = 1
    if world > 1:
        times = torch.zeros(world, dtype=torch.float64, device='cuda')
        times[rank] = elapsed
        torch.distributed.all_reduce(times)
        per_rank = times.tolist()
        one = torch.ones(1, dtype=torch.float64, device='cuda')
        torch.distributed.all_reduce(one)
        ranks_seen = int(round(one.item()))
    elapsed = max(per_rank)
    ms = elapsed / a.steps * 1000.0
    exposed = None
    if world > 1 and a.comm_probe_steps > 0 and ctrl.reducer.enabled:
        # diagnostics AFTER the timed region: the same steps with the bucket collectives off
        # (gradients stay rank-local); the step-time difference is the all-reduce time the
        # backward does not hide
        ctrl.reducer.enabled = False
        torch.cuda.synchronize()
        torch.distributed.barrier()
        t1 = time.perf_counter()
        for _ in range(a.comm_probe_steps):
            step()
        torch.cuda.synchronize()
        nc = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device='cuda')
        torch.distributed.all_reduce(nc, op=torch.distributed.ReduceOp.MAX)
        ctrl.reducer.enabled = True
        exposed = ms - float(nc.item()) / a.comm_probe_steps * 1000.0
    busbw, dev_map = None, None
    if world > 1:
        busbw = allreduce_busbw(ctrl, world)
        # rank -> (node-local device index, PCI bus id): which GPUs the ranks really drove
        me = torch.tensor([rank, dev_index, _bus_id(dev_index)], dtype=torch.int64, device='cuda')
        allm = [torch.zeros_like(me) for _ in range(world)]
        torch.distributed.all_gather(allm, me)
        dev_map = {int(t[0]): [int(t[1]), '{:02x}'.format(int(t[2]))] for t in allm}
    global_batch = a.batch * a.update_freq * world
    value = global_batch * a.steps / elapsed
    ref = REF_SAMPLES_PER_SEC.get(world)
    if rank == 0:
        rec = {
            'metric': METRIC,
            'value': round(value, 2),
            'unit': 'samples/s',
            'n_gpus': world,
            'steps': a.steps,
            'warmup': a.warmup,
            'ms_per_step': round(ms, 3),
            'sec_per_step': round(ms / 1000.0, 5),
            # host time to enqueue the timed steps (rank 0): near ms_per_step when the host bounds it
            'host_enqueue_ms_per_step': round(host_ms, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': round(value / ref, 2) if ref else None,
            'dtype': 'fp32' if a.precision == 'fp32' else 'bf16',
            'data': 'synthetic (NVIDIA-schema HDF5 shards, random-init weights)',
            'config': {'model': 'bert-base (L12 H768 A12 V30522, 110.1M params)' if a.model == 'base' else a.model,
                       'global_batch': global_batch, 'per_gpu_batch': a.batch * a.update_freq,
                       'seq_len': a.seq, 'max_pred': a.max_pred,
                       'parallelism': 'dp{}'.format(world) + (' (nodes {})'.format('+'.join(
                           a.nodes_meta.split(','))) if a.nodes_meta else ''), 'optimizer': 'adam(fused)',
                       'nodes': [int(x) for x in a.nodes_meta.split(',')] if a.nodes_meta else None,
                       'fused_kernels': not a.no_fused, 'gemm_tuning': a.gemm_tuning,
                       'fp32_gemm': a.fp32_gemm if a.precision == 'fp32' else None,
                       'fp32_attention': 'fp16x3' if a.precision == 'fp32' and a.fp32_gemm == 'fp16x3' else None,
                       'allreduce': a.allreduce_impl if world > 1 else None},
            'final_logged_loss': round(loss, 5),
            'ranks_seen': ranks_seen,
            'per_rank_ms': {'min': round(min(per_rank) / a.steps * 1e3, 3),
                            'max': round(max(per_rank) / a.steps * 1e3, 3)},
            'exposed_comm_ms': round(exposed, 3) if exposed is not None else None,
            'transport': ('xgmi' if getattr(ctrl.reducer, 'xgmi', None) is not None else a.backend)
                         if world > 1 else None,
            'comm_cus': getattr(ctrl, 'comm_cus', 0),
            # N > 1: the gradient buckets' all-reduce measured alone after the timed region
            # (bus bandwidth = 2 (W - 1) / W x bytes / time, the RCCL-tests convention), the RCCL
            # channel cap in effect, and the rank -> [device index, PCI bus] map
            'allreduce_busbw_gbs': busbw,
            'rccl_max_nchannels': os.environ.get('NCCL_MAX_NCHANNELS') if world > 1 else None,
            'rank_devices': dev_map,
        }
        if ranks_seen != world:
            rec['error'] = 'communicator reduced over {} ranks, world is {}'.format(ranks_seen, world)
        print(json.dumps(rec), flush=True)
    if a.profile_phases or a.sync_debug:
        # diagnostics run AFTER the timed region so they cannot perturb it
        if a.sync_debug:
            torch.cuda.set_sync_debug_mode('warn')
        ctrl.phase_report()
        n, data_t = 5, 0.0
        t1 = time.perf_counter()
        for _ in range(n):
            td = time.perf_counter()
            samples = next(itr)
            data_t += time.perf_counter() - td
            ctrl.train_step(samples)
        host_t = time.perf_counter() - t1
        torch.cuda.synchronize()
        tot = time.perf_counter() - t1
        torch.cuda.set_sync_debug_mode(0)
        ph = ctrl.phase_report()
        ph['host']['data_next'] = data_t
        fmt = lambda d: ', '.join('{}={:.2f}'.format(k, v * 1e3 / n) for k, v in d.items())
        print('phases host ms/step: ' + fmt(ph['host']) + ' | host loop {:.2f} ms/step, device-complete {:.2f} '
              'ms/step'.format(host_t * 1e3 / n, tot * 1e3 / n), file=sys.stderr, flush=True)
        if ph['device']:
            print('phases device ms/step: ' + fmt(ph['device']), file=sys.stderr, flush=True)
            # host lead: how much queued work the GPU had when each phase was opened
            ctrl.phases.lead_trace = []
            ev0 = torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            ev0.record()
            t0 = time.perf_counter()
            for _ in range(2 * n):
                ctrl.train_step(next(itr))
            torch.cuda.synchronize()
            lead = ctrl.phases.host_lead(t0, ev0)
            ctrl.phase_report()
            print('host lead at phase start, ms (mean/min): ' + ', '.join(
                '{}={:.2f}/{:.2f}'.format(k, m, lo) for k, (m, lo) in lead.items()), file=sys.stderr, flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()
    if ranks_seen != world:
        print('bench: ranks_seen {} != world {}'.format(ranks_seen, world), file=sys.stderr)
        return 3
    return 0


if __name__ == '__main__':
    main()
