"""NER fine-tuning step time (BASELINE config 5: CoNLL-2003, batch 32 per update,
reference observed 0.214 s/update on 1 GPU).

Synthetic CoNLL-format sentences (8-40 words, CoNLL-2003-like lengths), a
BERT-base configuration with random init (no checkpoint download possible),
the real ``BertForTokenClassification`` task / collator / engine.  Prints one
JSON line with seconds per update (rank 0; the max over ranks).

One GPU: ``python tools/bench_ner.py [--steps 50] [--warmup 5] [--batch 32]``.
Data parallel, the reference's 4-GPU fine-tuning run
(STORE_RUN_FILE/Train_bert_fine_tuning_ner/bert_from_reddit_to_aida_ner/run_bert_fine_tuning_ner.sh:17-37,
--find-unused-parameters): ``python -m torch.distributed.run --nproc-per-node 4 --master-addr
127.0.0.1 --master-port P tools/bench_ner.py --gpus 4`` -- env:// rendezvous, rank r on GPU
LOCAL_RANK, ``--batch`` sentences per rank, timed region bracketed by barrier + device sync.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=50)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--precision', default='fp32', choices=['fp32', 'bf16'])
    ap.add_argument('--profile-phases', action='store_true', help='host/device time per step phase (stderr)')
    ap.add_argument('--gemm-tuning', default='table', choices=['off', 'table'])
    ap.add_argument('--graph-train-step', dest='graph_train_step', action='store_const', const='on', default='auto',
                    help='replay captured HIP graphs of the update (default auto = the framework default: on for '
                         'this task on a GPU)')
    ap.add_argument('--no-graph-train-step', dest='graph_train_step', action='store_const', const='off',
                    help='eager updates')
    ap.add_argument('--repeats', type=int, default=5,
                    help='timed blocks of --steps updates each; min / median / max of their s/update reported '
                         '(value = the median)')
    ap.add_argument('--no-overlap-wgrad', action='store_true', help='weight gradients on the compute stream')
    ap.add_argument('--overlap-wgrad', action='store_true', help='weight gradients on the side stream at every size')
    ap.add_argument('--cprofile', default=None, metavar='OUT',
                    help='after the timed steps, cProfile 20 more steps and write the top host functions to OUT')
    ap.add_argument('--gpus', type=int, default=1, help='ranks (launched by torch.distributed.run when > 1)')
    ap.add_argument('--backend', default='nccl', choices=['nccl', 'gloo'])
    ap.add_argument('--same-device', action='store_true', help='rehearsal: every rank on GPU 0')
    ap.add_argument('--model', default='base', choices=['base', 'tiny'])
    ap.add_argument('--fp32-gemm', default=None, choices=['fp16x3', 'native'],
                    help='fp32 GEMM mode (default: the framework default)')
    ap.add_argument('--force-reducer', action='store_true',
                    help='one GPU: run the gradient reducer on a one-rank RCCL group (buckets, used flags in the '
                         'stats all-reduce) -- with --graph-train-step, captured into the update graph')
    a = ap.parse_args()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    dev = 0 if a.same_device else local_rank
    torch.cuda.set_device(dev)
    from hetseq_9cme_amd import options, tasks
    from hetseq_9cme_amd.controller import Controller
    from hetseq_9cme_amd.data import iterators
    from hetseq_9cme_amd.data.synthetic import (BERT_BASE, BERT_TINY, WORDS, write_bert_config,
                                                write_synthetic_conll, write_vocab)
    from hetseq_9cme_amd.parallel import distributed as dist_utils
    n = (a.steps * max(1, a.repeats) + a.warmup + 22) * a.batch * world
    d = os.path.join(tempfile.gettempdir(), 'hx_ner_{}_{}_{}'.format(a.model, n, os.getpid() if world == 1 else
                                                                      os.environ.get('MASTER_PORT', '0')))
    vocab, cfg, tr = os.path.join(d, 'vocab.txt'), os.path.join(d, 'bert.json'), os.path.join(d, 'train.txt')
    if rank == 0 and not os.path.exists(os.path.join(d, 'READY')):
        os.makedirs(d, exist_ok=True)
        write_vocab(vocab, 30522, extra_words=WORDS)
        write_bert_config(cfg, **(BERT_BASE if a.model == 'base' else dict(BERT_TINY, vocab_size=30522)))
        write_synthetic_conll(tr, n, seed=0, min_len=8, max_len=40)
        open(os.path.join(d, 'READY'), 'w').close()
    while not os.path.exists(os.path.join(d, 'READY')):
        time.sleep(0.2)
    argv = ['--task', 'BertForTokenClassification', '--optimizer', 'adam', '--fast-stat-sync', '--lr', '5e-5',
            '--dict', vocab, '--config_file', cfg, '--train_file', tr, '--extension_file', 'conll',
            '--max-sentences', str(a.batch), '--num-workers', '2', '--find-unused-parameters',
            '--disable-validation', '--no-save', '--log-format', 'none', '--precision', a.precision,
            '--gemm-tuning', a.gemm_tuning]
    if a.profile_phases:
        argv.append('--profile-phases')
    if a.graph_train_step != 'auto':
        argv.append('--graph-train-step' if a.graph_train_step == 'on' else '--no-graph-train-step')
    if a.no_overlap_wgrad:
        argv.append('--no-overlap-wgrad')
    if a.overlap_wgrad:
        argv.append('--overlap-wgrad')
    if a.fp32_gemm:
        argv += ['--fp32-gemm', a.fp32_gemm]
    if a.force_reducer:
        argv.append('--force-reducer')
    args = options.parse_training_args(argv + ['--distributed-world-size', str(world)])
    args.device_id = dev
    args.distributed_backend = a.backend
    if world > 1:
        args.distributed_init_method = 'env://'
        args.distributed_rank = rank
        dist_utils.distributed_init(args)
    elif a.force_reducer:
        import socket
        with socket.socket() as sk:
            sk.bind(('127.0.0.1', 0))
            port = sk.getsockname()[1]
        args.distributed_init_method = 'tcp://127.0.0.1:{}'.format(port)
        args.distributed_rank = 0
        dist_utils.distributed_init(args)
    else:
        args.distributed_rank = 0
    torch.manual_seed(args.seed)
    task = tasks.setup_task(args)
    model = task.build_model(args)
    ctrl = Controller(args, task, model)
    epoch_itr = ctrl.get_train_iterator(epoch=0, load_dataset=True)
    ctrl.lr_step(epoch_itr.epoch)
    itr = iterators.GroupedIterator(epoch_itr.next_epoch_itr(shuffle=True), 1)
    for _ in range(a.warmup):
        ctrl.train_step(next(itr))
    torch.cuda.synchronize()
    ctrl.phase_report()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t_data = t_step = 0.0
    blocks = []
    for _ in range(max(1, a.repeats)):
        t0 = time.perf_counter()
        for _ in range(a.steps):
            ta = time.perf_counter()
            batch = next(itr)
            tb = time.perf_counter()
            ctrl.train_step(batch)
            t_data += tb - ta
            t_step += time.perf_counter() - tb
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.steps
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device='cuda')
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            dt = float(t.item())
        blocks.append(dt)
    nb = len(blocks)
    spread = sorted(blocks)
    dt = spread[nb // 2]
    t_data /= nb
    t_step /= nb
    gs = ctrl._graph_step
    replay_ms = None
    if gs is not None:
        print('graph-train-step: {} captures, {} replays'.format(gs.captures, gs.replays), file=sys.stderr)
        if gs.graphs:
            # device time of one captured update alone: its graph replayed back to back (same inputs)
            ent = max(gs.graphs.values(), key=lambda e: id(e))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(10):
                ent.graph.replay()
            e1.record()
            e1.synchronize()
            replay_ms = round(e0.elapsed_time(e1) / 10, 3)
    if a.cprofile:
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(20):
            ctrl.train_step(next(itr))
        torch.cuda.synchronize()
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats('tottime').print_stats(40)
        with open(a.cprofile, 'w') as f:
            f.write(buf.getvalue())
    if a.profile_phases:
        rep = ctrl.phase_report()
        for kind in ('host', 'device'):
            print('phases {} ms/step: '.format(kind) + ', '.join(
                '{}={:.2f}'.format(k, v * 1e3 / max(rep['steps'], 1)) for k, v in rep[kind].items()), file=sys.stderr)
    if rank == 0:
        print(json.dumps({'metric': 'NER fine-tune (BertForTokenClassification, BERT-{}) s/update'.format(a.model),
                          'value': round(dt, 5), 'unit': 's/update', 'higher_is_better': False,
                          'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
                          'reference_1gpu': 0.214, 'speedup_vs_reference': round(0.214 / dt, 1),
                          'batch': a.batch, 'global_batch': a.batch * world, 'dtype': a.precision,
                          'graph_train_step': gs is not None, 'force_reducer': a.force_reducer,
                          'repeats': nb, 's_per_update_min_median_max': [round(spread[0], 5), round(dt, 5),
                                                                         round(spread[-1], 5)],
                          'first_block_s': round(blocks[0], 5),
                          'fp32_gemm': args.fp32_gemm if a.precision == 'fp32' else None,
                          'graph_replays': gs.replays if gs is not None else 0,
                          'graph_replay_device_ms': replay_ms,
                          'host_ms': {'next_batch': round(t_data * 1e3 / a.steps, 3),
                                      'train_step_call': round(t_step * 1e3 / a.steps, 3)},
                          'parallelism': 'dp{}'.format(world) + (' (find-unused-parameters)' if world > 1 else ''),
                          'data': 'synthetic CoNLL-format sentences (8-40 words), random-init BERT-{}'.format(
                              a.model)}), flush=True)
    if world > 1 or a.force_reducer:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
