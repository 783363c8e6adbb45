"""Where an NER fine-tuning update spends its time (BASELINE config 5, batch 32, BERT-base): the
same batch run (a) eagerly -- host enqueue time vs device time -- and (b) as a replayed HIP graph
of the whole update (utils/train_graph.py), replays back to back with no data loading in
between.  ``python tools/probe/ner_graph_probe.py [--precision fp32|bf16] [--fp32-gemm ...]
[--no-overlap-wgrad]``."""
import argparse
import os
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--precision', default='fp32', choices=['fp32', 'bf16'])
    ap.add_argument('--fp32-gemm', default='fp16x3', choices=['fp16x3', 'native'])
    ap.add_argument('--no-overlap-wgrad', action='store_true')
    ap.add_argument('--n', type=int, default=20)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    from hetseq_9cme_amd import options, tasks
    from hetseq_9cme_amd.controller import Controller
    from hetseq_9cme_amd.data import iterators
    from hetseq_9cme_amd.data.synthetic import BERT_BASE, WORDS, write_bert_config, write_synthetic_conll, write_vocab
    d = tempfile.mkdtemp(prefix='hx_ner_probe_')
    vocab = write_vocab(os.path.join(d, 'vocab.txt'), 30522, extra_words=WORDS)
    cfg = write_bert_config(os.path.join(d, 'bert.json'), **BERT_BASE)
    tr = write_synthetic_conll(os.path.join(d, 'train.txt'), 32 * 40, seed=0, min_len=8, max_len=40)
    argv = ['--task', 'BertForTokenClassification', '--optimizer', 'adam', '--fast-stat-sync', '--lr', '5e-5',
            '--dict', vocab, '--config_file', cfg, '--train_file', tr, '--extension_file', 'conll',
            '--max-sentences', '32', '--num-workers', '0', '--find-unused-parameters', '--disable-validation',
            '--no-save', '--log-format', 'none', '--precision', a.precision, '--fp32-gemm', a.fp32_gemm,
            '--graph-train-step', '--distributed-world-size', '1', '--pad-to-multiple-of', '64']
    if a.no_overlap_wgrad:
        argv.append('--no-overlap-wgrad')
    args = options.parse_training_args(argv)
    args.device_id = 0
    args.distributed_rank = 0
    torch.manual_seed(args.seed)
    task = tasks.setup_task(args)
    ctrl = Controller(args, task, task.build_model(args))
    ep = ctrl.get_train_iterator(epoch=0, load_dataset=True)
    ctrl.lr_step(ep.epoch)
    itr = iterators.GroupedIterator(ep.next_epoch_itr(shuffle=False), 1)
    batch = next(itr)
    sample = ctrl._prepare_sample(batch[0])
    print('batch shapes', {k: tuple(v.shape) for k, v in sample['net_input'].items()
                           if torch.is_tensor(v)} if isinstance(sample, dict) and 'net_input' in sample else '',
          flush=True)

    def timed(fn, n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(n):
            fn()
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        return (t1 - t0) * 1e3 / n, e0.elapsed_time(e1) / n, (t2 - t0) * 1e3 / n

    # eager: the same batch every time
    for _ in range(3):
        ctrl._train_step([sample])
    host, dev, wall = timed(lambda: ctrl._train_step([sample]), a.n)
    print('eager : host enqueue {:.2f} ms/update, device {:.2f} ms, wall {:.2f} ms'.format(host, dev, wall), flush=True)
    # graph: capture through the controller (2 eager warm-ups, then capture), then replay alone
    for _ in range(4):
        ctrl.train_step(batch)
    gs = ctrl._graph_step
    print('graph : captures {} replays {}'.format(gs.captures, gs.replays), flush=True)
    host, dev, wall = timed(lambda: ctrl.train_step(batch), a.n)
    print('graph : train_step host {:.2f} ms/update, device {:.2f} ms, wall {:.2f} ms'.format(host, dev, wall),
          flush=True)
    ent = next(iter(gs.graphs.values()))
    host, dev, wall = timed(lambda: ent.graph.replay(), a.n)
    print('graph : bare replay host {:.2f} ms, device {:.2f} ms, wall {:.2f} ms'.format(host, dev, wall), flush=True)


if __name__ == '__main__':
    main()
