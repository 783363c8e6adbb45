"""Long-horizon fp32 parity of the fp32-GEMM modes.

Trains BERT (default: base, phase-1 shape, dropout on) for ``--updates`` Adam updates
from the SAME seed on the SAME synthetic shards (a learnable bigram corpus, so the
loss actually falls) once per ``--modes`` entry, each in
its own child process (``--fp32-gemm native`` = fp32 MFMA, ``fp16x3`` = fp16-piece
emulation), records the per-update loss and grad norm, and compares every
mode against ``native``:

* per-update |loss difference| (max / mean, absolute and relative),
* per-update grad-norm relative difference,
* final parameters: ||p_mode - p_native|| / ||p_native - p_init|| (the divergence
  measured against how far training moved the weights) and / ||p_native||.

Dropout masks depend only on (seed, update) (Philox, ``ops.set_step_seed``), so the
trajectories are directly comparable.  Writes ``<out>/parity.md`` + ``parity.json``
(small; the parameter snapshots stay in a temp dir).

    python tools/parity_run.py --updates 300 --out gpurun_out/parity
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--updates', type=int, default=300)
    ap.add_argument('--modes', default='native,native#2,fp16x3',
                    help='"native#2" = a second native run (the run-to-run noise floor)')
    ap.add_argument('--model', default='base', choices=['base', 'tiny'])
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--seq', type=int, default=128)
    ap.add_argument('--max-pred', type=int, default=20)
    ap.add_argument('--lr', type=float, default=1e-4)
    ap.add_argument('--warmup-updates', type=int, default=30)
    ap.add_argument('--checkpoints', default='',
                    help='comma-separated update counts (e.g. 300,1000) at which the parameter divergence is also '
                         'measured (the final update always is): a growth trend of fp16x3 vs the noise floor')
    ap.add_argument('--out', default='gpurun_out/parity')
    ap.add_argument('--work', default=None, help='scratch dir for shards and parameter snapshots')
    ap.add_argument('--child', default=None, help=argparse.SUPPRESS)
    return ap.parse_args()


def child(a):
    """One training run in ``--fp32-gemm a.child``; saves losses, gnorms and parameters."""
    import torch
    from hetseq_9cme_amd import options, tasks
    from hetseq_9cme_amd.controller import Controller

    torch.cuda.set_device(0)
    argv = ['--task', 'bert', '--data', a.work, '--config_file', os.path.join(a.work, 'bert_config.json'),
            '--max-sentences', str(a.batch), '--fast-stat-sync', '--lr', str(a.lr),
            '--warmup-updates', str(a.warmup_updates), '--weight-decay', '0.01',
            '--total-num-update', str(max(10 * a.updates, 1000)), '--clip-norm', '25', '--num-workers', '2',
            '--log-format', 'none', '--disable-validation', '--no-save', '--distributed-world-size', '1']
    # mode = GEMM mode ['#' repeat], e.g. 'fp16x3#2'
    gemm_mode = a.child.split('#')[0]
    argv += ['--fp32-gemm', gemm_mode]
    args = options.parse_training_args(argv)
    args.device_id = 0
    args.distributed_rank = 0
    torch.manual_seed(args.seed)
    task = tasks.setup_task(args)
    model = task.build_model(args)
    ctrl = Controller(args, task, model)
    p0 = ctrl.flat.param_flat.detach().clone()
    epoch_itr = ctrl.get_train_iterator(epoch=0, load_dataset=True)
    ctrl.lr_step(epoch_itr.epoch)
    itr = iter(epoch_itr.next_epoch_itr(shuffle=True))
    losses, gnorms = [], []
    snaps = {}
    cks = sorted(int(x) for x in a.checkpoints.split(',') if x and 0 < int(x) < a.updates)
    t0 = time.time()
    for u in range(a.updates):
        if u in cks:
            snaps[u] = ctrl.flat.param_flat.detach().cpu().clone()
        out = ctrl.train_step([next(itr)])
        # (clone: the logged values may be views of persistent stats buffers)
        losses.append(torch.as_tensor(out['loss'], device='cuda').detach().float().reshape(()).clone())
        gnorms.append(torch.as_tensor(ctrl.meters['gnorm']._val, device='cuda').detach().float().reshape(()).clone())
        if (u + 1) % 50 == 0:
            print('[{}] update {} loss {:.4f} ({:.1f}s)'.format(a.child, u + 1, float(losses[-1]), time.time() - t0),
                  flush=True)
    torch.cuda.synchronize()
    torch.save({'loss': torch.stack(losses).cpu(), 'gnorm': torch.stack(gnorms).cpu(),
                'p0': p0.cpu(), 'p': ctrl.flat.param_flat.detach().cpu(), 'snaps': snaps},
               os.path.join(a.work, 'run_{}.pt'.format(a.child.replace('#', '_').replace(':', '-'))))


def main():
    a = parse()
    if a.child:
        return child(a)
    import torch
    from hetseq_9cme_amd.data.synthetic import BERT_BASE, BERT_TINY, write_bert_config, write_synthetic_bert_shards

    os.makedirs(a.out, exist_ok=True)
    a.work = a.work or tempfile.mkdtemp(prefix='hx_parity_')
    cfg = BERT_BASE if a.model == 'base' else BERT_TINY
    n = (a.updates + 2) * a.batch
    write_synthetic_bert_shards(a.work, n_files=max(1, (n + 8191) // 8192), samples_per_file=8192, seq_len=a.seq,
                                max_pred=a.max_pred, vocab_size=cfg['vocab_size'], seed=4321, split='train',
                                pattern='bigram')
    write_bert_config(os.path.join(a.work, 'bert_config.json'), **cfg)
    modes = a.modes.split(',')
    assert modes[0] == 'native', 'the first mode is the reference'
    base = [sys.executable, '-u', os.path.abspath(__file__), '--updates', str(a.updates), '--model', a.model,
            '--batch', str(a.batch), '--seq', str(a.seq), '--max-pred', str(a.max_pred), '--lr', str(a.lr),
            '--warmup-updates', str(a.warmup_updates), '--work', a.work, '--checkpoints', a.checkpoints]
    for m in modes:
        r = subprocess.run(base + ['--child', m])
        if r.returncode:
            sys.exit(r.returncode)
    runs = {m: torch.load(os.path.join(a.work, 'run_{}.pt'.format(m.replace('#', '_').replace(':', '-'))), weights_only=True)
            for m in modes}
    ref = runs['native']
    moved = (ref['p'].double() - ref['p0'].double()).norm().item()
    res = {'model': a.model, 'updates': a.updates, 'batch': a.batch, 'seq': a.seq, 'lr': a.lr,
           'warmup_updates': a.warmup_updates, 'dropout': 0.1, 'modes': {}}
    for m in modes:
        r = runs[m]
        dl = (r['loss'].double() - ref['loss'].double()).abs()
        rel_l = dl / ref['loss'].double().abs()
        rg = (r['gnorm'].double() - ref['gnorm'].double()).abs() / ref['gnorm'].double().abs()
        dp = (r['p'].double() - ref['p'].double()).norm().item()
        res['modes'][m] = {
            'final_loss': float(r['loss'][-1]), 'final_loss_avg10': float(r['loss'][-10:].mean()),
            'loss_absdiff_max': float(dl.max()), 'loss_absdiff_mean': float(dl.mean()),
            'loss_reldiff_max': float(rel_l.max()), 'gnorm_reldiff_max': float(rg.max()),
            'gnorm_reldiff_mean': float(rg.mean()),
            'param_diff_over_update': dp / moved if moved else float('nan'),
            'param_diff_over_norm': dp / ref['p'].double().norm().item(),
            'finite': bool(torch.isfinite(r['loss']).all() and torch.isfinite(r['gnorm']).all()),
        }
    # divergence at every checkpoint (parameters BEFORE update u, i.e. after u updates) and at the end
    ck = sorted(ref.get('snaps', {}).keys())
    res['divergence'] = {}
    for u in ck + [a.updates]:
        pr = ref['snaps'][u] if u in ref.get('snaps', {}) else ref['p']
        mv = (pr.double() - ref['p0'].double()).norm().item()
        row = {}
        for m in modes[1:]:
            pm = runs[m]['snaps'][u] if u in runs[m].get('snaps', {}) else runs[m]['p']
            row[m] = (pm.double() - pr.double()).norm().item() / mv if mv else float('nan')
        res['divergence'][u] = row
    res['loss_curve'] = {m: [round(float(x), 5) for x in runs[m]['loss']] for m in modes}
    res['gnorm_curve'] = {m: [round(float(x), 5) for x in runs[m]['gnorm']] for m in modes}
    with open(os.path.join(a.out, 'parity.json'), 'w') as f:
        json.dump(res, f)
    lines = ['# fp32-GEMM mode parity: BERT-{} x {} updates'.format(a.model, a.updates), '',
             'batch {} x seq {} (max_pred {}), Adam lr {} warmup {}, wd 0.01, clip 25, dropout 0.1, same seed and '
             'bigram-corpus shards for every mode; reference = `--fp32-gemm native` (fp32 MFMA); `native#2` = a '
             'second native run (run-to-run noise floor). Loss in the logged unit (sum / sample_size / ln 2, '
             'as the reference logs it).'.format(
                 a.batch, a.seq, a.max_pred, a.lr, a.warmup_updates), '',
             '| mode | final loss (avg last 10) | max abs loss diff | mean abs loss diff | max rel gnorm diff | '
             'mean rel gnorm diff | param diff / update norm | param diff / param norm |',
             '|---|---|---|---|---|---|---|---|']
    for m in modes:
        s = res['modes'][m]
        lines.append('| {} | {:.5f} | {:.3e} | {:.3e} | {:.3e} | {:.3e} | {:.3e} | {:.3e} |'.format(
            m, s['final_loss_avg10'], s['loss_absdiff_max'], s['loss_absdiff_mean'], s['gnorm_reldiff_max'],
            s['gnorm_reldiff_mean'], s['param_diff_over_update'], s['param_diff_over_norm']))
    others = modes[1:]
    lines += ['', 'Parameter difference / update norm after u updates (||p_mode - p_native|| / ||p_native - p_init||)'
              + (' and its ratio to the native#2 noise floor' if 'native#2' in others else '') + ':', '',
              '| updates | ' + ' | '.join(others) + (' | ratio to native#2 |' if 'native#2' in others else ' |'),
              '|---|' + '---|' * (len(others) + ('native#2' in others))]
    for u, row in sorted(res['divergence'].items()):
        cells = ['{:.3e}'.format(row[m]) for m in others]
        if 'native#2' in others:
            fl = row['native#2']
            cells.append(', '.join('{}: {:.2f}x'.format(m, row[m] / fl) for m in others if m != 'native#2' and fl))
        lines.append('| {} | '.format(u) + ' | '.join(cells) + ' |')
    lines += ['', 'Per-update loss (every {}th update):'.format(max(1, a.updates // 30)), '',
              '| update | ' + ' | '.join(modes) + ' |', '|---|' + '---|' * len(modes)]
    for u in range(0, a.updates, max(1, a.updates // 30)):
        lines.append('| {} | '.format(u + 1) + ' | '.join('{:.5f}'.format(float(runs[m]['loss'][u])) for m in modes)
                     + ' |')
    with open(os.path.join(a.out, 'parity.md'), 'w') as f:
        f.write('\n'.join(lines) + '\n')
    print('\n'.join(lines[:6 + len(modes)]))
    bad = [m for m in modes if not res['modes'][m]['finite']]
    if bad:
        sys.exit('non-finite trajectory: {}'.format(bad))


if __name__ == '__main__':
    main()
