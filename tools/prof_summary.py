"""Summarise a rocprofv3 kernel trace into a markdown table.

``python tools/prof_summary.py RUN_results.db [--steps N] [--marker adam_k] [--top 30]``
(rocpd SQLite output of ``rocprofv3 --kernel-trace``), or a legacy
``*_kernel_stats.csv`` (``--stats --output-format csv``).

With ``--steps N`` only the last N training steps are kept: a step ends at each
dispatch whose name contains ``--marker`` (the fused optimizer kernel), so
warm-up / data-generation / tuning kernels do not pollute the per-step numbers.
Also reports the GEMM / non-GEMM split and the device idle time (gaps between
consecutive dispatches) inside those steps.
"""
import argparse
import collections
import csv
import sqlite3


def is_gemm(name):
    return name.startswith('Cijk_') or 'gemm' in name.lower() or name.startswith('rocblas')


def from_db(path, steps, marker):
    c = sqlite3.connect(path)
    rows = c.execute('select name, start, end from kernels order by start').fetchall()
    if steps:
        ends = [i for i, r in enumerate(rows) if marker in r[0]]
        if len(ends) > steps:
            rows = rows[ends[-steps - 1] + 1:ends[-1] + 1]
    gaps = sum(max(0, rows[i][1] - rows[i - 1][2]) for i in range(1, len(rows)))
    span = rows[-1][2] - rows[0][1] if rows else 0
    global GAP_ROWS
    GAP_ROWS = rows
    agg = collections.OrderedDict()
    for n, s, e in rows:
        a = agg.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
    return agg, gaps, span


GAP_ROWS = None


def gap_report(rows, steps, top):
    """Largest idle gaps, aggregated by (previous kernel, next kernel) pair."""
    agg = collections.defaultdict(lambda: [0, 0])
    for i in range(1, len(rows)):
        g = rows[i][1] - rows[i - 1][2]
        if g > 0:
            a = agg[(rows[i - 1][0][:60], rows[i][0][:60])]
            a[0] += 1
            a[1] += g
    print('\n| idle before | after | count/step | idle us/step |')
    print('|---|---|---|---|')
    for (a, b), (n, g) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print('| `{}` | `{}` | {:.1f} | {:.1f} |'.format(b.replace('|', '/'), a.replace('|', '/'), n / steps,
                                                       g / 1e3 / steps))


def from_csv(path):
    agg = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        agg[r['Name']] = [int(r['Calls']), float(r['TotalDurationNs'])]
    return agg, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('path')
    ap.add_argument('--steps', type=int, default=None)
    ap.add_argument('--marker', default='adam_k')
    ap.add_argument('--top', type=int, default=30)
    ap.add_argument('--gaps', type=int, default=0, help='also list the N largest idle-gap kernel pairs')
    ap.add_argument('--seq', type=float, default=0,
                    help='print the last step as a dispatch sequence, marking gaps over this many us')
    a = ap.parse_args()
    if a.path.endswith('.db'):
        agg, gaps, span = from_db(a.path, a.steps, a.marker)
    else:
        agg, gaps, span = from_csv(a.path)
    steps = a.steps or 1
    tot = sum(v[1] for v in agg.values())
    gemm = sum(v[1] for k, v in agg.items() if is_gemm(k))
    print('| kernel | calls/step | ms/step | % | avg us |')
    print('|---|---|---|---|---|')
    for name, (calls, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print('| `{}` | {:.1f} | {:.3f} | {:.2f} | {:.1f} |'.format(
            name[:90].replace('|', '/'), calls / steps, ns / 1e6 / steps, 100.0 * ns / tot, ns / 1e3 / calls))
    print('\nKernel time {:.2f} ms/step: GEMM {:.2f}, other {:.2f}; {:.0f} dispatches/step'.format(
        tot / 1e6 / steps, gemm / 1e6 / steps, (tot - gemm) / 1e6 / steps, sum(v[0] for v in agg.values()) / steps))
    if gaps is not None:
        print('Device span {:.2f} ms/step, idle between dispatches {:.2f} ms/step'.format(
            span / 1e6 / steps, gaps / 1e6 / steps))
    if a.gaps and GAP_ROWS:
        gap_report(GAP_ROWS, steps, a.gaps)
    if a.seq and GAP_ROWS:
        ends = [i for i, r in enumerate(GAP_ROWS) if a.marker in r[0]]
        rows = GAP_ROWS[ends[-2] + 1:ends[-1] + 1] if len(ends) > 1 else GAP_ROWS
        print('\n```')
        for i, (n, st, e) in enumerate(rows):
            g = (st - rows[i - 1][2]) / 1e3 if i else 0.0
            print('{:4d} {:>8.1f} {:>8.1f}  {}{}'.format(i, g, (e - st) / 1e3, '>> ' if g > a.seq else '   ', n[:150]))
        print('```')


if __name__ == '__main__':
    main()
