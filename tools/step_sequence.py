"""One training step's dispatch sequence from a rocprofv3 rocpd SQLite trace, in issue order:
index, kernel (short name), grid / workgroup size when the trace has them, duration (us) and the
gap before it -- names every GEMM call of the step by its place (QKV, attention out, FFN, ...).

``python tools/step_sequence.py RUN_results.db [--marker adam_k] [--step -2] [--min-us 0]``"""
import argparse
import sqlite3


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('void ', '')
    return n.split('(')[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--marker', default='adam_k')
    ap.add_argument('--step', type=int, default=-2, help='which step (python index over marker-delimited steps)')
    ap.add_argument('--min-us', type=float, default=0.0)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute('pragma table_info("kernels")')]
    want = [x for x in ('grid_size_x', 'grid_size', 'grid_x', 'workgroup_size_x', 'workgroup_size', 'workgroup_x',
                        'stream_id', 'queue_id') if x in cols]
    q = 'select name, start, end{} from kernels order by start'.format(''.join(', ' + w for w in want))
    rows = c.execute(q).fetchall()
    ends = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(ends) < 2:
        print('fewer than two steps found; columns:', cols)
        return
    e = ends[a.step]
    s = ends[ends.index(e) - 1] + 1
    step = rows[s:e + 1]
    t0 = step[0][1]
    print('| # | kernel | ' + ' | '.join(want) + ' | us | gap us | t us |')
    print('|---|---|' + '---|' * len(want) + '---|---|---|')
    prev_end = None
    for i, r in enumerate(step):
        dur = (r[2] - r[1]) / 1e3
        gap = (r[1] - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = r[2] if prev_end is None else max(prev_end, r[2])
        if dur < a.min_us:
            continue
        print('| {} | `{}` | {} | {:.1f} | {:.1f} | {:.0f} |'.format(i, short(r[0]), ' | '.join(str(x) for x in r[3:]),
                                                                  dur, gap, (r[1] - t0) / 1e3))
    print()
    print('columns available: ' + ', '.join(cols))


if __name__ == '__main__':
    main()
