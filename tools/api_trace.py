"""Long-blocking HIP API calls in the last training steps of a rocprofv3 run.

``rocprofv3 --hip-trace --kernel-trace -d DIR -o run -- python3 bench.py ...`` then
``python tools/api_trace.py DIR/.../run_results.db [--steps 3] [--min-us 200]``: lists
every HIP runtime call longer than ``--min-us`` inside the last N steps (a step ends at
the fused Adam kernel), with its thread id, so a host-side synchronisation that lets
the GPU drain between steps shows up by name.
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--min-us', type=float, default=200.0)
    ap.add_argument('--marker', default='adam_k')
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    views = [r[0] for r in c.execute("select name from sqlite_master where type in ('view','table')")]
    ks = c.execute('select name, start, end from kernels order by start').fetchall()
    ends = [r for r in ks if a.marker in r[0]]
    t0 = ends[-a.steps - 1][2] if len(ends) > a.steps else ks[0][1]
    t1 = ends[-1][2]
    if 'regions' not in views:
        print('views:', views)
        return
    cols = [r[1] for r in c.execute('pragma table_info(regions)')]
    tid = 'tid' if 'tid' in cols else ('thread_id' if 'thread_id' in cols else None)
    q = 'select name, start, end{} from regions where start >= ? and end <= ? order by start'.format(
        ', ' + tid if tid else '')
    rows = c.execute(q, (t0, t1)).fetchall()
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for r in rows:
        d = (r[2] - r[1]) / 1e3
        x = agg[r[0]]
        x[0] += 1
        x[1] += d
        x[2] = max(x[2], d)
    print('HIP API time per step over the last {} steps ({:.2f} ms/step wall):'.format(a.steps, (t1 - t0) / 1e6 / a.steps))
    print('| call | calls/step | ms/step | max us |')
    print('|---|---|---|---|')
    for n, (k, s, m) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print('| {} | {:.1f} | {:.3f} | {:.1f} |'.format(n, k / a.steps, s / 1e3 / a.steps, m))
    print('\nCalls over {} us (offset from window start, ms):'.format(a.min_us))
    for r in rows:
        d = (r[2] - r[1]) / 1e3
        if d >= a.min_us:
            print('{:9.3f} {:9.1f} us  {}{}'.format((r[1] - t0) / 1e6, d, r[0], '  tid={}'.format(r[3]) if tid else ''))
    # kernel gaps in the same window, for alignment
    print('\nDevice idle gaps over {} us (offset ms, gap us, next kernel):'.format(a.min_us))
    win = [k for k in ks if k[1] >= t0 and k[2] <= t1]
    for i in range(1, len(win)):
        g = (win[i][1] - win[i - 1][2]) / 1e3
        if g >= a.min_us:
            print('{:9.3f} {:9.1f} us  {}'.format((win[i][1] - t0) / 1e6, g, win[i][0][:80]))


if __name__ == '__main__':
    main()
