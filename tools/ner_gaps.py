"""Gaps between consecutive kernel dispatches of a rocprofv3 kernel trace (rocpd SQLite):
``python tools/ner_gaps.py RUN_results.db [--last 2000]`` -- the distribution of idle time
between kernels over the last N dispatches, and the largest gaps with the kernels around them
(is a graph-replayed update launch-bound on the device or waiting on the host?)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--last', type=int, default=2000)
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute('select name, start, end from kernels order by start').fetchall()
    rows = rows[-a.last:]
    gaps = [(rows[i][1] - rows[i - 1][2], i) for i in range(1, len(rows))]
    busy = sum(e - s for _, s, e in rows)
    span = rows[-1][2] - rows[0][1]
    print('{} dispatches, span {:.3f} ms, busy {:.3f} ms, idle {:.3f} ms'.format(
        len(rows), span / 1e6, busy / 1e6, (span - busy) / 1e6))
    g = sorted(x for x, _ in gaps)
    for q in (0.1, 0.5, 0.9, 0.99):
        print('gap p{:02d}: {:.2f} us'.format(int(q * 100), g[int(q * (len(g) - 1))] / 1e3))
    for x, i in sorted(gaps, reverse=True)[:15]:
        print('{:9.1f} us before {} (after {})'.format(x / 1e3, rows[i][0][:60], rows[i - 1][0][:60]))


if __name__ == '__main__':
    main()
