"""The library / framework kernels of one training step in a rocprofv3 kernel trace (rocpd SQLite):
``python tools/small_kernels.py RUN_results.db [--marker adam_k]`` -- every dispatch of the last
complete step (between the last two optimizer kernels) that is not one of this package's own
kernels, with its duration and the own kernels around it, to find per-step glue worth fusing."""
import argparse
import sqlite3

OWN = ('void (anonymous namespace)::', '(anonymous namespace)::', 'hx::', 'amax_', 'slab_combine_k')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--marker', default='adam_k')
    a = ap.parse_args()
    rows = sqlite3.connect(a.db).execute('select name, start, end from kernels order by start').fetchall()
    idx = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(idx) < 2:
        raise SystemExit('fewer than two marker kernels')
    lo, hi = idx[-2] + 1, idx[-1] + 1
    step = rows[lo:hi]
    tot = 0.0

    def own(n):
        return n.startswith(OWN)
    for i, (n, s, e) in enumerate(step):
        if own(n):
            continue
        prev = next((step[j][0] for j in range(i - 1, -1, -1) if own(step[j][0])), '-')
        nxt = next((step[j][0] for j in range(i + 1, len(step)) if own(step[j][0])), '-')
        tot += (e - s) / 1e3
        print('{:8.1f} us  {:70s}  after {:50s}  before {}'.format((e - s) / 1e3, n[:70], prev[:50], nxt[:50]))
    print('non-package kernels in the step: {:.1f} us of {:.1f} us'.format(
        tot, sum(e - s for _, s, e in step) / 1e3))


if __name__ == '__main__':
    main()
