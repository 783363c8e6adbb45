"""Activity totals of a rocprofv3 rocpd SQLite trace: every table/view with start and end columns
-> row count, summed duration and span (``python tools/trace_tables.py RUN_results.db``); with
``--gaps`` also the kernel-to-kernel gaps of the last N kernels.  Finds device work that is not a
kernel (memory copies, barriers) in a captured update."""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    names = [r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")]
    for n in sorted(names):
        try:
            cols = [r[1] for r in c.execute('pragma table_info("{}")'.format(n))]
        except sqlite3.Error:
            continue
        if 'start' in cols and 'end' in cols:
            try:
                cnt, tot, lo, hi = c.execute('select count(*), sum(end - start), min(start), max(end) from "{}"'.format(n)).fetchone()
            except sqlite3.Error as e:
                print(n, 'error', e)
                continue
            print('{:40s} rows {:8d}  busy {:10.3f} ms  span {:10.3f} ms  cols {}'.format(
                n, cnt, (tot or 0) / 1e6, ((hi or 0) - (lo or 0)) / 1e6, ','.join(cols[:12])))
    for n in names:
        if 'copy' in n.lower() or 'memcpy' in n.lower():
            cols = [r[1] for r in c.execute('pragma table_info("{}")'.format(n))]
            print('--', n, cols)
            for r in c.execute('select * from "{}" limit 5'.format(n)).fetchall():
                print('   ', r)


if __name__ == '__main__':
    main()
