"""Summarise a rocprofv3 ``--pmc ... --output-format csv`` counter file as markdown.

``python tools/pmc_summary.py gpurun_out/pmc_NAME/run_counter_collection.csv [--match wgrad]``
prints, per kernel (name truncated, optionally filtered by substring), the mean of every
counter per dispatch and the dispatch count.
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--match', default='')
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    order = []
    for r in csv.DictReader(open(a.csv)):
        name = r['Kernel_Name']
        if a.match and a.match not in name:
            continue
        short = name.replace('(anonymous namespace)::', '')
        short = (short[5:] if short.startswith('void ') else short).split('(')[0][:70]
        if short not in vals:
            order.append(short)
        vals[short][r['Counter_Name']].append(float(r['Counter_Value']))
    ctrs = sorted({c for k in vals for c in vals[k]})
    print('| kernel | dispatches | ' + ' | '.join(ctrs) + ' |')
    print('|---|---|' + '---|' * len(ctrs))
    for k in order:
        n = max(len(v) for v in vals[k].values())
        cells = []
        for c in ctrs:
            v = vals[k].get(c)
            cells.append('{:.4g}'.format(sum(v) / len(v)) if v else '')
        print('| `{}` | {} | {} |'.format(k, n, ' | '.join(cells)))


if __name__ == '__main__':
    main()
