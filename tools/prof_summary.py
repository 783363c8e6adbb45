"""Summarise a rocprofv3 --kernel-trace --stats CSV into a markdown table."""
import csv
import sys


def main(path, steps=None, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r['TotalDurationNs']) for r in rows)
    print('| kernel | calls | total ms | % | avg us |')
    print('|---|---|---|---|---|')
    for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
        print('| `{}` | {} | {:.2f} | {:.2f} | {:.1f} |'.format(r['Name'][:90].replace('|', '/'), r['Calls'],
                                                              float(r['TotalDurationNs']) / 1e6,
                                                              float(r['Percentage']), float(r['AverageNs']) / 1e3))
    print('\nTotal GPU kernel time: {:.2f} ms'.format(tot / 1e6) +
          (' ({:.2f} ms/step over {} steps)'.format(tot / 1e6 / steps, steps) if steps else ''))


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
