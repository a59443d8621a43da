"""Summarise a rocprofv3 kernel-trace database (rocpd .db) into a per-kernel CSV + text table.

    python tools/prof_summary.py gpurun_out/prof1 profiles/r01_bench_kernels
"""
import csv
import glob
import os
import sqlite3
import sys


def main(src, dst):
    db = glob.glob(os.path.join(src, '**', '*.db'), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute('select name, count(*), sum(duration), avg(duration), min(duration), '
                          'max(duration) from kernels group by name order by sum(duration) desc'))
    total = sum(r[2] for r in rows) or 1
    with open(dst + '.csv', 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(['kernel', 'calls', 'total_ns', 'avg_ns', 'min_ns', 'max_ns', 'percent'])
        for r in rows:
            w.writerow([r[0], r[1], int(r[2]), int(r[3]), int(r[4]), int(r[5]),
                        round(100.0 * r[2] / total, 3)])
    with open(dst + '.txt', 'w') as f:
        f.write('{:>10} {:>6} {:>14} {:>14} {:>7}  kernel\n'.format('total_ms', 'calls', 'avg_us',
                                                                    'max_us', '%'))
        for r in rows:
            name = r[0].replace('(anonymous namespace)::', '').split('(')[0]
            f.write('{:10.3f} {:6d} {:14.1f} {:14.1f} {:7.2f}  {}\n'.format(
                r[2] / 1e6, r[1], r[3] / 1e3, r[5] / 1e3, 100.0 * r[2] / total, name[:110]))
    print(open(dst + '.txt').read())


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
