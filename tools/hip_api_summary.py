"""Longest HIP API calls and per-API totals from a rocprofv3 --hip-trace database, so the
database itself need not leave the GPU box. Also the kernel timeline gaps.

    python tools/hip_api_summary.py <trace dir> > summary.txt
"""
import glob
import os
import sqlite3
import sys
from collections import defaultdict


def main(src):
    db = glob.glob(os.path.join(src, '**', '*.db'), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute('select name, start, end from regions order by start'))
    if not rows:
        print('no regions')
        return
    t0 = rows[0][1]
    tot = defaultdict(lambda: [0, 0.0])
    for n, s, e in rows:
        tot[n][0] += 1
        tot[n][1] += (e - s) / 1e6
    print('per-API totals (ms):')
    for n, (k, ms) in sorted(tot.items(), key=lambda x: -x[1][1])[:25]:
        print('  {:10.2f} {:8d}  {}'.format(ms, k, n))
    print('calls >= 5 ms (start ms from first call):')
    for n, s, e in rows:
        if (e - s) / 1e6 >= 5:
            print('  {:10.2f} {:9.2f} ms  {}'.format((s - t0) / 1e6, (e - s) / 1e6, n))
    ks = list(c.execute('select name, start, end from kernels order by start'))
    print('kernels >= 2 ms:')
    for n, s, e in ks:
        if (e - s) / 1e6 >= 2:
            print('  {:10.2f} {:9.2f} ms  {}'.format((s - t0) / 1e6, (e - s) / 1e6, n[:70]))


if __name__ == '__main__':
    main(sys.argv[1])
