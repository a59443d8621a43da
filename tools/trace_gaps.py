"""Timeline of a rocprofv3 kernel trace: kernels in start order with the idle gap before each
(gaps > threshold ms are where the host stalls the GPU).

    python tools/trace_gaps.py gpurun_out/<dir>/trace [min_gap_ms]
"""
import glob
import os
import sqlite3
import sys


def main(src, thr=1.0):
    db = glob.glob(os.path.join(src, '**', '*.db'), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute('select name, start, end from kernels order by start'))
    try:
        rows += [('<copy>', s, e) for s, e in c.execute('select start, end from memory_copies')]
    except sqlite3.Error:
        pass
    rows.sort(key=lambda r: r[1])
    t0 = rows[0][1]
    busy_end = t0
    total_gap = 0.0
    for name, s, e in rows:
        gap = (s - busy_end) / 1e6
        if gap > thr:
            total_gap += gap
            print('{:10.2f} ms  gap {:8.2f} ms before {}'.format((s - t0) / 1e6, gap, name[:80]))
        busy_end = max(busy_end, e)
    print('total gaps > {} ms: {:.1f} ms over {:.1f} ms'.format(thr, total_gap, (busy_end - t0) / 1e6))


if __name__ == '__main__':
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
