"""Kernels of a rocprofv3 trace from the last launch of a named kernel on, with start / end / duration
(ms relative to that launch): python tools/timeline_after.py gpurun_out/<dir>/trace [kernel] [n]"""
import glob
import os
import sqlite3
import sys


def main(src, name='plan_replay', n=30):
    db = glob.glob(os.path.join(src, '**', '*.db'), recursive=True)[0]
    rows = list(sqlite3.connect(db).execute('select name, start, end from kernels order by start'))
    i = [k for k, r in enumerate(rows) if name in r[0]][-1]
    t0 = rows[i][1]
    for nm, s, e in rows[i:i + n]:
        print('%8.2f %8.2f %7.2f  %s' % ((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, nm[:70]))


if __name__ == '__main__':
    main(sys.argv[1], *(sys.argv[2:3]), *([int(sys.argv[3])] if len(sys.argv) > 3 else []))
