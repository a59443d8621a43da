"""Kernel statistics (rocprofv3 --stats style) from a rocprofv3 SQLite output (`*_results.db`):
one line per kernel name, sorted by total time.

    python tools/db_stats.py gpurun_out/<dir>/trace/k_results.db [top_n] > profiles/<name>.txt
"""
import sqlite3
import sys


def main(path, top=30):
    c = sqlite3.connect(path)
    rows = c.execute('select name, count(*), sum(end - start), avg(end - start), min(end - start), '
                     'max(end - start) from kernels group by name order by sum(end - start) desc'
                     ).fetchall()
    tot = sum(r[2] for r in rows) or 1
    print('# {}: {} kernel dispatches, {:.3f} ms of kernel time'.format(
        path, sum(r[1] for r in rows), tot / 1e6))
    print('{:>10} {:>6} {:>10} {:>10} {:>10} {:>6}  {}'.format(
        'total_ms', 'calls', 'avg_ms', 'min_ms', 'max_ms', '%', 'kernel'))
    for name, n, s, a, lo, hi in rows[:top]:
        print('{:10.3f} {:6d} {:10.4f} {:10.4f} {:10.4f} {:6.2f}  {}'.format(
            s / 1e6, n, a / 1e6, lo / 1e6, hi / 1e6, 100.0 * s / tot, name[:150]))


if __name__ == '__main__':
    main(sys.argv[1], *(int(a) for a in sys.argv[2:3]))
