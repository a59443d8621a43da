"""Summarise rocprofv3 --pmc output (SQLite *_results.db) per kernel: mean counter value per dispatch.

    python tools/pmc_summary.py gpurun_out/pmc1/tok_results.db [kernel-substring]
"""
import sqlite3
import sys
from collections import defaultdict


def summarise(path, filt=''):
    c = sqlite3.connect(path)
    rows = c.execute('select kernel_name, dispatch_id, counter_name, value, duration, vgpr_count, '
                     'lds_block_size, grid_size, workgroup_size from counters_collection').fetchall()
    agg = defaultdict(lambda: defaultdict(list))
    meta = {}
    for k, d, n, v, dur, vg, lds, gs, ws in rows:
        if filt and filt not in k:
            continue
        agg[k][n].append(v)
        meta[k] = (vg, lds, gs, ws)
    out = {}
    for k, cs in agg.items():
        out[k] = {n: sum(v) / len(v) for n, v in cs.items()}
    return out, meta


if __name__ == '__main__':
    res, meta = summarise(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else '')
    for k, cs in res.items():
        print(k[:90], 'vgpr,lds,grid,wg =', meta[k])
        for n, v in sorted(cs.items()):
            print('   {:28s} {:.4g}'.format(n, v))
