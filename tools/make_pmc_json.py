"""Per-kernel HBM traffic per launch from separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes
(bench.py --steps 1 --warmup 0) -> profiles/pmc_traffic.json, read by bench.py for
`roofline.traffic` when the batch size matches.

    python tools/make_pmc_json.py gpurun_out/<dir> <batch_bytes> <label>
"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarise  # noqa: E402


def short(name):
    n = name.replace('(anonymous namespace)::', '').replace('lddl::', '').replace('void ', '')
    return n.split('(')[0]


def main(src, batch_bytes, label):
    f = glob.glob(os.path.join(src, 'pmc_fetch', '**', '*.db'), recursive=True)[0]
    w = glob.glob(os.path.join(src, 'pmc_write', '**', '*.db'), recursive=True)[0]
    fr, _ = summarise(f)
    wr, _ = summarise(w)
    out = {'batch_bytes': batch_bytes, 'source': (
        'rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes over bench.py --steps 1 '
        '--warmup 0 ({}); mean per dispatch, KB -> bytes; no gfx950 x2 streaming-read correction '
        '(these kernels do byte-granular and gather loads, not the 16 B/lane streaming shape the '
        'correction is calibrated for)').format(label), 'kernels': {}}
    for k in sorted(set(fr) | set(wr)):
        fk = fr.get(k, {}).get('FETCH_SIZE', 0.0)
        wk = wr.get(k, {}).get('WRITE_SIZE', 0.0)
        out['kernels'][short(k)] = {'fetch_kb': fk, 'write_kb': wk,
                                    'hbm_bytes_per_launch': (fk + wk) * 1024.0}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
