"""Per-kernel counters per launch from separate rocprofv3 --pmc passes over one bench step
(tools/prof_counters.sh) -> profiles/pmc_<tag>.json, read by bench.py for `roofline.traffic`
and the VALU-issue roofline when the batch size matches.

    python tools/make_pmc_json.py gpurun_out/<dir>/pmc <batch_bytes> <label> [git head] > profiles/pmc.json

The library's build id (lddl_build_id, a hash of its sources) is taken from the passes' bench
JSON lines, so bench.py can tell whether the counters describe the build it runs.

HBM bytes: FETCH_SIZE and WRITE_SIZE (KB) in their own passes. MI355X_MICROARCH.md: on gfx950
FETCH_SIZE tallies 128-B memory requests at 64 B, i.e. reports half the bytes of coalesced
streaming reads; the tokenizer's sequential text reads confirm an under-count here (FETCH_SIZE
8.1 GB for >= 10.65 GB of text and offsets read once). The read side is therefore doubled
(hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE), which can only overstate the traffic of
kernels whose requests are smaller than a line.
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


def bench_build_id(src):
    """lddl_build_id of the library the passes ran (the bench JSON line in the passes' logs)."""
    logs = glob.glob(os.path.join(src, '*.log')) + glob.glob(os.path.join(os.path.dirname(src.rstrip('/')), '*.log'))
    for log in sorted(logs):
        with open(log, errors='replace') as f:
            for ln in f:
                if ln.startswith('{') and '"build_id"' in ln:
                    try:
                        return json.loads(ln).get('build_id')
                    except ValueError:
                        pass
    return None


def main(src, batch_bytes, label, git_head=None):
    kernels = {}
    for sub in sorted(os.listdir(src)):
        dbs = glob.glob(os.path.join(src, sub, '**', '*.db'), recursive=True)
        if not dbs:
            continue
        res, _ = summarise(dbs[0])
        for k, cs in res.items():
            kernels.setdefault(short(k), {}).update(cs)
    for k, cs in kernels.items():
        if 'FETCH_SIZE' in cs or 'WRITE_SIZE' in cs:
            cs['hbm_bytes_per_launch'] = (2.0 * cs.get('FETCH_SIZE', 0.0) + cs.get('WRITE_SIZE', 0.0)) * 1024.0
    out = {'batch_bytes': batch_bytes, 'build_id': bench_build_id(src), 'git_head': git_head,
           'source': ('rocprofv3 --pmc passes (one counter group per run) over bench.py --steps 1 '
                      '--warmup 0 ({}); mean per dispatch; FETCH_SIZE/WRITE_SIZE KB -> '
                      'hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE counts '
                      '128-B read requests at 64 B; MI355X_MICROARCH.md HBM section)').format(label),
           'kernels': kernels}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == '__main__':
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], *sys.argv[4:5])
