"""Load balancer: the count-only replay of the reference's _balance (lddl/dask/load_balance.py
:321-369) against plans produced by the reference itself (tests/golden/balance.json), and the
file-level CLI (shard layout, .num_samples.json, deletion of the inputs)."""
import json
import os
import types

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from conftest import GOLDEN

from lddl_amd.dask import load_balance as LB


def _uids(ready, counts):
    starts = {'part.{}.parquet_0'.format(i): s
              for i, s in enumerate(np.concatenate([[0], np.cumsum(counts)[:-1]]).tolist())}
    out = {}
    for sh in ready:
        u = []
        for src, a, n in sh.segments():
            s = starts[os.path.basename(src)]
            u += list(range(s + a, s + a + n))
        out[os.path.basename(sh.output_path)] = u
    return out


def _cases():
    with open(os.path.join(GOLDEN, 'balance.json')) as f:
        return json.load(f)


@pytest.mark.parametrize('case', _cases(), ids=lambda c: '{}-{}'.format(c['counts'], c['num_shards']))
def test_plan_matches_reference(case):
    counts, S = case['counts'], case['num_shards']
    paths = ['/in/part.{}.parquet_0'.format(i) for i in range(len(counts))]
    ready = LB.plan_balance(sorted(paths), [counts[i] for i in
                                           [int(os.path.basename(p).split('.')[1])
                                            for p in sorted(paths)]], S, '/out', '_0')
    got = _uids(ready, counts)
    if case['status'] == 'ok':
        assert got == case['shards']
    # every case (including the reference's non-terminating H6 and crashing H7 ones): balanced,
    # every sample exactly once
    sizes = [len(v) for v in got.values()]
    assert len(sizes) == S
    assert max(sizes) - min(sizes) <= 1
    assert sorted(u for v in got.values() for u in v) == list(range(sum(counts)))


def _write_parts(d, counts, bins=1):
    uid = 0
    for b in range(bins):
        for i, c in enumerate(counts):
            t = pa.table({'A': pa.array(['a{}'.format(u) for u in range(uid, uid + c)], pa.string()),
                          'uid': pa.array(range(uid, uid + c), pa.int64())})
            pq.write_table(t, os.path.join(d, 'part.{}.parquet_{}'.format(i, b)))
            uid += c
    return uid


def test_cli_binned(tmp_path):
    d = tmp_path / 'data'
    d.mkdir()
    total = _write_parts(str(d), [7, 3, 0, 11, 5], bins=3)
    args = LB.attach_args().parse_args(['--indir', str(d), '--num-shards', '4'])
    ns = LB.main(args)
    files = sorted(os.listdir(d))
    assert '.num_samples.json' in files
    assert not any(f.startswith('part.') for f in files)  # inputs deleted (no --keep-orig)
    with open(d / '.num_samples.json') as f:
        js = json.load(f)
    assert js == ns and len(js) == 12
    seen = []
    for b in range(3):
        sizes = []
        for k in range(4):
            t = pq.read_table(d / 'shard-{}.parquet_{}'.format(k, b))
            assert t.num_rows == js['shard-{}.parquet_{}'.format(k, b)]
            sizes.append(t.num_rows)
            seen += t.column('uid').to_pylist()
        assert max(sizes) - min(sizes) <= 1
    assert sorted(seen) == list(range(total))


def test_cli_empty_bin_and_more_shards_than_files(tmp_path):
    """H7 (num_shards > files) and H8 (bin without samples) produce complete layouts."""
    d = tmp_path / 'data'
    d.mkdir()
    _write_parts(str(d), [0, 0], bins=1)
    for i, c in enumerate([2, 1]):
        pq.write_table(pa.table({'A': pa.array(['x'] * c, pa.string()),
                                 'uid': pa.array(range(c), pa.int64())}),
                       d / 'part.{}.parquet_1'.format(i))
    out = tmp_path / 'out'
    LB.main(LB.attach_args().parse_args(['--indir', str(d), '--outdir', str(out), '--num-shards',
                                         '3', '--keep-orig']))
    for b, want in ((0, [0, 0, 0]), (1, [1, 1, 1])):
        got = [pq.read_table(out / 'shard-{}.parquet_{}'.format(k, b)).num_rows for k in range(3)]
        assert got == want
    assert os.path.exists(d / 'part.0.parquet_1')  # --keep-orig


def test_generate_num_samples_cache(tmp_path):
    _write_parts(str(tmp_path), [3, 4])
    LB.generate_num_samples_cache(['--indir', str(tmp_path)])
    with open(tmp_path / '.num_samples.json') as f:
        assert json.load(f) == {'part.0.parquet_0': 3, 'part.1.parquet_0': 4}


# ---- world size 2 (gloo): rank-striped footer reads + all_reduce, shard k written by rank k % 2
def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lb_worker(rank, world, port, indir, outdir, S):
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    import torch.distributed as dist
    LB.main(LB.attach_args().parse_args(['--indir', indir, '--outdir', outdir, '--num-shards',
                                         str(S), '--keep-orig']))
    dist.destroy_process_group()


@pytest.mark.parametrize('case', [c for c in _cases() if c['status'] == 'ok'],
                         ids=lambda c: '{}-{}'.format(c['counts'], c['num_shards']))
def test_cli_world2_matches_reference_plan(tmp_path, case):
    """balance_dask_output under two gloo ranks writes the shards of the reference's plan
    (tests/golden/balance.json, generated by the reference's _balance) with the rows in the
    reference's order, whichever rank wrote them."""
    import torch.multiprocessing as mp
    counts, S = case['counts'], case['num_shards']
    d, out = tmp_path / 'data', tmp_path / 'out'
    d.mkdir()
    uid = 0
    for i, c in enumerate(counts):
        pq.write_table(pa.table({'A': pa.array(['a{}'.format(u) for u in range(uid, uid + c)],
                                               pa.string()),
                                 'uid': pa.array(range(uid, uid + c), pa.int64())}),
                       d / 'part.{}.parquet_0'.format(i))
        uid += c
    mp.spawn(_lb_worker, args=(2, _free_port(), str(d), str(out), S), nprocs=2, join=True)
    with open(out / '.num_samples.json') as f:
        js = json.load(f)
    got = {k: pq.read_table(out / k).column('uid').to_pylist() for k in js}
    assert got == case['shards']
    assert js == {k: len(v) for k, v in case['shards'].items()}
