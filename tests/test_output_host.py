"""Host logic of the chunked device-to-host copy of rendered batches (output.chunk_groups,
output._Shifted): partition groups cover every partition once, in order, each within the byte
budget unless a single partition exceeds it, and a shifted byte column slices like the full one."""
import numpy as np
import pytest

from lddl_amd.output import Rendered, _Shifted, chunk_groups, table


def _offsets(rng, n_rows, mean):
    return np.concatenate([[0], np.cumsum(rng.integers(0, 2 * mean, n_rows))]).astype(np.int64)


@pytest.mark.parametrize('chunk', [0, 1, 50, 1000, 10 ** 9])
def test_chunk_groups_cover_in_order_within_budget(chunk):
    rng = np.random.default_rng(chunk)
    sizes = rng.integers(0, 6, 40)  # rows per partition, some empty
    part_rows = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    offs = [_offsets(rng, int(part_rows[-1]), 7), _offsets(rng, int(part_rows[-1]), 3)]
    groups = chunk_groups(part_rows, offs, chunk)
    assert [g[0] for g in groups] == [0] + [g[1] for g in groups[:-1]]
    assert groups[-1][1] == len(part_rows) - 1
    for p0, p1 in groups:
        r0, r1 = int(part_rows[p0]), int(part_rows[p1])
        nbytes = sum(int(o[r1]) - int(o[r0]) for o in offs)
        assert p1 > p0
        assert nbytes <= chunk or p1 == p0 + 1  # over budget only as a single partition
        if p1 < len(part_rows) - 1:  # the group stopped because the next partition would not fit
            r2 = int(part_rows[p1 + 1])
            assert sum(int(o[r2]) - int(o[r0]) for o in offs) > chunk
    if chunk >= 10 ** 9:
        assert groups == [(0, len(part_rows) - 1)]


def test_chunk_groups_no_partitions():
    assert chunk_groups(np.zeros(1, np.int64), [np.zeros(1, np.int64)], 100) == []


def test_shifted_column_builds_the_same_table():
    rng = np.random.default_rng(3)
    n = 30
    a_off, b_off = _offsets(rng, n, 9), _offsets(rng, n, 5)
    a = rng.integers(97, 123, int(a_off[-1]), dtype=np.uint8)
    b = rng.integers(97, 123, int(b_off[-1]), dtype=np.uint8)
    rn = rng.integers(0, 2, n).astype(bool)
    nt = rng.integers(3, 100, n).astype(np.uint16)
    full = Rendered(a_off, a, b_off, b, rn, nt)
    r0, r1 = 7, 19
    part = Rendered(a_off, _Shifted(a[a_off[r0]:a_off[r1]].copy(), int(a_off[r0])), b_off,
                    _Shifted(b[b_off[r0]:b_off[r1]].copy(), int(b_off[r0])), rn, nt)
    assert table(part, r0, r1, False, False).equals(table(full, r0, r1, False, False))
    assert [part.row(r) for r in range(r0, r1)] == [full.row(r) for r in range(r0, r1)]


def test_sharded_row_order_with_empty_ranges():
    """ShardWriters' (shard, bin, r0, r1) ranges come shard-major while the rows are bin-major;
    shards that got no rows of a bin have empty ranges that start where the next bin's first
    non-empty range starts. Sorted by (r0, r1) they still tile the rows, so the chunked copy runs
    (sorting on r0 alone put the empty range after the non-empty one)."""
    from lddl_amd.dask.bert.pretrain import _row_order
    rng = np.random.default_rng(5)
    for trial in range(200):
        S, B = int(rng.integers(1, 9)), int(rng.integers(1, 6))
        counts = rng.integers(0, 3, (B, S)) * (rng.random((B, S)) < 0.6)  # many empty
        starts, o = {}, 0
        for b in range(B):  # bin-major rows
            for s in range(S):
                starts[(s, b)] = (o, o + int(counts[b, s]))
                o += int(counts[b, s])
        ranges = [(s, b) + starts[(s, b)] for s in range(S) for b in range(B)]  # shard-major
        srt, bounds, contiguous = _row_order(ranges)
        assert contiguous, (trial, ranges)
        assert bounds[0] == 0 and bounds[-1] == o
        assert sorted(srt) == sorted(ranges)
    # a gap is still reported
    assert not _row_order([(0, 0, 0, 2), (1, 0, 3, 4)])[2]
