"""HBM load balance across ranks (lddl_amd/balance.py).

* the plan (pure host) for random count matrices and shard counts;
* `balance_virtual` (W ranks in one process) and `balance` under gloo at world size 2 on the
  CPU, both running the product's plan / pack / regroup code with CPU data-movement
  primitives (tests/balance_util.py);
* on the GPU: `balance_virtual` over W = 1, 2, 4, 8 virtual ranks with the HIP kernels, on real
  pair tables, against the oracle's stable bin order (oracle.bin_samples).
Invariants follow lddl/dask/load_balance.py:321-378 (per bin, N or N+1 samples per shard)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from balance_util import TorchCpuOps, check_balanced, random_table
from lddl_amd.balance import balance, balance_virtual, plan_exchange, shard_targets


def _check_plan(counts, S=None):
    W, B = counts.shape
    target, send, first = plan_exchange(counts, S)
    assert (target.sum(0) == counts.sum(0)).all()
    st = shard_targets(counts, W if S is None else S)
    assert (st.max(0) - st.min(0) <= 1).all()
    assert (send.sum(1) == counts).all() and (send.sum(0) == target).all()
    for b in range(B):  # global (rank-major) order is preserved: receivers get contiguous runs
        gid = np.concatenate([[0], np.cumsum(counts[:, b])])
        got = []
        for k in range(W):
            for j in range(W):
                n = send[j, k, b]
                if n:
                    got += list(range(gid[j] + first[j, k, b], gid[j] + first[j, k, b] + n))
        assert got == list(range(counts[:, b].sum()))


def test_plan_exchange_cases():
    rng = np.random.default_rng(0)
    for W, B in ((1, 4), (2, 64), (3, 5), (8, 64)):
        for S in (None, W, 2 * W + 1, 64):
            for _ in range(10):
                c = rng.integers(0, 50, (W, B))
                c[:, 0] = 0
                _check_plan(c, S)


def test_plan_balanced_input_moves_nothing():
    c = np.full((4, 8), 10, np.int64)
    _, send, _ = plan_exchange(c)
    assert (send[np.arange(4), np.arange(4)] == c).all()
    assert send.sum() == c.sum()  # everything stays home


def _to_host_out(bb, ops):
    m = bb.materialize(ops)
    return (m.table.to_host(), bb.bin_off, bb.shards, bb.shard_counts)


@pytest.mark.parametrize('W,S,masking', [(1, 1, True), (1, 3, False), (2, 2, True), (3, 7, True),
                                         (4, 4, False), (8, 8, True), (8, 20, True)])
def test_balance_virtual_cpu(W, S, masking):
    rng = np.random.default_rng(W * 100 + S)
    ops = TorchCpuOps()
    pbs = [random_table(rng, int(rng.integers(0, 120)), 64, r, masking) for r in range(W)]
    outs = balance_virtual(ops, pbs, 8, 8, num_shards=S)
    check_balanced([pb.to_host() for pb in pbs], [_to_host_out(o, ops) for o in outs], 8, 8, S)
    if W == 1:
        assert outs[0].moved_rows == 0 and outs[0].rows is not None  # no copy at world size 1


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, S, out):
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:{}'.format(port), rank=rank,
                            world_size=world)
    rng = np.random.default_rng(1000 + rank)
    ops = TorchCpuOps()
    pb = random_table(rng, [150, 40][rank], 64, rank, True)
    bb = balance(None, pb, 8, 8, num_shards=S, ops=ops)
    out[rank] = (pb.to_host(), _to_host_out(bb, ops), bb.moved_rows)
    dist.destroy_process_group()


@pytest.mark.parametrize('S', [2, 5])
def test_balance_gloo_world2(S):
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, _free_port(), S, out), nprocs=2, join=True)
        res = dict(out)
    check_balanced([res[0][0], res[1][0]], [res[0][1], res[1][1]], 8, 8, S)
    assert res[1][2] > 0  # the lighter rank received rows over the exchange


# ---- GPU ------------------------------------------------------------------------------------
@pytest.fixture(scope='module')
def gpu_tables():
    from conftest import VOCAB_UNCASED
    from lddl_amd import synth
    from lddl_amd.context import Context
    from lddl_amd.pairs import make_pairs
    ctx = Context(VOCAB_UNCASED)
    corp = synth.generate(seed=8, n_bytes=1_200_000)
    so = torch.from_numpy(corp.sent_off).cuda()
    ids, sl = ctx.tokenize(torch.from_numpy(corp.text).cuda(), so)
    nparts = 8
    part = np.linspace(0, corp.n_doc, nparts + 1).astype(np.int64)
    pb = make_pairs(ctx, so, ids, sl, torch.from_numpy(corp.doc_sent_off).cuda(),
                    torch.from_numpy(part).cuda(), torch.arange(1, nparts + 1).cuda(), seq=512,
                    dup=2, masking=True)
    return ctx, pb


def _split_rows(pb, cuts):
    """Row ranges of one PairBatch as separate PairBatches (one per virtual rank)."""
    from lddl_amd.pairs import PairBatch
    out = []
    for a, z in zip(cuts[:-1], cuts[1:]):
        t0, t1 = int(pb.tok_off[a]), int(pb.tok_off[z])
        m0, m1 = int(pb.pos_off[a]), int(pb.pos_off[z])
        out.append(PairBatch(pb.tokens[t0:t1].clone(), pb.tok_off[a:z + 1] - t0,
                             pb.len_a[a:z].clone(), pb.is_random_next[a:z].clone(),
                             pb.pos[m0:m1].clone(), pb.labels[m0:m1].clone(),
                             pb.pos_off[a:z + 1] - m0))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize('W,S', [(1, 1), (2, 2), (4, 4), (8, 8), (8, 24), (3, 5)])
def test_balance_virtual_gpu(gpu_tables, W, S):
    """W virtual ranks on one GPU, HIP kernels: uneven row splits (skewed so that rows must
    move), checked against the invariants and, for the concatenated order, the oracle."""
    from oracle import oracle as O
    from lddl_amd.balance import HipOps
    ctx, pb = gpu_tables
    n = pb.n_pairs
    w = np.arange(1, W + 1, dtype=np.float64) ** 2
    cuts = np.concatenate([[0], np.round(np.cumsum(w) / w.sum() * n)]).astype(np.int64)
    pbs = _split_rows(pb, cuts)
    ops = HipOps(ctx)
    outs = balance_virtual(ops, pbs, 8, 64, num_shards=S)
    hosts = [p.to_host() for p in pbs]
    check_balanced(hosts, [_to_host_out(o, ops) for o in outs], 8, 64, S)
    # the oracle's stable bin order of the whole (rank-major) table is what the ranks hold
    nt = np.diff(pb.tok_off.cpu().numpy()) + 3
    eb, eo, ec = O.bin_samples(nt.astype(np.int32), 8, 64)
    assert sum(o.n_rows for o in outs) == n
    np.testing.assert_array_equal(sum(np.diff(o.bin_off) for o in outs), ec)
    if W > 1:
        assert sum(o.moved_rows for o in outs) > 0


@pytest.mark.gpu
def test_balance_world1_no_copy(gpu_tables):
    """World size 1 (collective driver without a process group): a row order over the table,
    nothing packed or moved; equal to the oracle's stable bin order."""
    from oracle import oracle as O
    ctx, pb = gpu_tables
    bb = balance(ctx, pb, 8, 64)
    assert bb.moved_rows == 0 and bb.rows is not None and bb.table is pb
    nt = np.diff(pb.tok_off.cpu().numpy()) + 3
    eb, eo, ec = O.bin_samples(nt.astype(np.int32), 8, 64)
    np.testing.assert_array_equal(bb.rows.cpu().numpy(), eo)
    np.testing.assert_array_equal(np.diff(bb.bin_off), ec)
    np.testing.assert_array_equal(bb.bin_ids().cpu().numpy(), eb[eo])
    assert bb.n_tokens == int(pb.tokens.numel())
