"""Streaming load balance across ranks (lddl_amd/balance.py).

* the plan (pure host): `surplus_moves` against a brute-force two-list fill (only the imbalance
  moves), N / N+1 after every prefix of batches;
* `stream_virtual` (W ranks in one process, several batches) and `StreamBalancer` under gloo at
  world size 2 on the CPU, both running the product's plan / pack / regroup code with CPU
  data-movement primitives (tests/balance_util.py);
* on the GPU: `stream_virtual` over W = 1 .. 8 virtual ranks with the HIP kernels, on real pair
  tables split into batches, against the contract and the oracle's stable bin order.
Invariants follow lddl/dask/load_balance.py:321-378 (per bin, N or N+1 samples per shard)."""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from balance_util import TorchCpuOps, check_stream, random_table
from lddl_amd.balance import (StreamBalancer, balance, batch_shard_counts, rank_quota,
                              shard_targets, stream_virtual, surplus_moves)


def test_surplus_moves_brute_force():
    """Surplus ranks (rank order) fill deficit ranks (rank order); the moved total is exactly the
    imbalance sum(max(0, c - q)) and every rank ends at its quota."""
    rng = np.random.default_rng(0)
    for _ in range(300):
        W = int(rng.integers(1, 9))
        B = int(rng.integers(1, 4))
        counts = rng.integers(0, 30, (W, B))
        q = np.zeros((W, B), np.int64)
        for b in range(B):  # a random quota with the same total
            q[:, b] = np.bincount(rng.integers(0, W, counts[:, b].sum()), minlength=W)
        m, off = surplus_moves(counts, q)
        for b in range(B):
            pool = [(j, i) for j in range(W) for i in range(max(0, counts[j, b] - q[j, b]))]
            exp = np.zeros((W, W), np.int64)
            for k in range(W):
                need = max(0, q[k, b] - counts[k, b])
                take, pool = pool[:need], pool[need:]
                for j, i in take:
                    exp[j, k] += 1
                    if exp[j, k] == 1:
                        assert off[j, k, b] == i
            np.testing.assert_array_equal(m[:, :, b], exp)
        assert m.sum() == np.maximum(counts - q, 0).sum()
        np.testing.assert_array_equal(np.minimum(counts, q) + m.sum(0), q)


def test_batch_prefixes_balanced():
    """Any sequence of batches of any sizes leaves every shard within one row (N or N+1), and a
    rank's quota is the sum of its shards'."""
    rng = np.random.default_rng(1)
    for W, S, B in ((1, 1, 3), (2, 5, 4), (4, 4, 8), (8, 24, 64), (3, 2, 5)):
        prior = np.zeros(B, np.int64)
        tot = np.zeros((S, B), np.int64)
        for _ in range(6):
            counts = rng.integers(0, 40, (W, B))
            n = batch_shard_counts(prior, counts.sum(0), S)
            tot += n
            prior += counts.sum(0)
            np.testing.assert_array_equal(tot, shard_targets(prior[None, :], S))
            q = rank_quota(n, W)
            np.testing.assert_array_equal(q.sum(0), counts.sum(0))


def _to_host_out(bb, ops):
    m = bb.materialize(ops)
    return (m.table.to_host(), bb.bin_off, bb.shards, bb.shard_counts)


@pytest.mark.parametrize('W,S,masking,T', [(1, 1, True, 1), (1, 3, False, 3), (2, 2, True, 2),
                                           (3, 7, True, 3), (4, 4, False, 1), (8, 8, True, 2),
                                           (8, 20, True, 1), (2, 1, True, 2)])
def test_stream_virtual_cpu(W, S, masking, T):
    rng = np.random.default_rng(W * 100 + S + T)
    ops = TorchCpuOps()
    batches = [[random_table(rng, int(rng.integers(0, 120)), 64, r, masking, tag=t)
                for r in range(W)] for t in range(T)]
    outs = stream_virtual(ops, batches, 8, 8, num_shards=S)
    check_stream([[pb.to_host() for pb in pbs] for pbs in batches],
                 [[_to_host_out(o, ops) for o in os_] for os_ in outs], 8, 8, S,
                 moved=[[o.moved_rows for o in os_] for os_ in outs])
    if W == 1:
        assert all(o[0].moved_rows == 0 and o[0].rows is not None for o in outs)  # no copy


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
    sb = StreamBalancer(None, 8, 8, num_shards=S, ops=ops)
    res = []
    for t, n in enumerate([[150, 40], [0, 70], [33, 33]]):  # an empty batch on rank 0 too
        pb = random_table(rng, n[rank], 64, rank, True, tag=t)
        bb = sb.step(pb)
        res.append((pb.to_host(), _to_host_out(bb, ops), bb.moved_rows))
    out[rank] = (res, sb.all_shard_counts)
    dist.destroy_process_group()


@pytest.mark.parametrize('S', [2, 5])
def test_stream_gloo_world2(S):
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, _free_port(), S, out), nprocs=2, join=True)
        res = dict(out)
    T = len(res[0][0])
    cum = check_stream([[res[r][0][t][0] for r in range(2)] for t in range(T)],
                       [[res[r][0][t][1] for r in range(2)] for t in range(T)], 8, 8, S,
                       moved=[[res[r][0][t][2] for r in range(2)] for t in range(T)])
    for r in range(2):  # every rank's running layout is the same, and the one checked
        np.testing.assert_array_equal(res[r][1], cum)
    # rows crossed in both directions (batch 0: rank 0 -> 1, batch 1: rank 1 -> 0)
    assert res[1][0][0][2] > 0 and res[0][0][1][2] > 0


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
    """Row ranges of one PairBatch as separate PairBatches."""
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
@pytest.mark.parametrize('W,S,T', [(1, 1, 1), (1, 8, 3), (2, 2, 2), (4, 4, 1), (8, 8, 2),
                                   (8, 24, 1), (3, 5, 3)])
def test_stream_virtual_gpu(gpu_tables, W, S, T):
    """W virtual ranks x T batches on one GPU, HIP kernels: skewed row splits (rows must move),
    checked against the balance contract (moved rows == the imbalance); bin totals against the oracle's stable bin order."""
    from oracle import oracle as O
    from lddl_amd.balance import HipOps
    ctx, pb = gpu_tables
    n = pb.n_pairs
    w = np.tile(np.arange(1, W + 1, dtype=np.float64) ** 2, T)
    cuts = np.concatenate([[0], np.round(np.cumsum(w) / w.sum() * n)]).astype(np.int64)
    parts = _split_rows(pb, cuts)
    batches = [parts[t * W:(t + 1) * W] for t in range(T)]
    ops = HipOps(ctx)
    outs = stream_virtual(ops, batches, 8, 64, num_shards=S)
    check_stream([[p.to_host() for p in pbs] for pbs in batches],
                 [[_to_host_out(o, ops) for o in os_] for os_ in outs], 8, 64, S,
                 moved=[[o.moved_rows for o in os_] for os_ in outs])
    nt = np.diff(pb.tok_off.cpu().numpy()) + 3
    eb, eo, ec = O.bin_samples(nt.astype(np.int32), 8, 64)
    assert sum(o.n_rows for os_ in outs for o in os_) == n
    np.testing.assert_array_equal(sum(np.diff(o.bin_off) for os_ in outs for o in os_), ec)
    for os_ in outs:
        for o in os_:
            assert o.n_tokens == int(_to_host_out(o, ops)[0]['tok_off'][-1])
    if W > 1:
        assert sum(o.moved_rows for os_ in outs for o in os_) > 0


@pytest.mark.gpu
def test_balance_world1_no_copy(gpu_tables):
    """World size 1, one shard (collective driver without a process group): a row order over the
    table, nothing packed or moved; equal to the oracle's stable bin order."""
    from oracle import oracle as O
    ctx, pb = gpu_tables
    bb = balance(ctx, pb, 8, 64)
    assert bb.moved_rows == 0 and bb.rows is not None and bb.table is pb
    nt = np.diff(pb.tok_off.cpu().numpy()) + 3
    eb, eo, ec = O.bin_samples(nt.astype(np.int32), 8, 64)
    np.testing.assert_array_equal(bb.rows.cpu().numpy(), eo)
    np.testing.assert_array_equal(np.diff(bb.bin_off), ec)
    np.testing.assert_array_equal(bb.bin_ids(), eb[eo])
    assert bb.n_tokens == int(pb.tokens.numel())


@pytest.mark.gpu
def test_stream_virtual_gpu_balanced_moves_nothing(gpu_tables):
    """W = 8 virtual ranks dealt the rows round-robin (every rank within one row of every bin's
    share): only rounding remainders move, at most W - 1 rows per bin, where the round-robin deal
    of round 3 moved (W - 1) / W of all rows."""
    import torch as _t
    from lddl_amd.balance import HipOps, _gather_table
    ctx, pb = gpu_tables
    W, nb = 8, 64
    ops = HipOps(ctx)
    parts = [_gather_table(ops, pb, None, _t.arange(r, pb.n_pairs, W, device=pb.tok_off.device))
             for r in range(W)]
    outs = stream_virtual(ops, [parts], 8, nb, num_shards=W)
    moved = sum(o.moved_rows for o in outs[0])
    check_stream([[p.to_host() for p in parts]], [[_to_host_out(o, ops) for o in outs[0]]], 8, nb,
                 W, moved=[[o.moved_rows for o in outs[0]]])
    # per bin, each rank holds floor or ceil of its share and so does its quota: at most W - 1
    # rows move per bin (the round-robin deal of round 3 moved (W - 1) / W of all rows)
    assert moved <= (W - 1) * nb and moved < 0.2 * pb.n_pairs


@pytest.fixture
def nccl_world1():
    """A world-size-1 `nccl` (RCCL) process group on cuda:0, torn down after the test."""
    import datetime
    assert not dist.is_initialized()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:{}'.format(_free_port()),
                            rank=0, world_size=1, timeout=datetime.timedelta(seconds=120),
                            device_id=torch.device('cuda', 0))
    try:
        yield
    finally:
        dist.destroy_process_group()


def _same_out(a, b):
    ta, tb = a[0], b[0]
    assert set(ta) == set(tb)
    for k in ta:
        np.testing.assert_array_equal(np.asarray(ta[k]), np.asarray(tb[k]), err_msg=k)
    for x, y in zip(a[1:], b[1:]):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))


@pytest.mark.gpu
def test_rccl_branch_world1(gpu_tables, nccl_world1):
    """The device-tensor (RCCL) branch of the balance's collectives, which multi-GPU runs take and
    the gloo tests never do (lddl/dask/load_balance.py:210-223 replaced by all_gather /
    all_to_all_single over RCCL): per-bin counts all-gathered from a device tensor; all-to-all-v
    of a 16-bit id column moved as bytes, of int32 row metadata and of empty splits, all on the
    device; then StreamBalancer's exchange path forced on at world size 1, equal to the in-process
    driver (stream_virtual) batch by batch."""
    from lddl_amd import balance as B
    ctx, pb = gpu_tables
    dev = pb.tok_off.device
    assert dist.get_backend() == 'nccl' and not B._host_staged(None)
    c = torch.arange(3, 67, dtype=torch.int64, device=dev)
    np.testing.assert_array_equal(B.gather_counts(c, collective=True), c.cpu().numpy()[None])
    ids = pb.tokens[:4099]
    assert ids.element_size() == ctx.id_bytes
    b8 = ids.view(torch.uint8)
    r = B._a2a((b8, [b8.numel()], [b8.numel()]), None)
    assert r.is_cuda and r.dtype == torch.uint8 and torch.equal(r.view(ids.dtype), ids)
    meta = torch.arange(4 * 777, dtype=torch.int32, device=dev) * 7 - 5
    r = B._a2a((meta, [meta.numel()], [meta.numel()]), None)
    assert r.is_cuda and torch.equal(r, meta)
    r = B._a2a((torch.zeros(0, dtype=torch.uint8, device=dev), [0], [0]), None)
    assert r.is_cuda and r.numel() == 0
    # StreamBalancer with the exchange forced on (nothing moves at W = 1, but every split is
    # computed, packed, sent over RCCL and unpacked) against stream_virtual
    n = pb.n_pairs
    parts = _split_rows(pb, [0, n // 3, n // 3, n])  # the middle batch is empty
    sb = StreamBalancer(ctx, 8, 64, num_shards=4, collective=True)
    assert sb.multi
    ops = B.HipOps(ctx)
    ref = stream_virtual(ops, [[p] for p in parts], 8, 64, num_shards=4)
    for p, rv in zip(parts, ref):
        bb = sb.step(p)
        assert bb.moved_rows == 0
        _same_out(_to_host_out(bb, ops), _to_host_out(rv[0], ops))
    np.testing.assert_array_equal(sb.all_shard_counts, sum(r[0].all_shard_counts for r in ref))
