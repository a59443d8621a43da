"""HBM load balance across ranks (lddl_amd/balance.py): the exchange plan with gloo world_size 2
(CPU) and the full data path on the GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from lddl_amd.balance import gather_counts, plan_exchange


def _check_plan(counts):
    W, B = counts.shape
    target, send, first = plan_exchange(counts)
    assert (target.sum(0) == counts.sum(0)).all()
    assert (target.max(0) - target.min(0) <= 1).all()
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
        for _ in range(20):
            c = rng.integers(0, 50, (W, B))
            c[:, 0] = 0
            _check_plan(c)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    dist.init_process_group('gloo', init_method='tcp://127.0.0.1:{}'.format(port), rank=rank,
                            world_size=world)
    local = torch.tensor([[5, 0, 7], [1, 2, 3]][rank], dtype=torch.int64)
    counts = gather_counts(local)
    target, send, _ = plan_exchange(counts)
    # the row exchange of balance(): all_to_all_single of per-destination row payloads
    ids = torch.arange(int(local.sum()), dtype=torch.int64) + 1000 * rank
    send_n = [int(send[rank, k].sum()) for k in range(world)]
    recv_n = [int(send[j, rank].sum()) for j in range(world)]
    recv = torch.empty(sum(recv_n), dtype=torch.int64)
    dist.all_to_all_single(recv, ids, recv_n, send_n)
    out[rank] = (counts.tolist(), target[rank].tolist(), recv.tolist())
    dist.destroy_process_group()


def test_gather_and_exchange_gloo_world2():
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        res = dict(out)
    assert res[0][0] == res[1][0] == [[5, 0, 7], [1, 2, 3]]
    assert res[0][1] == [3, 1, 5] and res[1][1] == [3, 1, 5]
    assert sorted(res[0][2] + res[1][2]) == sorted(list(range(12)) + [1000 + i for i in range(6)])


@pytest.mark.gpu
def test_balance_single_rank_gpu():
    """World size 1: balance() regroups the table bin-major, stable, nothing lost."""
    from conftest import VOCAB_UNCASED
    from lddl_amd import synth
    from lddl_amd.balance import balance
    from lddl_amd.context import Context
    from lddl_amd.pairs import make_pairs
    ctx = Context(VOCAB_UNCASED)
    corp = synth.generate(seed=8, n_bytes=400_000)
    so = torch.from_numpy(corp.sent_off).cuda()
    ids, sl = ctx.tokenize(torch.from_numpy(corp.text).cuda(), so)
    part = torch.tensor([0, corp.n_doc // 2, corp.n_doc], dtype=torch.int64).cuda()
    pb = make_pairs(ctx, so, ids, sl, torch.from_numpy(corp.doc_sent_off).cuda(), part,
                    torch.tensor([1, 2], dtype=torch.int64).cuda(), seq=512, dup=2, masking=True)
    h = pb.to_host()
    bb = balance(ctx, pb, 8, 64)
    nt = h['num_tokens']
    bins = np.minimum((nt - 1) // 8, 63)
    order = np.argsort(bins, kind='stable')
    np.testing.assert_array_equal(np.diff(bb.bin_off), np.bincount(bins, minlength=64))
    tok = bb.tokens.cpu().numpy()
    off = bb.tok_off.cpu().numpy()
    la = bb.len_a.cpu().numpy()
    for i, q in enumerate(order[::5]):
        i = i * 5
        np.testing.assert_array_equal(tok[off[i]:off[i + 1]],
                                      h['tokens'][h['tok_off'][q]:h['tok_off'][q + 1]])
        assert la[i] == h['len_a'][q]
    pos = bb.pos.cpu().numpy().view(np.uint16)
    po = bb.pos_off.cpu().numpy()
    q = order[-1]
    np.testing.assert_array_equal(pos[po[-2]:po[-1]], h['pos'][h['pos_off'][q]:h['pos_off'][q + 1]])
