"""Streaming load balance across GPUs (configs C3/C4).

The reference balances shards through the filesystem after preprocessing
(lddl/dask/load_balance.py:41-369: MPI Allreduce of per-file counts, then read / concat /
rewrite of parquet files, moving only `L - (L + S) // 2` samples between a large and a small
shard, :129-140) so that, per bin, every shard ends with N or N+1 samples (`Progress` targets,
:161-169). Here the same contract is met batch by batch while the samples are in HBM, so a rank
never holds more than one batch of pair tables, at any corpus size, and only the imbalance
crosses ranks:

  * per batch, each rank all-gathers its per-bin counts (int64[W, B], RCCL: the north star's
    bin-count all-gather). From them and the totals of earlier batches every rank derives the
    same plan (host integer math, replicated);
  * shard targets: after the batch, shard s holds cum_s(n) = n // S + (s < n % S) rows of a bin
    that has seen n rows in all — N or N+1 after EVERY batch (`shard_cum`); this batch adds
    cum_s(prior + total) - cum_s(prior) rows to shard s (`batch_shard_counts`);
  * shard s belongs to rank s * W // S; a rank's quota of bin b is the sum over its shards. Each
    rank keeps the first min(count, quota) of its bin-b rows (stable bin order); the surplus
    tails of the ranks above quota, in rank order, fill the ranks below quota, in rank order (a
    two-pointer merge, `surplus_moves`). So exactly sum_j max(0, c_jb - q_jb) rows of bin b move,
    the least any plan can move, and nothing when the ranks' batches are already balanced;
  * the moving rows cross in one all-to-all-v of row metadata and one per ragged column (token
    ids, masked positions as bytes, labels);
  * a rank's output of bin b is [its kept rows | received rows, by source rank], dealt in
    consecutive runs to its shards in ascending order: a row order over [own table | received
    rows] built on the device (`lddl_expand_segments`), materialised into one table (two-source
    ragged gathers) only when rows arrived.

At world size 1 nothing moves: the result is a row order over the batch's own table.

Every device step is a HIP kernel of liblddl_amd.so (`HipOps`); the plan is host integer math,
replicated on every rank. The per-rank phases (`RankBalance`: bin, plan, pack, unpack, regroup)
are shared by the collective driver (`StreamBalancer`, torch.distributed: RCCL on GPUs, gloo on
CPUs) and the in-process driver over virtual ranks (`stream_virtual`, W ranks on one device).
"""
import time
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.distributed as dist

from ._native import lib, check
from .context import _ptr, _stream
from .pairs import PairBatch


# ---- plan (host, replicated on every rank) ---------------------------------------------------
def shard_owner(num_shards, world):
    """Rank that owns shard s: contiguous runs of shards per rank."""
    return (np.arange(num_shards, dtype=np.int64) * world) // num_shards


def shard_cum(n, num_shards):
    """int64[S, B]: rows of each shard once n[b] rows of bin b have been dealt in all: N or N+1,
    the first n % S shards +1 (the reference's Progress targets, load_balance.py:161-169)."""
    n = np.asarray(n, np.int64)
    S = int(num_shards)
    return n[None, :] // S + (np.arange(S)[:, None] < (n % S)[None, :]).astype(np.int64)


def shard_targets(counts, num_shards):
    """int64[S, B]: samples of bin b per shard after sum(counts) rows (shard_cum of the total)."""
    total = np.asarray(counts, np.int64).reshape(-1, np.shape(counts)[-1]).sum(0)
    return shard_cum(total, num_shards)


def batch_shard_counts(prior, total, num_shards):
    """int64[S, B]: rows of bin b that one batch of total[b] rows adds to shard s, after prior[b]
    rows in earlier batches; the running layout stays N / N+1 after every batch."""
    return shard_cum(np.asarray(prior, np.int64) + total, num_shards) - shard_cum(prior, num_shards)


def rank_quota(shard_n, world):
    """int64[W, B]: rows of bin b that rank k must hold after the batch (its shards' counts)."""
    S, B = shard_n.shape
    q = np.zeros((world, B), np.int64)
    np.add.at(q, shard_owner(S, world), shard_n)
    return q


def surplus_moves(counts, quota):
    """(m, off), int64[W, W, B]: m[j, k, b] rows of bin b go from rank j to rank k; they are the
    rows off[j, k, b] .. + m of j's surplus (its bin-b rows past its quota). Surplus ranks in rank
    order fill deficit ranks in rank order; only the imbalance moves:
    m.sum() == sum(max(0, counts - quota))."""
    counts, quota = np.asarray(counts, np.int64), np.asarray(quota, np.int64)
    sur = np.maximum(counts - quota, 0)
    need = np.maximum(quota - counts, 0)
    s0 = np.cumsum(sur, 0) - sur
    d0 = np.cumsum(need, 0) - need
    lo = np.maximum(s0[:, None, :], d0[None, :, :])
    hi = np.minimum((s0 + sur)[:, None, :], (d0 + need)[None, :, :])
    m = np.maximum(hi - lo, 0)
    return m, np.where(m > 0, lo - s0[:, None, :], 0)


def _host_staged(group):
    """True when the backend moves host tensors only (gloo): device tensors are then staged
    through host memory (the one-GPU rehearsal of several ranks; RCCL takes them directly)."""
    return dist.get_backend(group) != 'nccl'


def gather_counts(local_counts, group=None, collective=None):
    """all_gather of the per-bin counts (RCCL when the tensor is on the GPU). collective=True runs
    the collective even at world size 1 (the GPU test of the RCCL branch on one device)."""
    W = dist.get_world_size(group) if dist.is_initialized() else 1
    if W == 1 and not collective:
        return local_counts.reshape(1, -1).cpu().numpy()
    flat = local_counts.contiguous().reshape(-1)
    if flat.is_cuda and _host_staged(group):
        flat = flat.cpu()
    out = torch.empty(W * flat.numel(), dtype=flat.dtype, device=flat.device)
    dist.all_gather_into_tensor(out, flat, group=group)
    return out.cpu().numpy().reshape((W,) + tuple(local_counts.shape))


# ---- data-movement primitives ----------------------------------------------------------------
def _alloc(n, dtype, dev):
    return torch.empty(max(int(n), 1), dtype=dtype, device=dev)[:int(n)]


class HipOps:
    """The balance's device primitives: HIP kernels of liblddl_amd.so on torch's current stream.
    Two-source row addressing: row r < n_a is row r of the first table, else row r - n_a of the
    second (include/lddl_amd.h, row movement)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def bin_stable(self, pb, bin_size, nbins):
        """(perm int64[n], counts int64[nbins]): stable regroup of the rows by
        bin_id = min((num_tokens - 1) // bin_size, nbins - 1) (binning.py:63-93)."""
        from .output import bin_stable
        perm, _, cnt = bin_stable(self.ctx, tok_off=pb.tok_off, bin_size=bin_size, nbins=nbins,
                                  with_bin_id=False)
        return perm, cnt

    def scan(self, x):
        from .output import scan
        return scan(self.ctx, x)

    def expand(self, src, seg, seg_off, dev):
        """int64 row list of the segment table seg[k] = (start, stride, direct) over outputs
        seg_off[k] .. seg_off[k+1] (lddl_expand_segments)."""
        total = int(seg_off[-1])
        out = _alloc(total, torch.int64, dev)
        if total:
            d_seg = torch.from_numpy(np.ascontiguousarray(seg, np.int64)).to(dev)
            d_off = torch.from_numpy(np.ascontiguousarray(seg_off, np.int64)).to(dev)
            check(lib.lddl_expand_segments(_stream(), _ptr(src), _ptr(d_seg), _ptr(d_off),
                                           len(seg), total, _ptr(out)))
        return out

    def take(self, a, n_a, b, rows, dtype=None):
        out = _alloc(rows.numel(), a.dtype, a.device)
        check(lib.lddl_take(_stream(), _ptr(a), int(n_a), _ptr(b), a.element_size(), _ptr(rows),
                            rows.numel(), _ptr(out)))
        return out

    def ragged_offsets(self, off_a, n_a, off_b, rows):
        out = torch.empty(rows.numel() + 1, dtype=torch.int64, device=off_a.device)
        check(lib.lddl_ragged_offsets(self.ctx.handle, _stream(), _ptr(off_a), int(n_a),
                                      _ptr(off_b), _ptr(rows), rows.numel(), _ptr(out)))
        return out

    def gather(self, a, off_a, n_a, b, off_b, rows, dst_off, total):
        out = _alloc(total, a.dtype, a.device)
        if rows.numel():
            check(lib.lddl_gather_ragged(_stream(), _ptr(a), _ptr(off_a), int(n_a), _ptr(b),
                                         _ptr(off_b), a.element_size(), _ptr(rows), rows.numel(),
                                         _ptr(dst_off), _ptr(out)))
        return out

    def meta_pack(self, pb, rows):
        out = _alloc(4 * rows.numel(), torch.int32, pb.tok_off.device)
        check(lib.lddl_pairs_meta_pack(_stream(), _ptr(pb.tok_off), _ptr(pb.len_a),
                                       _ptr(pb.is_random_next), _ptr(pb.pos_off), _ptr(rows),
                                       rows.numel(), _ptr(out)))
        return out

    def meta_unpack(self, meta):
        n = meta.numel() // 4
        dev = meta.device
        ntok, nmask = _alloc(n, torch.int64, dev), _alloc(n, torch.int64, dev)
        len_a, is_rn = _alloc(n, torch.int32, dev), _alloc(n, torch.uint8, dev)
        check(lib.lddl_pairs_meta_unpack(_stream(), _ptr(meta), n, _ptr(ntok), _ptr(len_a),
                                         _ptr(is_rn), _ptr(nmask)))
        return ntok, len_a, is_rn, nmask


def _host_at(ops, off, idx):
    """off[idx] for a few host indices (one small device take + copy)."""
    if not len(idx):
        return np.zeros(0, np.int64)
    i = torch.from_numpy(np.asarray(idx, np.int64)).to(off.device)
    return ops.take(off, off.numel(), None, i).cpu().numpy()


# ---- result ----------------------------------------------------------------------------------
@dataclass
class BalancedBins:
    """One rank's share of one batch after the balance, bin-major.

    Output row i is row `rows[i]` of `table` (rows None = identity, i.e. the table itself is
    bin-major). Bin b is output rows [bin_off[b], bin_off[b+1]); inside a bin the rank's shards
    follow each other: shard shards[m] holds shard_counts[m, b] of them, in global order."""
    table: PairBatch
    rows: torch.Tensor
    bin_off: np.ndarray
    shards: list = field(default_factory=list)
    shard_counts: np.ndarray = None
    n_tokens: int = 0              # sum of len(A) + len(B) over the output rows
    moved_rows: int = 0            # rows received from other ranks
    all_shard_counts: np.ndarray = None  # int64[S, B]: this batch's rows per shard and bin (all ranks)

    @property
    def n_rows(self):
        return int(self.bin_off[-1])

    def shard_range(self, m, b):
        """Output rows [r0, r1) of this rank's m-th shard in bin b."""
        r0 = int(self.bin_off[b] + self.shard_counts[:m, b].sum())
        return r0, r0 + int(self.shard_counts[m, b])

    def bin_ids(self):
        """int64[n_rows] bin id of every output row (host)."""
        return np.repeat(np.arange(len(self.bin_off) - 1, dtype=np.int64), np.diff(self.bin_off))

    def materialize(self, ops):
        """The contiguous bin-major table (copies only if `rows` is not the identity)."""
        if self.rows is None:
            return self
        t = _gather_table(ops, self.table, None, self.rows)
        return BalancedBins(t, None, self.bin_off, self.shards, self.shard_counts, self.n_tokens,
                            self.moved_rows, self.all_shard_counts)


def _gather_table(ops, pa, pr, rows):
    """Rows `rows` of the virtual concatenation [pa | pr] (pr may be None) as one contiguous
    PairBatch: every output row copied once, from whichever table holds it."""
    dev = pa.tok_off.device
    na = pa.n_pairs

    def col(xa, xr):
        return ops.take(xa, na, xr, rows)

    def ragged(xa, oa, xr, orr):
        off = ops.ragged_offsets(oa, na, orr, rows)
        n = int(off[-1].item())
        return ops.gather(xa, oa, na, xr, orr, rows, off, n), off, n
    pr_ = pr if pr is not None else PairBatch(None, None, None, None)
    tokens, tok_off, _ = ragged(pa.tokens, pa.tok_off, pr_.tokens, pr_.tok_off)
    out = PairBatch(tokens, tok_off, col(pa.len_a, pr_.len_a),
                    col(pa.is_random_next, pr_.is_random_next))
    if pa.pos is not None:
        out.pos, out.pos_off, n_m = ragged(pa.pos, pa.pos_off, pr_.pos, pr_.pos_off)
        out.labels = ops.gather(pa.labels, pa.pos_off, na, pr_.labels, pr_.pos_off, rows,
                                out.pos_off, n_m)
        out.n_masked = n_m
    assert out.tokens.device == dev
    return out


# ---- per-rank phases -------------------------------------------------------------------------
class RankBalance:
    """One rank's part of one batch: bin (local), plan (replicated), pack / unpack around the two
    exchange rounds (row metadata, then the ragged columns), regroup."""

    def __init__(self, ops, pb, bin_size, nbins, rank, world, num_shards=None):
        self.ops, self.pb, self.nbins = ops, pb, nbins
        self.me, self.W = rank, world
        self.S = world if num_shards is None else int(num_shards)
        self.dev = pb.tok_off.device
        self.masking = pb.pos is not None
        if self.masking:
            assert pb.pos.element_size() == 2
            assert pb.labels.element_size() == pb.tokens.element_size()
        assert pb.tokens.element_size() in (2, 4)  # uint16 or int32 ids (Context.id_dtype)
        self.perm, self.local_counts = ops.bin_stable(pb, bin_size, nbins)

    # plan ----------------------------------------------------------------------------------
    def set_plan(self, counts, prior):
        """counts int64[W, B]: every rank's rows per bin in this batch; prior int64[B]: rows of
        each bin in earlier batches (all ranks). Replicated: every rank computes the same plan."""
        W, me, B, S = self.W, self.me, self.nbins, self.S
        self.counts = np.asarray(counts, np.int64)
        shard_n = batch_shard_counts(prior, self.counts.sum(0), S)   # [S, B]
        quota = rank_quota(shard_n, W)                                # [W, B]
        m, off = surplus_moves(self.counts, quota)                    # [W, W, B]
        self.shards = [int(x) for x in np.nonzero(shard_owner(S, W) == me)[0]]
        mine = np.asarray(self.shards, np.int64)
        keep = np.minimum(self.counts[me], quota[me])
        bin0 = np.concatenate([[0], np.cumsum(self.counts[me])])[:-1]
        # rows leaving this rank: destination-major, then bin; one contiguous run of the bin's
        # surplus tail each (through perm, the stable bin order)
        seg, lens = [], []
        for k in range(W):
            for b in range(B):
                c = int(m[me, k, b])
                if c:
                    seg.append((int(bin0[b] + keep[b] + off[me, k, b]), 1, 0))
                    lens.append(c)
        self._send_seg = (seg, lens)
        self.send_rows_per_dst = [int(x) for x in m[me].sum(1)]
        self.n_send = sum(self.send_rows_per_dst)
        self.recv_rows_per_src = [int(x) for x in m[:, me].sum(1)]
        self.n_recv = sum(self.recv_rows_per_src)
        recv0 = np.concatenate([[0], np.cumsum(self.recv_rows_per_src)])
        within = np.cumsum(m[:, me, :], 1) - m[:, me, :]  # [W, B]: bin b's run inside j's rows
        # output order over [own rows (through perm) | received rows]: per bin, the kept rows,
        # then the received ones by source rank
        n_local = self.pb.n_pairs
        seg, lens = [], []
        for b in range(B):
            if keep[b]:
                seg.append((int(bin0[b]), 1, 0))
                lens.append(int(keep[b]))
            for j in range(W):
                c = int(m[j, me, b])
                if c:
                    seg.append((int(n_local + recv0[j] + within[j, b]), 1, 1))
                    lens.append(c)
        self._order_seg = (seg, lens)
        assert np.array_equal(keep + m[:, me, :].sum(0), quota[me])
        self.bin_off = np.concatenate([[0], np.cumsum(quota[me])]).astype(np.int64)
        self.batch_shard_counts = shard_n
        self.shard_counts = shard_n[mine] if len(mine) else np.zeros((0, B), np.int64)
        self.send_idx = self._expand(self._send_seg)

    def _expand(self, segs):
        seg, lens = segs
        seg_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        arr = np.asarray(seg, np.int64).reshape(-1, 3)
        return self.ops.expand(self.perm, arr, seg_off, self.dev)

    # round 1: row metadata -----------------------------------------------------------------
    def pack_meta(self):
        meta = self.ops.meta_pack(self.pb, self.send_idx)
        return meta, [4 * x for x in self.send_rows_per_dst], [4 * x for x in self.recv_rows_per_src]

    def unpack_meta(self, rmeta):
        ntok, len_a, is_rn, nmask = self.ops.meta_unpack(rmeta)
        self.rt = PairBatch(None, self.ops.scan(ntok), len_a, is_rn)
        if self.masking:
            self.rt.pos_off = self.ops.scan(nmask)

    # round 2: ragged columns ---------------------------------------------------------------
    def _ragged(self, data, data_off, recv_off):
        r = self.send_idx
        off = self.ops.ragged_offsets(data_off, self.pb.n_pairs, None, r)
        cut = np.concatenate([[0], np.cumsum(self.send_rows_per_dst)])
        rcut = np.concatenate([[0], np.cumsum(self.recv_rows_per_src)])
        sb = _host_at(self.ops, off, cut)
        rb = _host_at(self.ops, recv_off, rcut)
        buf = self.ops.gather(data, data_off, self.pb.n_pairs, None, None, r, off, int(sb[-1]))
        ss, rs = np.diff(sb).tolist(), np.diff(rb).tolist()
        if buf.element_size() == 2:  # RCCL has no 16-bit integer type: move the bytes
            b8 = buf.view(torch.uint8) if buf.numel() else torch.zeros(0, dtype=torch.uint8,
                                                                       device=buf.device)
            return b8, [2 * x for x in ss], [2 * x for x in rs]
        return buf, ss, rs

    def pack_data(self):
        out = [self._ragged(self.pb.tokens, self.pb.tok_off, self.rt.tok_off)]
        if self.masking:
            out.append(self._ragged(self.pb.pos, self.pb.pos_off, self.rt.pos_off))
            out.append(self._ragged(self.pb.labels, self.pb.pos_off, self.rt.pos_off))
        return out

    # regroup -------------------------------------------------------------------------------
    def finish(self, recvs):
        order = self._expand(self._order_seg)
        kw = dict(bin_off=self.bin_off, shards=self.shards, shard_counts=self.shard_counts,
                  moved_rows=self.n_recv, all_shard_counts=self.batch_shard_counts)
        if self.n_recv == 0:
            # nothing arrived: a row order over the rank's own table, no copy
            if self.n_send == 0:
                n_tokens = int(self.pb.tokens.numel())
            else:
                n_tokens = int(_host_at(self.ops, self.ops.ragged_offsets(
                    self.pb.tok_off, self.pb.n_pairs, None, order), [order.numel()])[0])
            return BalancedBins(self.pb, order, n_tokens=n_tokens, **kw)
        rt = self.rt
        rt.tokens = recvs[0] if recvs[0].dtype == self.pb.tokens.dtype else recvs[0].view(
            self.pb.tokens.dtype)
        if self.masking:
            rt.pos = recvs[1].view(self.pb.pos.dtype) if recvs[1].numel() else torch.zeros(
                0, dtype=self.pb.pos.dtype, device=self.dev)
            rt.labels = recvs[2].view(self.pb.labels.dtype)
        t = _gather_table(self.ops, self.pb, rt, order)
        return BalancedBins(t, None, n_tokens=int(t.tokens.numel()), **kw)


# ---- drivers ---------------------------------------------------------------------------------
def _a2a(payload, group):
    send, send_splits, recv_splits = payload
    dev = send.device
    if send.is_cuda and _host_staged(group):
        send = send.cpu()
    recv = _alloc(sum(recv_splits), send.dtype, send.device)
    dist.all_to_all_single(recv, send, [int(x) for x in recv_splits],
                           [int(x) for x in send_splits], group=group)
    return recv.to(dev)


class StreamBalancer:
    """The balance of a stream of batches over every rank of `group` into `num_shards` (default:
    world size) per-bin shards. Call `step(pb)` once per batch on every rank, in the same order
    (a rank without rows passes an empty PairBatch); `all_shard_counts` is the layout so far
    (every shard N or N+1 rows per bin after every step)."""

    def __init__(self, ctx, bin_size, nbins, num_shards=None, group=None, ops=None,
                 collective=None):
        # collective: None = the exchange runs when the group has more than one rank; True forces
        # it at world size 1 too (tests/test_balance_rccl_gpu.py: the RCCL branch on one GPU)
        self.multi = dist.is_initialized() and (dist.get_world_size(group) > 1 or bool(collective))
        self.W = dist.get_world_size(group) if self.multi else 1
        self.me = dist.get_rank(group) if self.multi else 0
        self.S = self.W if num_shards is None else int(num_shards)
        self.bin_size, self.nbins, self.group = bin_size, nbins, group
        self.ops = ops or HipOps(ctx)
        self.prior = np.zeros(nbins, np.int64)
        self.all_shard_counts = np.zeros((self.S, nbins), np.int64)

    def step(self, pb, timings=None):
        def mark(name):
            if timings is not None:
                if pb.tok_off.is_cuda:
                    torch.cuda.synchronize()
                timings[name] = time.perf_counter()
        mark('start')
        rb = RankBalance(self.ops, pb, self.bin_size, self.nbins, self.me, self.W, self.S)
        mark('bin')
        counts = gather_counts(rb.local_counts, self.group, collective=self.multi)
        rb.set_plan(counts, self.prior)
        mark('plan')
        if self.multi:
            rb.unpack_meta(_a2a(rb.pack_meta(), self.group))
            recvs = [_a2a(p, self.group) for p in rb.pack_data()]
        else:
            recvs = []
        mark('exchange')
        out = rb.finish(recvs)
        mark('regroup')
        self.prior += counts.sum(0)
        self.all_shard_counts += rb.batch_shard_counts
        return out


def balance(ctx, pb, bin_size, nbins, group=None, timings=None, num_shards=None, ops=None):
    """Balance one batch `pb` of every rank of `group` (a one-step StreamBalancer)."""
    return StreamBalancer(ctx, bin_size, nbins, num_shards, group, ops).step(pb, timings)


def _local_a2a(payloads, k):
    """In-process all-to-all: what rank k receives from payloads[j] = (send, send_splits, _)."""
    pieces = []
    for send, ss, _ in payloads:
        o = int(sum(ss[:k]))
        pieces.append(send[o:o + int(ss[k])])
    return torch.cat(pieces) if pieces else None


def stream_virtual(ops, batches, bin_size, nbins, num_shards=None):
    """The same balance over W virtual ranks held by one process: batches[t][r] = rank r's table
    of batch t. Returns outs[t][r] (BalancedBins) — the plan, pack and regroup of StreamBalancer,
    with the exchange done by slicing."""
    W = len(batches[0])
    S = W if num_shards is None else int(num_shards)
    prior = np.zeros(nbins, np.int64)
    outs = []
    for pbs in batches:
        rbs = [RankBalance(ops, pb, bin_size, nbins, r, W, S) for r, pb in enumerate(pbs)]
        counts = np.stack([rb.local_counts.cpu().numpy() for rb in rbs])
        for rb in rbs:
            rb.set_plan(counts, prior)
        metas = [rb.pack_meta() for rb in rbs]
        for k, rb in enumerate(rbs):
            rb.unpack_meta(_local_a2a(metas, k))
        datas = [rb.pack_data() for rb in rbs]
        outs.append([rb.finish([_local_a2a([d[c] for d in datas], k)
                                for c in range(len(datas[k]))]) for k, rb in enumerate(rbs)])
        prior += counts.sum(0)
    return outs


def balance_virtual(ops, pbs, bin_size, nbins, num_shards=None):
    """One batch over W virtual ranks (pbs[r] = rank r's table)."""
    return stream_virtual(ops, [pbs], bin_size, nbins, num_shards)[0]
