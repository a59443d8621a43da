"""HBM-resident load balance across GPUs (configs C3/C4).

The reference balances shards through the filesystem (lddl/dask/load_balance.py:41-369: MPI
Allreduce of per-file counts, then read/concat/rewrite of parquet files) so that, per bin, every
shard ends with N or N+1 samples (`Progress` targets, load_balance.py:161-169). When the samples
are already in HBM on every GPU, the same contract is met with two collectives over RCCL/xGMI and
no file traffic:

  1. every rank orders its samples by bin (stable; `lddl_bin_stable`) and all-gathers its per-bin
     counts (int64[world, nbins]) — the global bin-count all-gather of the north star;
  2. all ranks compute the same plan (`plan_exchange`): bin b's samples in rank-major order are
     cut into `num_shards` contiguous ranges of base or base+1 samples (the first total % S
     shards get +1); shard s belongs to rank s * world // S, so each rank owns a contiguous run
     of every bin and only the imbalance crosses ranks;
  3. an all-to-all-v of the row metadata, then one per ragged column (token ids, masked
     positions as bytes, labels), carries ONLY rows that change rank: rows that stay are never
     packed or sent. The receiver's bin-major order interleaves its own rows with the received
     ones in global order.

Output (`BalancedBins`): when a rank received nothing (always at world size 1) the result is a
row order over the rank's own table — no bytes move; otherwise the rank's rows are materialised
once into a contiguous bin-major table (two ragged gathers: own rows, received rows).

The algorithm is split into per-rank phases (`RankBalance`) so that the collective driver
(`balance`, torch.distributed: RCCL on GPUs, gloo on CPUs) and the in-process driver over
virtual ranks (`balance_virtual`, used by the tests to run W ranks on one GPU) execute the same
plan, pack and regroup code. Data movement goes through `HipOps` (HIP kernels through the C ABI);
there is no other implementation in the product.
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


def shard_targets(counts, num_shards):
    """int64[S, B]: samples of bin b in shard s (N or N+1; the first total % S shards get +1,
    the reference's Progress targets, load_balance.py:161-169)."""
    total = np.asarray(counts, np.int64).sum(0)
    base, rem = total // num_shards, total % num_shards
    return base[None, :] + (np.arange(num_shards)[:, None] < rem[None, :]).astype(np.int64)


def plan_exchange(counts, num_shards=None):
    """counts int64[W, B] (rank j's samples in bin b) -> (target [W, B], send [W, W, B],
    first [W, W, B]): rank j sends send[j, k, b] of its bin-b rows, starting at its local bin-b
    row first[j, k, b], to rank k; rank k then holds target[k, b] bin-b samples (the sum of its
    shards' targets). send[j, j, b] are the rows that stay on rank j."""
    counts = np.asarray(counts, np.int64)
    W, B = counts.shape
    S = W if num_shards is None else int(num_shards)
    st = shard_targets(counts, S)
    target = np.zeros((W, B), np.int64)
    np.add.at(target, shard_owner(S, W), st)
    src0 = np.cumsum(counts, 0) - counts
    dst0 = np.cumsum(target, 0) - target
    lo = np.maximum(src0[:, None, :], dst0[None, :, :])
    hi = np.minimum((src0 + counts)[:, None, :], (dst0 + target)[None, :, :])
    send = np.maximum(hi - lo, 0)
    first = np.where(send > 0, lo - src0[:, None, :], 0)
    return target, send, first


def gather_counts(local_counts, group=None):
    """all_gather of the per-bin counts (RCCL when the tensor is on the GPU)."""
    W = dist.get_world_size(group) if dist.is_initialized() else 1
    if W == 1:
        return local_counts.reshape(1, -1).cpu().numpy()
    out = [torch.empty_like(local_counts) for _ in range(W)]
    dist.all_gather(out, local_counts, group=group)
    return torch.stack(out).cpu().numpy()


# ---- data-movement primitives ----------------------------------------------------------------
class HipOps:
    """The balance's device primitives: HIP kernels of liblddl_amd.so on torch's current stream."""

    def __init__(self, ctx):
        self.ctx = ctx

    def bin_stable(self, num_tokens, bin_size, nbins):
        """(perm int64[n], counts int64[nbins]): stable regroup of the rows by
        bin_id = min((num_tokens - 1) // bin_size, nbins - 1) (binning.py:63-93)."""
        from .output import bin_stable
        perm, _, cnt = bin_stable(self.ctx, num_tokens, bin_size, nbins)
        return perm, cnt

    def scan(self, x):
        out = torch.empty(x.numel() + 1, dtype=torch.int64, device=x.device)
        check(lib.lddl_scan_i64(_stream(), _ptr(x), x.numel(), _ptr(out)))
        return out

    def gather_into(self, src, src_off, rows, dst_off, dst):
        """dst[dst_off[i] ...] = src[src_off[rows[i]] .. src_off[rows[i] + 1])."""
        if rows.numel() == 0:
            return dst
        check(lib.lddl_gather_ragged(_stream(), _ptr(src), _ptr(src_off), src.element_size(),
                                     _ptr(rows), rows.numel(), _ptr(dst_off), _ptr(dst)))
        return dst


def _alloc(n, dtype, dev):
    return torch.empty(max(int(n), 1), dtype=dtype, device=dev)[:int(n)]


def _expand(vec, starts, lens, dev):
    """Concatenation of the slices vec[starts[i] : starts[i] + lens[i]] (one device gather)."""
    total = int(sum(lens))
    if total == 0:
        return torch.zeros(0, dtype=vec.dtype, device=dev)
    st = torch.tensor(starts, dtype=torch.int64, device=dev)
    ln = torch.tensor(lens, dtype=torch.int64, device=dev)
    first = torch.cumsum(ln, 0) - ln
    idx = torch.repeat_interleave(st - first, ln, output_size=total) + torch.arange(
        total, dtype=torch.int64, device=dev)
    return vec.index_select(0, idx)


def _group_sums(v, sizes):
    """Per-group sums of consecutive runs of `v` (host list); sizes = run lengths."""
    if not len(sizes):
        return []
    c = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    if v.numel() == 0:
        return [0] * len(sizes)
    s = torch.cat([torch.zeros(1, dtype=torch.int64, device=v.device), torch.cumsum(v, 0)])
    return (s[torch.from_numpy(c[1:]).to(v.device)] -
            s[torch.from_numpy(c[:-1]).to(v.device)]).cpu().tolist()


# ---- result ----------------------------------------------------------------------------------
@dataclass
class BalancedBins:
    """One rank's share after the balance, bin-major.

    Output row i is row `rows[i]` of `table` (rows None = identity, i.e. the table itself is
    bin-major). Bin b is output rows [bin_off[b], bin_off[b+1]); inside a bin the rank's shards
    follow each other: shard shards[m] holds shard_counts[m, b] of them."""
    table: PairBatch
    rows: torch.Tensor
    bin_off: np.ndarray
    shards: list = field(default_factory=list)
    shard_counts: np.ndarray = None
    n_tokens: int = 0              # sum of len(A) + len(B) over the output rows
    moved_rows: int = 0            # rows received from other ranks
    all_shard_counts: np.ndarray = None  # int64[S, B]: every shard's samples per bin (all ranks)

    @property
    def n_rows(self):
        return int(self.bin_off[-1])

    @property
    def tokens(self):  # materialised token ids in output order (tests / diagnostics)
        return self.materialize().table.tokens

    def shard_rows(self, m):
        """Output rows of this rank's m-th shard, bin after bin (host int64), and their bins."""
        idx, bins = [], []
        for b in range(len(self.bin_off) - 1):
            a = int(self.bin_off[b] + self.shard_counts[:m, b].sum())
            c = int(self.shard_counts[m, b])
            idx.append(np.arange(a, a + c, dtype=np.int64))
            bins.append(np.full(c, b, np.int64))
        return np.concatenate(idx), np.concatenate(bins)

    def bin_ids(self):
        """int64[n_rows] bin id of every output row (device)."""
        dev = self.table.tok_off.device
        nb = len(self.bin_off) - 1
        return torch.repeat_interleave(torch.arange(nb, dtype=torch.int64, device=dev),
                                       torch.from_numpy(np.diff(self.bin_off)).to(dev),
                                       output_size=self.n_rows)

    def materialize(self, ops=None):
        """The contiguous bin-major table (copies only if `rows` is not the identity)."""
        if self.rows is None:
            return self
        ops = ops or HipOps(None)
        t = _gather_table(ops, self.table, self.rows)
        return BalancedBins(t, None, self.bin_off, self.shards, self.shard_counts, self.n_tokens,
                            self.moved_rows, self.all_shard_counts)


def _gather_table(ops, pb, rows):
    """Rows `rows` of PairBatch pb as a new contiguous PairBatch."""
    dev = pb.tok_off.device
    ntok = (pb.tok_off[1:] - pb.tok_off[:-1]).index_select(0, rows)
    tok_off = ops.scan(ntok.contiguous())
    n_tok = int(tok_off[-1].item())
    tokens = ops.gather_into(pb.tokens, pb.tok_off, rows, tok_off, _alloc(n_tok, pb.tokens.dtype, dev))
    out = PairBatch(tokens, tok_off, pb.len_a.index_select(0, rows),
                    pb.is_random_next.index_select(0, rows))
    if pb.pos is not None:
        nm = (pb.pos_off[1:] - pb.pos_off[:-1]).index_select(0, rows)
        pos_off = ops.scan(nm.contiguous())
        n_m = int(pos_off[-1].item())
        out.pos = ops.gather_into(pb.pos, pb.pos_off, rows, pos_off, _alloc(n_m, pb.pos.dtype, dev))
        out.labels = ops.gather_into(pb.labels, pb.pos_off, rows, pos_off,
                                     _alloc(n_m, pb.labels.dtype, dev))
        out.pos_off = pos_off
        out.n_masked = n_m
    return out


# ---- per-rank phases -------------------------------------------------------------------------
class RankBalance:
    """One rank's part of the balance: bin (local), plan (replicated), pack / unpack around the
    two exchange rounds (row metadata, then the ragged columns), regroup."""

    def __init__(self, ops, pb, bin_size, nbins, rank, world, num_shards=None):
        self.ops, self.pb, self.nbins = ops, pb, nbins
        self.me, self.W = rank, world
        self.S = world if num_shards is None else int(num_shards)
        self.dev = pb.tok_off.device
        self.ntok = pb.tok_off[1:] - pb.tok_off[:-1]
        self.masking = pb.pos is not None
        self.nmask = (pb.pos_off[1:] - pb.pos_off[:-1]) if self.masking else None
        self.perm, self.local_counts = ops.bin_stable((self.ntok + 3).to(torch.int32), bin_size,
                                                      nbins)

    # plan ----------------------------------------------------------------------------------
    def set_plan(self, counts):
        W, me, B = self.W, self.me, self.nbins
        self.counts = np.asarray(counts, np.int64)
        self.target, self.send, self.first = plan_exchange(self.counts, self.S)
        bin0 = np.concatenate([[0], np.cumsum(self.counts[me])])
        starts, lens = [], []
        self.send_rows_per_dst = [0] * W
        for k in range(W):  # rows leaving this rank, destination-major then bin
            if k == me:
                continue
            for b in range(B):
                c = int(self.send[me, k, b])
                if c:
                    starts.append(int(bin0[b] + self.first[me, k, b]))
                    lens.append(c)
                    self.send_rows_per_dst[k] += c
        self.send_idx = _expand(self.perm, starts, lens, self.dev)
        self.recv_rows_per_src = [0 if j == me else int(self.send[j, me].sum()) for j in range(W)]
        self.n_recv = sum(self.recv_rows_per_src)
        # output order over the virtual source [local rows (via perm) | received rows]
        n_local = self.pb.n_pairs
        src0 = np.concatenate([[0], np.cumsum(self.recv_rows_per_src)])
        starts, lens = [], []
        for b in range(B):
            for j in range(W):
                c = int(self.send[j, me, b])
                if not c:
                    continue
                if j == me:
                    starts.append(int(bin0[b] + self.first[me, me, b]))
                else:
                    starts.append(int(n_local + src0[j] + self.send[j, me, :b].sum()))
                lens.append(c)
        self._order_src = (starts, lens)
        self.bin_off = np.concatenate([[0], np.cumsum(self.target[me])]).astype(np.int64)
        owner = shard_owner(self.S, W)
        self.shards = [int(s) for s in np.nonzero(owner == me)[0]]
        self.all_shard_counts = shard_targets(self.counts, self.S)
        self.shard_counts = self.all_shard_counts[self.shards]

    # round 1: row metadata -----------------------------------------------------------------
    def pack_meta(self):
        r = self.send_idx
        cols = [self.ntok.index_select(0, r), self.pb.len_a.index_select(0, r).long(),
                self.pb.is_random_next.index_select(0, r).long(),
                self.nmask.index_select(0, r) if self.masking else torch.zeros_like(r)]
        meta = torch.stack(cols, 1).reshape(-1) if r.numel() else torch.zeros(
            0, dtype=torch.int64, device=self.dev)
        return meta, [4 * x for x in self.send_rows_per_dst], [4 * x for x in self.recv_rows_per_src]

    def unpack_meta(self, rmeta):
        self.rmeta = rmeta.view(-1, 4)

    # round 2: ragged columns ---------------------------------------------------------------
    def _ragged(self, data, data_off, sizes, recv_sizes):
        r = self.send_idx
        off = self.ops.scan(sizes.index_select(0, r).contiguous())
        n = int(off[-1].item()) if r.numel() else 0
        buf = self.ops.gather_into(data, data_off, r, off, _alloc(n, data.dtype, self.dev))
        ss = _group_sums(sizes.index_select(0, r), self.send_rows_per_dst)
        rs = _group_sums(recv_sizes, self.recv_rows_per_src)
        if buf.element_size() == 2:  # RCCL has no 16-bit integer type: move the bytes
            return buf.view(torch.uint8), [2 * x for x in ss], [2 * x for x in rs]
        return buf, ss, rs

    def pack_data(self):
        out = [self._ragged(self.pb.tokens, self.pb.tok_off, self.ntok, self.rmeta[:, 0])]
        if self.masking:
            out.append(self._ragged(self.pb.pos, self.pb.pos_off, self.nmask, self.rmeta[:, 3]))
            out.append(self._ragged(self.pb.labels, self.pb.pos_off, self.nmask, self.rmeta[:, 3]))
        return out

    # regroup -------------------------------------------------------------------------------
    def finish(self, recvs):
        n_local = self.pb.n_pairs
        if self.n_recv == 0 and sum(self.send_rows_per_dst) == 0:
            # every row stays (always at world size 1): the output is the local bin order itself
            return BalancedBins(self.pb, self.perm, self.bin_off, self.shards, self.shard_counts,
                                int(self.pb.tokens.numel()), 0, self.all_shard_counts)
        src = torch.cat([self.perm, torch.arange(n_local, n_local + self.n_recv, dtype=torch.int64,
                                                  device=self.dev)])
        order = _expand(src, *self._order_src, self.dev)
        ntok_v = torch.cat([self.ntok, self.rmeta[:, 0]])
        n_tokens = int(ntok_v.index_select(0, order).sum().item()) if order.numel() else 0
        bb = BalancedBins(self.pb, order, self.bin_off, self.shards, self.shard_counts, n_tokens,
                          self.n_recv, self.all_shard_counts)
        if self.n_recv == 0:
            return bb  # nothing arrived: a row order over the rank's own table, no copy
        # received rows as a PairBatch, then one materialisation of the two sources
        rtok = recvs[0]
        rt = PairBatch(rtok, self.ops.scan(self.rmeta[:, 0].contiguous()),
                       self.rmeta[:, 1].to(torch.int32), self.rmeta[:, 2].to(torch.uint8))
        if self.masking:
            rt.pos = recvs[1].view(self.pb.pos.dtype)
            rt.labels = recvs[2]
            rt.pos_off = self.ops.scan(self.rmeta[:, 3].contiguous())
        return BalancedBins(_gather_two(self.ops, self.pb, rt, order), None, self.bin_off,
                            self.shards, self.shard_counts, n_tokens, self.n_recv,
                            self.all_shard_counts)


def _gather_two(ops, pa, pr, order):
    """Rows `order` of the virtual concatenation [pa | pr] as one contiguous PairBatch: each
    output row is copied once, from whichever table holds it."""
    dev = pa.tok_off.device
    na = pa.n_pairs
    is_a = order < na
    ia = torch.nonzero(is_a).reshape(-1)
    ir = torch.nonzero(~is_a).reshape(-1)
    ra, rr = order.index_select(0, ia), order.index_select(0, ir) - na

    def per_row(xa, xr):
        return torch.cat([xa, xr]).index_select(0, order)

    ntok = per_row(pa.tok_off[1:] - pa.tok_off[:-1], pr.tok_off[1:] - pr.tok_off[:-1])
    tok_off = ops.scan(ntok.contiguous())
    tokens = _alloc(int(tok_off[-1].item()), pa.tokens.dtype, dev)
    ops.gather_into(pa.tokens, pa.tok_off, ra, tok_off.index_select(0, ia), tokens)
    ops.gather_into(pr.tokens, pr.tok_off, rr, tok_off.index_select(0, ir), tokens)
    out = PairBatch(tokens, tok_off, per_row(pa.len_a, pr.len_a),
                    per_row(pa.is_random_next, pr.is_random_next))
    if pa.pos is not None:
        nm = per_row(pa.pos_off[1:] - pa.pos_off[:-1], pr.pos_off[1:] - pr.pos_off[:-1])
        pos_off = ops.scan(nm.contiguous())
        n_m = int(pos_off[-1].item())
        pos = _alloc(n_m, pa.pos.dtype, dev)
        lab = _alloc(n_m, pa.labels.dtype, dev)
        da, dr = pos_off.index_select(0, ia), pos_off.index_select(0, ir)
        ops.gather_into(pa.pos, pa.pos_off, ra, da, pos)
        ops.gather_into(pr.pos, pr.pos_off, rr, dr, pos)
        ops.gather_into(pa.labels, pa.pos_off, ra, da, lab)
        ops.gather_into(pr.labels, pr.pos_off, rr, dr, lab)
        out.pos, out.labels, out.pos_off, out.n_masked = pos, lab, pos_off, n_m
    return out


# ---- drivers ---------------------------------------------------------------------------------
def _a2a(payload, group):
    send, send_splits, recv_splits = payload
    recv = _alloc(sum(recv_splits), send.dtype, send.device)
    dist.all_to_all_single(recv, send, [int(x) for x in recv_splits],
                           [int(x) for x in send_splits], group=group)
    return recv


def balance(ctx, pb, bin_size, nbins, group=None, timings=None, num_shards=None, ops=None):
    """Balance the PairBatch `pb` of every rank of `group` into `num_shards` (default: world
    size) per-bin shards of N or N+1 samples; collective over torch.distributed (RCCL for cuda
    tensors). timings: optional dict filled with synchronised per-phase wall times."""
    def mark(name):
        if timings is not None:
            if pb.tok_off.is_cuda:
                torch.cuda.synchronize()
            timings[name] = time.perf_counter()
    mark('start')
    multi = dist.is_initialized() and dist.get_world_size(group) > 1
    W = dist.get_world_size(group) if multi else 1
    me = dist.get_rank(group) if multi else 0
    rb = RankBalance(ops or HipOps(ctx), pb, bin_size, nbins, me, W, num_shards)
    mark('bin')
    rb.set_plan(gather_counts(rb.local_counts, group))
    mark('counts')
    if multi:
        rb.unpack_meta(_a2a(rb.pack_meta(), group))
        recvs = [_a2a(p, group) for p in rb.pack_data()]
    else:
        rb.unpack_meta(torch.zeros(0, dtype=torch.int64, device=rb.dev))
        recvs = []
    mark('exchange')
    out = rb.finish(recvs)
    mark('regroup')
    return out


def _local_a2a(payloads, k):
    """In-process all-to-all: what rank k receives from payloads[j] = (send, send_splits, _)."""
    pieces = []
    for send, ss, _ in payloads:
        o = int(sum(ss[:k]))
        pieces.append(send[o:o + int(ss[k])])
    return torch.cat(pieces) if pieces else None


def balance_virtual(ops, pbs, bin_size, nbins, num_shards=None):
    """The same balance over W virtual ranks held by one process (pbs[r] = rank r's table):
    the plan, pack and regroup of `balance`, with the exchange done by slicing."""
    W = len(pbs)
    rbs = [RankBalance(ops, pb, bin_size, nbins, r, W, num_shards) for r, pb in enumerate(pbs)]
    counts = np.stack([rb.local_counts.cpu().numpy() for rb in rbs])
    for rb in rbs:
        rb.set_plan(counts)
    metas = [rb.pack_meta() for rb in rbs]
    for k, rb in enumerate(rbs):
        rb.unpack_meta(_local_a2a(metas, k))
    datas = [rb.pack_data() for rb in rbs]
    return [rb.finish([_local_a2a([d[c] for d in datas], k) for c in range(len(datas[k]))])
            for k, rb in enumerate(rbs)]
