"""HBM-resident load balance across GPUs (configs C3/C4).

The reference balances shards through the filesystem (lddl/dask/load_balance.py:41-369: MPI
Allreduce of per-file counts, then read/concat/rewrite of parquet files). When the samples are
already in HBM on every GPU, the same contract — per bin, every shard ends with N or N+1
samples — is met with two collectives over RCCL/xGMI and no file traffic:

  1. every rank orders its samples by bin (stable; `lddl_bin_partitions` over one segment) and
     all-gathers its per-bin counts (int64[world, nbins]);
  2. all ranks compute the same plan: bin b's samples in rank-major order are cut into world
     contiguous ranges of base or base+1 samples (the first total % world ranks get +1), so
     only the imbalance moves;
  3. one all-to-all-v per column (row metadata, token ids, masked positions, labels) moves the
     rows; the receiver regroups them bin-major (global order preserved within a bin).

Rows are packed for the exchange by the HIP gather kernel `lddl_gather_ragged`.
"""
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from ._native import lib, check
from .context import _ptr, _stream


def plan_exchange(counts):
    """counts int64[W, B] (rank j's samples in bin b) -> (target [W, B], send [W, W, B],
    first [W, W, B]): rank j sends send[j, k, b] of its bin-b rows, starting at its local bin-b
    row first[j, k, b], to rank k; rank k then holds target[k, b] bin-b samples."""
    counts = np.asarray(counts, np.int64)
    W, B = counts.shape
    total = counts.sum(0)
    base, rem = total // W, total % W
    target = base[None, :] + (np.arange(W)[:, None] < rem[None, :]).astype(np.int64)
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


def _scan(x):
    out = torch.empty(x.numel() + 1, dtype=torch.int64, device=x.device)
    check(lib.lddl_scan_i64(_stream(), _ptr(x), x.numel(), _ptr(out)))
    return out


def _gather(src, src_off, rows, dst_off, n_elems):
    dst = torch.empty(max(int(n_elems), 1), dtype=src.dtype, device=src.device)[:int(n_elems)]
    check(lib.lddl_gather_ragged(_stream(), _ptr(src), _ptr(src_off), src.element_size(),
                                 _ptr(rows), rows.numel(), _ptr(dst_off), _ptr(dst)))
    return dst


@dataclass
class BalancedBins:
    """Per-rank result: the sample table in bin-major order and the row range of every bin."""
    tokens: torch.Tensor
    tok_off: torch.Tensor
    len_a: torch.Tensor
    is_random_next: torch.Tensor
    bin_off: np.ndarray          # int64[nbins + 1]
    pos: torch.Tensor = None
    labels: torch.Tensor = None
    pos_off: torch.Tensor = None

    @property
    def n_rows(self):
        return self.len_a.numel()


def _a2a(send, send_splits, recv_splits, group):
    recv = torch.empty(int(sum(recv_splits)), dtype=send.dtype, device=send.device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_to_all_single(recv, send, [int(x) for x in recv_splits],
                               [int(x) for x in send_splits], group=group)
    else:
        recv.copy_(send)
    return recv


def balance(ctx, pb, bin_size, nbins, group=None, timings=None):
    """Balance the PairBatch `pb` of every rank into per-bin shards of N or N+1 samples.
    timings: optional dict, filled with synchronised per-phase wall times (diagnostics)."""
    import time
    dev = pb.tok_off.device

    def mark(name):
        if timings is not None:
            torch.cuda.synchronize()
            timings[name] = time.perf_counter()
    mark('start')
    W = dist.get_world_size(group) if dist.is_initialized() else 1
    me = dist.get_rank(group) if dist.is_initialized() else 0
    from .output import bin_stable
    ntok = pb.tok_off[1:] - pb.tok_off[:-1]
    perm, _, cnt = bin_stable(ctx, (ntok + 3).to(torch.int32), bin_size, nbins)
    mark('bin')
    counts = gather_counts(cnt.reshape(-1), group)
    target, send, first = plan_exchange(counts)
    mark('counts')
    bin0 = np.concatenate([[0], np.cumsum(counts[me])])
    # rows to send, dst-major then bin (slices of the local bin order)
    pieces, send_rows_per_dst = [], []
    for k in range(W):
        n = 0
        for b in range(nbins):
            c = int(send[me, k, b])
            if c:
                a = int(bin0[b] + first[me, k, b])
                pieces.append(perm[a:a + c])
                n += c
        send_rows_per_dst.append(n)
    rows = torch.cat(pieces) if pieces else torch.zeros(0, dtype=torch.int64, device=dev)
    recv_rows_per_src = [int(send[j, me].sum()) for j in range(W)]
    masking = pb.pos is not None
    nmask = (pb.pos_off[1:] - pb.pos_off[:-1]) if masking else None
    # row metadata: (tokens, len_a, is_random_next, masked positions)
    meta = torch.stack([ntok.index_select(0, rows), pb.len_a.index_select(0, rows).long(),
                        pb.is_random_next.index_select(0, rows).long(),
                        nmask.index_select(0, rows) if masking else torch.zeros_like(rows)], 1)
    rmeta = _a2a(meta.reshape(-1), [4 * x for x in send_rows_per_dst],
                 [4 * x for x in recv_rows_per_src], group).view(-1, 4)

    def split_sums(v, per):
        c = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
        s = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), torch.cumsum(v, 0)])
        return (s[c[1:]] - s[c[:-1]]).cpu().tolist() if len(per) else []

    def exchange(data, data_off, sizes_recv_row):
        off = _scan(data_off[1:].index_select(0, rows) - data_off[:-1].index_select(0, rows))
        buf = _gather(data, data_off, rows, off, int(off[-1].item()))
        ss = split_sums(off[1:] - off[:-1], send_rows_per_dst) if rows.numel() else [0] * W
        rs = split_sums(sizes_recv_row, recv_rows_per_src)
        if buf.element_size() == 2:  # RCCL has no 16-bit integer type: move the bytes
            r = _a2a(buf.view(torch.uint8), [2 * x for x in ss], [2 * x for x in rs], group)
            return r.view(buf.dtype)
        return _a2a(buf, ss, rs, group)

    mark('meta')
    rtok = exchange(pb.tokens, pb.tok_off, rmeta[:, 0])
    rtok_off = _scan(rmeta[:, 0].contiguous())
    if masking:
        rpos = exchange(pb.pos, pb.pos_off, rmeta[:, 3])
        rlab = exchange(pb.labels, pb.pos_off, rmeta[:, 3])
        rpos_off = _scan(rmeta[:, 3].contiguous())
    mark('exchange')
    # regroup received rows bin-major (src order inside a bin = global order)
    src0 = np.concatenate([[0], np.cumsum(recv_rows_per_src)])
    order, bin_off = [], [0]
    for b in range(nbins):
        for j in range(W):
            c = int(send[j, me, b])
            if c:
                a = int(src0[j] + send[j, me, :b].sum())
                order.append(torch.arange(a, a + c, dtype=torch.int64, device=dev))
        bin_off.append(bin_off[-1] + int(target[me, b]))
    order = torch.cat(order) if order else torch.zeros(0, dtype=torch.int64, device=dev)
    ntok_o = rmeta[:, 0].index_select(0, order).contiguous()
    tok_off = _scan(ntok_o)
    out = BalancedBins(_gather(rtok, rtok_off, order, tok_off, int(tok_off[-1].item())), tok_off,
                       rmeta[:, 1].index_select(0, order).to(torch.int32),
                       rmeta[:, 2].index_select(0, order).to(torch.uint8),
                       np.asarray(bin_off, np.int64))
    if masking:
        nm = rmeta[:, 3].index_select(0, order).contiguous()
        pos_off = _scan(nm)
        out.pos = _gather(rpos, rpos_off, order, pos_off, int(pos_off[-1].item()))
        out.labels = _gather(rlab, rpos_off, order, pos_off, int(pos_off[-1].item()))
        out.pos_off = pos_off
    mark('regroup')
    return out
