"""Test helpers for lddl_amd/balance.py: CPU data-movement primitives (so the product's plan /
pack / regroup code runs under gloo without a GPU) and the invariant checker.

TorchCpuOps is test infrastructure: the product always uses balance.HipOps (HIP kernels)."""
import numpy as np
import torch

from lddl_amd.balance import shard_owner, shard_targets
from lddl_amd.pairs import PairBatch


def _np(t):
    return None if t is None else t.numpy()


class TorchCpuOps:
    """numpy restatement of HipOps on CPU tensors (two-source row addressing: row r < n_a is
    row r of the first table, else row r - n_a of the second)."""

    def bin_stable(self, pb, bin_size, nbins):
        nt = np.diff(pb.tok_off.numpy()) + 3
        b = np.minimum((nt - 1) // bin_size, nbins - 1)
        return (torch.from_numpy(np.argsort(b, kind='stable').astype(np.int64)),
                torch.from_numpy(np.bincount(b, minlength=nbins).astype(np.int64)))

    def scan(self, x):
        return torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(x.long(), 0)])

    def expand(self, src, seg, seg_off, dev):
        out = [np.zeros(0, np.int64)]
        for (st, sd, direct), a, z in zip(np.asarray(seg).reshape(-1, 3), seg_off[:-1], seg_off[1:]):
            v = st + np.arange(z - a, dtype=np.int64) * sd
            out.append(v if direct else src.numpy()[v])
        return torch.from_numpy(np.concatenate(out))

    @staticmethod
    def _pick(a, n_a, b, r):
        out = np.empty(len(r), a.dtype)
        m = r < n_a
        out[m] = a[r[m]]
        if (~m).any():
            out[~m] = b[r[~m] - n_a]
        return out

    def take(self, a, n_a, b, rows):
        return torch.from_numpy(self._pick(a.numpy(), n_a, _np(b), rows.numpy()))

    def _spans(self, off_a, n_a, off_b, rows):
        r = rows.numpy()
        oa, ob = off_a.numpy(), _np(off_b)
        lo = self._pick(oa[:-1], n_a, None if ob is None else ob[:-1], r)
        hi = self._pick(oa[1:], n_a, None if ob is None else ob[1:], r)
        return r, lo, hi

    def ragged_offsets(self, off_a, n_a, off_b, rows):
        _, lo, hi = self._spans(off_a, n_a, off_b, rows)
        return torch.from_numpy(np.concatenate([[0], np.cumsum(hi - lo)]).astype(np.int64))

    def gather(self, a, off_a, n_a, b, off_b, rows, dst_off, total):
        r, lo, hi = self._spans(off_a, n_a, off_b, rows)
        A, B = a.numpy(), _np(b)
        parts = [(A if q < n_a else B)[x:y] for q, x, y in zip(r, lo, hi)]
        out = np.concatenate(parts) if parts else np.zeros(0, A.dtype)
        assert len(out) == total
        return torch.from_numpy(out.astype(A.dtype))

    def meta_pack(self, pb, rows):
        r = rows.numpy()
        to = pb.tok_off.numpy()
        po = pb.pos_off.numpy() if pb.pos_off is not None else None
        m = np.stack([to[r + 1] - to[r], pb.len_a.numpy()[r], pb.is_random_next.numpy()[r],
                      (po[r + 1] - po[r]) if po is not None else np.zeros(len(r), np.int64)], 1)
        return torch.from_numpy(m.astype(np.int32).reshape(-1))

    def meta_unpack(self, meta):
        m = meta.numpy().reshape(-1, 4)
        return (torch.from_numpy(m[:, 0].astype(np.int64)), torch.from_numpy(m[:, 1].copy()),
                torch.from_numpy(m[:, 2].astype(np.uint8)), torch.from_numpy(m[:, 3].astype(np.int64)))


def random_table(rng, n, seq, rank, masking=True, device='cpu', tag=0):
    """A PairBatch of n rows whose token ids encode (tag, rank, row, k) so moves are traceable."""
    ntok = rng.integers(2, seq - 2, n).astype(np.int64)
    tok_off = np.concatenate([[0], np.cumsum(ntok)]).astype(np.int64)
    tokens = np.concatenate([np.full(c, tag * 50_000_000 + rank * 1_000_000 + r * 100, np.int64) +
                             np.arange(c) for r, c in enumerate(ntok)] or [np.zeros(0, np.int64)]
                            ) % (1 << 31)
    len_a = np.array([rng.integers(1, c) for c in ntok], np.int32)
    is_rn = rng.integers(0, 2, n).astype(np.uint8)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
    pb = PairBatch(t(tokens.astype(np.int32)), t(tok_off), t(len_a), t(is_rn))
    if masking:
        nm = np.maximum(1, (ntok + 3) * 15 // 100)
        pos_off = np.concatenate([[0], np.cumsum(nm)]).astype(np.int64)
        pos = np.concatenate([np.arange(1, c + 1) for c in nm] or [np.zeros(0)]).astype(np.uint16)
        lab = np.concatenate([np.full(c, rank * 1000 + r) for r, c in enumerate(nm)] or [np.zeros(0)]).astype(
            np.int32)
        pb.pos, pb.labels, pb.pos_off = t(pos.view(np.int16)), t(lab), t(pos_off)
        pb.n_masked = int(pos_off[-1])
    return pb


def host_rows(h):
    """Per-row tuples of a to_host() dict (tokens, len_a, is_rn[, pos, labels])."""
    out = []
    for q in range(len(h['len_a'])):
        r = (tuple(h['tokens'][h['tok_off'][q]:h['tok_off'][q + 1]].tolist()), int(h['len_a'][q]),
             bool(h['is_random_next'][q]))
        if 'pos' in h:
            a, z = h['pos_off'][q], h['pos_off'][q + 1]
            r += (tuple(h['pos'][a:z].tolist()), tuple(h['labels'][a:z].tolist()))
        out.append(r)
    return out


def check_stream(inputs, outputs, bin_size, nbins, num_shards, moved=None):
    """inputs[t][r]: rank r's to_host() table of batch t; outputs[t][r]: (host dict of the
    materialised output table, bin_off, shards, shard_counts); moved[t][r] (optional): the rows
    rank r received. Checks the balance contract, restated by brute force:

      * after every batch, shard s holds n // S (+1 for the first n % S shards) rows of a bin that
        has seen n rows (the reference's Progress targets): N or N+1;
      * shard s belongs to rank s * W // S; a rank's quota of bin b is its shards' share of the
        batch; each rank keeps the first min(count, quota) of its bin-b rows (stable bin order),
        the surplus tails of all ranks, in rank order, form a pool that the ranks below quota
        take from in rank order;
      * a rank's bin-b output is [kept | taken], dealt in consecutive runs to its shards in
        ascending order; the rows moved are exactly the pool (the imbalance, nothing else).
    Returns the cumulative int64[S, B] shard counts."""
    W, S = len(inputs[0]), num_shards
    owner = shard_owner(S, W)
    prior = np.zeros(nbins, np.int64)
    cum = np.zeros((S, nbins), np.int64)
    for t in range(len(inputs)):
        per_rank = []  # [r][b]: rank r's rows of bin b in stable order
        for h in inputs[t]:
            nt = np.diff(h['tok_off']) + 3
            bins = np.minimum((nt - 1) // bin_size, nbins - 1)
            rows = host_rows(h)
            lst = [[] for _ in range(nbins)]
            for q in np.argsort(bins, kind='stable'):
                lst[bins[q]].append(rows[q])
            per_rank.append(lst)
        total = np.array([sum(len(per_rank[r][b]) for r in range(W)) for b in range(nbins)])
        after = shard_targets((prior + total)[None, :], S)
        shard_n = after - shard_targets(prior[None, :], S)
        prior += total
        expect = [[None] * nbins for _ in range(W)]
        n_moved = np.zeros(W, np.int64)
        for b in range(nbins):
            quota = [int(shard_n[owner == r, b].sum()) for r in range(W)]
            pool = [(r, x) for r in range(W) for x in per_rank[r][b][quota[r]:]]
            for r in range(W):
                kept = per_rank[r][b][:quota[r]]
                take, pool = pool[:quota[r] - len(kept)], pool[quota[r] - len(kept):]
                n_moved[r] += len(take)
                assert all(src != r for src, _ in take)
                expect[r][b] = kept + [x for _, x in take]
            assert not pool
        for k, (h, bin_off, shards, shard_counts) in enumerate(outputs[t]):
            assert list(shards) == [s for s in range(S) if owner[s] == k]
            rows = host_rows(h)
            assert len(rows) == bin_off[-1]
            for b in range(nbins):
                assert rows[bin_off[b]:bin_off[b + 1]] == expect[k][b], \
                    'batch {} rank {} bin {} differs from the balance contract'.format(t, k, b)
                for m, s in enumerate(shards):
                    assert shard_counts[m][b] == shard_n[s, b]
            if moved is not None:
                assert moved[t][k] == n_moved[k]
        cum += shard_n
        np.testing.assert_array_equal(cum, after)
    return cum
