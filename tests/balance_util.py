"""Test helpers for lddl_amd/balance.py: CPU data-movement primitives (so the product's plan /
pack / regroup code runs under gloo without a GPU) and the invariant checker.

TorchCpuOps is test infrastructure: the product always uses balance.HipOps (HIP kernels)."""
import numpy as np
import torch

from lddl_amd.balance import plan_exchange, shard_owner, shard_targets
from lddl_amd.pairs import PairBatch


class TorchCpuOps:
    def bin_stable(self, num_tokens, bin_size, nbins):
        b = torch.clamp((num_tokens.long() - 1) // bin_size, max=nbins - 1)
        perm = torch.from_numpy(np.argsort(b.numpy(), kind='stable').astype(np.int64))
        return perm, torch.bincount(b, minlength=nbins).long()

    def scan(self, x):
        return torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(x.long(), 0)])

    def gather_into(self, src, src_off, rows, dst_off, dst):
        so, do = src_off.tolist(), dst_off.tolist()
        for i, r in enumerate(rows.tolist()):
            n = so[r + 1] - so[r]
            dst[do[i]:do[i] + n] = src[so[r]:so[r + 1]]
        return dst


def random_table(rng, n, seq, rank, masking=True, device='cpu'):
    """A PairBatch of n rows whose token ids encode (rank, row, k) so that moves are traceable."""
    ntok = rng.integers(2, seq - 2, n).astype(np.int64)
    tok_off = np.concatenate([[0], np.cumsum(ntok)]).astype(np.int64)
    tokens = np.concatenate([np.full(c, rank * 1_000_000 + r * 100, np.int64) + np.arange(c)
                             for r, c in enumerate(ntok)] or [np.zeros(0, np.int64)]) % (1 << 31)
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


def check_balanced(inputs, outputs, bin_size, nbins, num_shards):
    """inputs[r]: rank r's to_host() table before; outputs[r]: (host dict of the materialised
    output table, bin_off, shards, shard_counts). Checks the north-star / reference invariants:
    per bin every shard holds N or N+1 samples, each rank's table is bin-major, and the
    concatenation over ranks of bin b equals the global stable bin order (rank-major input)."""
    W = len(inputs)
    counts = []
    glob = [[] for _ in range(nbins)]
    for h in inputs:
        nt = np.diff(h['tok_off']) + 3
        bins = np.minimum((nt - 1) // bin_size, nbins - 1)
        counts.append(np.bincount(bins, minlength=nbins))
        rows = host_rows(h)
        for q in np.argsort(bins, kind='stable'):
            glob[bins[q]].append(rows[q])
    counts = np.asarray(counts, np.int64)
    target, _, _ = plan_exchange(counts, num_shards)
    st = shard_targets(counts, num_shards)
    assert (st.max(0) - st.min(0) <= 1).all()
    owner = shard_owner(num_shards, W)
    got = [[] for _ in range(nbins)]
    for k, (h, bin_off, shards, shard_counts) in enumerate(outputs):
        np.testing.assert_array_equal(np.diff(bin_off), target[k])
        assert list(shards) == [s for s in range(num_shards) if owner[s] == k]
        np.testing.assert_array_equal(shard_counts, st[shards])
        np.testing.assert_array_equal(np.asarray(shard_counts).sum(0), target[k])
        rows = host_rows(h)
        assert len(rows) == bin_off[-1]
        for b in range(nbins):
            got[b] += rows[bin_off[b]:bin_off[b + 1]]
    for b in range(nbins):
        assert got[b] == glob[b], 'bin {} differs from the global stable order'.format(b)
