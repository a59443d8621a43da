"""Dynamic-masking stream keys (per-bin seeds, epoch-based counters). Host logic
only: the Philox key of each (base_seed, rank, bin) loader and the counter sequence across
epochs and resumes; the kernel that consumes them is covered by test_collate_gpu.py."""
import types

import lddl_amd.torch.bert as B


def test_mask_seed_distinct_per_rank_and_bin():
    seeds = {B.mask_seed(12345, r, b) for r in range(8) for b in range(-1, 64)}
    assert len(seeds) == 8 * 65
    assert B.mask_seed(1, 0, 0) != B.mask_seed(2, 0, 0)


class _Pk:
    static = False


def _counters(monkeypatch, start_epoch, epochs, n_batches=3):
    seen = []

    def fake_encode(pk, ctx, align, ignore, mask=None, events=None, stager=None):
        seen.append(mask)
        return {'input_ids': types.SimpleNamespace(numel=lambda: 0)}

    monkeypatch.setattr(B, 'encode_packed', fake_encode)
    ld = B.GPUCollateLoader([_Pk() for _ in range(n_batches)], None, 0.15, -1, 8, lambda e: e,
                            seed=B.mask_seed(7, 0, 3), start_epoch=start_epoch)
    for _ in range(epochs):
        list(ld)
    return seen


def test_counters_never_repeat_across_epochs(monkeypatch):
    seen = _counters(monkeypatch, 0, 3)
    ctr = [m[2] for m in seen]
    assert len(set(ctr)) == len(ctr) == 9
    assert ctr[:3] == [0, 1, 2] and ctr[3] == 1 << 32 and ctr[6] == 2 << 32


def test_resumed_run_continues_the_streams(monkeypatch):
    fresh = _counters(monkeypatch, 0, 3)
    resumed = _counters(monkeypatch, 2, 1)
    assert [m[2] for m in resumed] == [m[2] for m in fresh[6:]]
    assert {m[1] for m in resumed} == {B.mask_seed(7, 0, 3)}
