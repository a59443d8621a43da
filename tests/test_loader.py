"""lddl_amd.torch.get_bert_pretrain_data_loader vs batches of the reference loader
(tests/golden/loader.npz, made by tests/golden/make_loader_golden.py from the reference):
sample order (files permutation, rank/worker striding, shuffle buffer), bin choice per step,
epochs, len(), and (GPU) the collated tensors."""
import logging
import os

import numpy as np
import pytest

from conftest import GOLDEN, VOCAB_UNCASED
from loader_data import make_loader_dataset


@pytest.fixture(scope='module')
def golden():
    with np.load(os.path.join(GOLDEN, 'loader.npz')) as z:
        return dict(z)


def test_raw_sample_order_matches_reference(tmp_path, golden):
    from lddl_amd.torch import get_bert_pretrain_data_loader
    d = str(tmp_path / 'raw')
    make_loader_dataset(d, VOCAB_UNCASED, binned=False, static=False)
    dl = get_bert_pretrain_data_loader(
        d, local_rank=0, shuffle_buffer_size=8, shuffle_buffer_warmup_factor=2,
        vocab_file=VOCAB_UNCASED, data_loader_kwargs={'batch_size': 3, 'num_workers': 2},
        return_raw_samples=True, base_seed=777, start_epoch=1, log_level=logging.WARNING)
    seq = []
    for _ in range(2):
        for batch in dl:
            seq += ['{}|{}|{}'.format(a, b, int(c)) for a, b, c in zip(*batch[:3])]
            seq.append('--batch--')
    assert len(dl) == int(golden['raw_len'])
    assert seq == golden['raw_order'].tolist()


@pytest.mark.gpu
def test_binned_static_batches_match_reference(tmp_path, golden):
    from lddl_amd.torch import get_bert_pretrain_data_loader
    d = str(tmp_path / 'bin')
    make_loader_dataset(d, VOCAB_UNCASED, binned=True, static=True)
    dl = get_bert_pretrain_data_loader(
        d, local_rank=0, shuffle_buffer_size=8, shuffle_buffer_warmup_factor=2,
        vocab_file=VOCAB_UNCASED, data_loader_kwargs={'batch_size': 3, 'num_workers': 2},
        base_seed=4242, log_level=logging.WARNING)
    assert len(dl) == int(golden['bin_len'])
    k = 0
    for _ in range(2):
        for batch in dl:
            for name in ('input_ids', 'token_type_ids', 'attention_mask', 'labels',
                         'next_sentence_labels'):
                got = batch[name]
                assert got.is_cuda
                np.testing.assert_array_equal(got.cpu().numpy(),
                                              golden['bin{}_{}'.format(k, name)], err_msg=name)
            k += 1
    assert k == int(golden['bin_steps'])


@pytest.mark.gpu
def test_dynamic_masking_loader(tmp_path):
    """Dynamic masking (no mask columns): rates over non-special slots, labels consistent."""
    import torch
    from lddl_amd.torch import get_bert_pretrain_data_loader
    d = str(tmp_path / 'dyn')
    make_loader_dataset(d, VOCAB_UNCASED, binned=True, static=False)
    dl = get_bert_pretrain_data_loader(
        d, vocab_file=VOCAB_UNCASED, data_loader_kwargs={'batch_size': 4, 'num_workers': 2},
        log_level=logging.WARNING)
    n = 0
    for batch in dl:
        assert set(batch) == {'input_ids', 'token_type_ids', 'attention_mask', 'labels',
                              'next_sentence_labels'}
        lab = batch['labels']
        assert ((lab == -1) | (batch['attention_mask'] == 1)).all()
        n += batch['input_ids'].size(0)
    assert n == sum(len(x.dataset) for x in dl._dataloaders)


class _CtxProbe(Exception):
    pass


def test_context_created_after_all_workers_start(tmp_path, monkeypatch):
    """The loader's HIP Context exists only after every bin's DataLoader workers have been
    started (no worker is forked from a process holding this library's HIP state).
    CPU: the Context is replaced by a probe that records the workers' state and stops."""
    from lddl_amd.torch import bert
    d = str(tmp_path / 'bin')
    make_loader_dataset(d, VOCAB_UNCASED, binned=True, static=False)
    seen = []
    holder = {}

    class Probe:
        def __init__(self, *a, **k):
            for gl in holder['dl']._dataloaders:
                it = gl._loader._iterator
                seen.append(it is not None and len(it._workers) == 2 and
                            all(w.is_alive() for w in it._workers))
            raise _CtxProbe()

    monkeypatch.setattr(bert, 'Context', Probe)
    dl = bert.get_bert_pretrain_data_loader(
        d, vocab_file=VOCAB_UNCASED, data_loader_kwargs={'batch_size': 4, 'num_workers': 2},
        log_level=logging.WARNING)
    holder['dl'] = dl
    assert len(dl._dataloaders) > 1
    assert all(gl._lazy.ctx is None for gl in dl._dataloaders)  # nothing created yet
    with pytest.raises(_CtxProbe):
        next(iter(dl))
    assert seen and all(seen), seen
    for gl in dl._dataloaders:  # end the persistent workers
        gl._loader._iterator._shutdown_workers()


def _assert_no_native(worker_id):
    import sys
    assert 'lddl_amd._native' not in sys.modules, 'a DataLoader worker loaded the native library'


def test_spawned_workers_same_order_without_native_library(tmp_path, golden):
    """Workers started with `spawn` (a fresh interpreter: nothing of the parent's HIP state is
    inherited) yield the reference's order, and import only the worker-side modules."""
    from lddl_amd.torch import get_bert_pretrain_data_loader
    d = str(tmp_path / 'raw')
    make_loader_dataset(d, VOCAB_UNCASED, binned=False, static=False)
    dl = get_bert_pretrain_data_loader(
        d, local_rank=0, shuffle_buffer_size=8, shuffle_buffer_warmup_factor=2,
        vocab_file=VOCAB_UNCASED,
        data_loader_kwargs={'batch_size': 3, 'num_workers': 2, 'multiprocessing_context': 'spawn',
                            'worker_init_fn': _assert_no_native},
        return_raw_samples=True, base_seed=777, start_epoch=1, log_level=logging.WARNING)
    seq = []
    for _ in range(2):
        for batch in dl:
            seq += ['{}|{}|{}'.format(a, b, int(c)) for a, b, c in zip(*batch[:3])]
            seq.append('--batch--')
    assert seq == golden['raw_order'].tolist()
