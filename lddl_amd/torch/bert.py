"""BERT pretraining loader — drop-in for lddl/torch/bert.py (`get_bert_pretrain_data_loader`,
199-413) with the collate on the GPU.

`_to_encoded_inputs` and `_mask_tokens` keep the reference's names, arguments and outputs, but
run as HIP kernels (lddl_collate_encode / lddl_mask_dynamic) and return cuda tensors (the
reference returns CPU tensors that the training loop then moves with `.to(device)`; on a cuda
tensor that call is a no-op).

Process split (SURVEY §7 "Fork + HIP"): the reference runs the whole collate inside forked
DataLoader workers. HIP must not be used there, so the workers only decode parquet record
batches, run the shuffle buffer and pack each batch into flat numpy buffers (`packing.py`,
which imports nothing of the native library); the process that owns the GPU uploads the packed
batch through a reused pinned ring (`HostStager`), runs the encode + masking kernel and then
the user's extra collate_fn. The HIP Context is created only after every bin's workers have
started (`_LazyContext`). Sample order, bin choice and epoch logic are the reference's.
"""
import logging
import os

import numpy as np
import torch

from .._native import lib, check
from ..context import Context, _ptr, _stream
from ..utils import get_all_bin_ids, get_all_parquets_under, get_file_paths_for_bin_id
from .dataloader import Binned, DataLoader
from .datasets import ParquetDataset  # noqa: F401
from .log import DatasetLogger
from .packing import (BertPretrainDataset, PackedBatch, _canon, _decode_record_batch,  # noqa: F401
                      _npy_u16, _ntok, _pack, _pack_batch)
from .utils import get_node_rank, get_nproc_per_node, get_rank


class HostStager:
    """A ring of reused pinned host buffers: all host arrays of one batch are packed into one
    slot and go to the device in ONE asynchronous copy.

    A copy from pageable memory would make the host wait for everything queued before it (the
    consumer's training step); a fresh `.pin_memory()` per array and batch (round 3) called
    hipHostMalloc whenever torch's host cache missed (86 calls, up to 143 ms each,
    profiles/r03h_c5_hip_api.txt). A slot is reused once the event recorded after its copy has
    completed, so at most `depth` batches are in flight and no pinned memory is allocated once
    the slots have grown to the largest batch."""

    ALIGN = 64

    def __init__(self, depth=4):
        self._bufs = [None] * depth
        self._done = [None] * depth
        self._i = 0
        self.allocations = 0  # pinned (re)allocations so far: flat after warm-up

    def stage(self, arrays, device):
        """arrays: host numpy arrays -> device tensors (same dtypes and shapes), in order."""
        arrays = [np.ascontiguousarray(a) for a in arrays]
        offs, n = [], 0
        for a in arrays:
            offs.append(n)
            n += -(-max(a.nbytes, 1) // self.ALIGN) * self.ALIGN
        k = self._i % len(self._bufs)
        self._i += 1
        if self._done[k] is not None:
            self._done[k].synchronize()  # this slot's previous copy has left the host buffer
        buf = self._bufs[k]
        if buf is None or buf.numel() < n:
            cap = 1 << max(16, (n - 1).bit_length())
            buf = self._bufs[k] = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            self.allocations += 1
        hv = buf.numpy()
        for a, o in zip(arrays, offs):
            hv[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
        # the copy and its slot-reuse event on the DESTINATION device's current stream (the
        # current device may be another one: an event recorded there would not cover the copy)
        with torch.cuda.device(device):
            d = torch.empty(n, dtype=torch.uint8, device=device)
            d.copy_(buf[:n], non_blocking=True)
            ev = self._done[k] = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(device))
        out = []
        for a, o in zip(arrays, offs):
            t = d[o:o + max(a.nbytes, 1)]
            if a.nbytes == 0:  # a 1-byte placeholder keeps the pointer valid (never read)
                out.append(t.view(torch.uint8)[:0])
            else:
                out.append(t.view(_TORCH_DTYPE[a.dtype.str[1:]]).view(a.shape))
        return out


_TORCH_DTYPE = {'u1': torch.uint8, 'i1': torch.int8, 'i2': torch.int16, 'i4': torch.int32,
                'i8': torch.int64, 'u2': torch.int16, 'f4': torch.float32}
_DEFAULT_STAGER = {}


def _stager_for(device):
    s = _DEFAULT_STAGER.get(str(device))
    if s is None:
        s = _DEFAULT_STAGER[str(device)] = HostStager()
    return s


def _to_encoded_inputs(batch, tokenizer, sequence_length_alignment=8, ignore_index=-1):
    """lddl/torch/bert.py:69-149. `tokenizer` is a lddl_amd.context.Context."""
    if len(batch[0]) > 3:
        assert len(batch[0]) == 5
    return encode_packed(PackedBatch(batch), tokenizer, sequence_length_alignment, ignore_index)


def _mask_tokens(inputs, special_tokens_mask=None, tokenizer=None, mlm_probability=0.15,
                 ignore_index=-1, seed=12345, counter=0, replay=None):
    """lddl/torch/bert.py:152-196 on the GPU; masks `inputs` in place and returns
    (inputs, labels).

    special_tokens_mask=None marks the slots whose id is a special token, as the reference's
    tokenizer.get_special_tokens_mask(ids, already_has_special_tokens=True) (bert.py:167-172).
    Native mode draws from Philox keyed by (seed, counter): pass a new counter per batch.
    replay = dict(masked=, replaced=, random=, words=) applies captured torch draws exactly.
    """
    ctx = tokenizer
    assert inputs.is_cuda and inputs.dtype == torch.long and inputs.is_contiguous()
    B, L = inputs.shape
    labels = torch.empty_like(inputs)
    stm = special_tokens_mask
    if stm is not None:
        stm = stm.to(device=inputs.device, dtype=torch.long).contiguous()
    r = [None] * 4
    if replay is not None:
        r = [replay['masked'].to(inputs.device, torch.uint8).contiguous(),
             replay['replaced'].to(inputs.device, torch.uint8).contiguous(),
             replay['random'].to(inputs.device, torch.uint8).contiguous(),
             replay['words'].to(inputs.device, torch.long).contiguous()]
    check(lib.lddl_mask_dynamic(ctx.handle, _stream(), _ptr(inputs), _ptr(labels), _ptr(stm), None,
                                None, B, L, float(mlm_probability), ignore_index, len(ctx), seed,
                                counter, *[_ptr(x) for x in r]))
    return inputs, labels


def encode_packed(pk, ctx, sequence_length_alignment=8, ignore_index=-1, mask=None, events=None,
                  stager=None):
    """`_to_encoded_inputs` on an already packed batch (main process, GPU).

    mask = (mlm_probability, seed, counter) on a dynamic-masking batch runs `_mask_tokens` fused
    into the same kernel (lddl_collate_encode_masked) and returns `labels` instead of
    `special_tokens_mask`. events: optional pair of torch.cuda.Event recorded around the
    encode kernel (timing). stager: the HostStager whose pinned ring carries the batch to the
    device (default: one per device)."""
    dev = ctx.device
    B = len(pk)
    seq = int((pk.na + pk.nb).max()) + 3  # the batch's shape (bert.py:91-96), known on the host
    L = ((seq - 1) // sequence_length_alignment + 1) * sequence_length_alignment
    host = [pk.blob, np.concatenate([pk.a_off, pk.b_off]), np.concatenate([pk.na, pk.nb]), pk.nsl]
    if pk.static:
        lab_off, pos, pos_off = pk.extra
        if len(pos) and int(pos.max()) >= L:  # the reference's labels[i][positions] raises
            raise IndexError('masked_lm_positions holds {} >= sequence length {}'.format(
                int(pos.max()), L))
        host += [lab_off, pos_off, pos.view(np.int16)]
    staged = (stager or _stager_for(dev)).stage(host, dev)  # one H2D copy for the whole batch
    d_blob, d_off, d_cnt, d_nsl = staged[:4]
    d_a, d_b = d_off[:B + 1], d_off[B + 1:]
    d_na, d_nb = d_cnt[:B], d_cnt[B:]
    out = {k: torch.empty(B, L, dtype=torch.long, device=dev)
           for k in ('input_ids', 'token_type_ids', 'attention_mask')}
    if mask is not None and not pk.static:
        p, seed, counter = mask
        labels = torch.empty(B, L, dtype=torch.long, device=dev)
        if events is not None:
            events[0].record()
        check(lib.lddl_collate_encode_masked(
            ctx.handle, _stream(), _ptr(d_blob), _ptr(d_a), _ptr(d_b), _ptr(d_na), _ptr(d_nb), B,
            L, _ptr(out['input_ids']), _ptr(out['token_type_ids']), _ptr(out['attention_mask']),
            _ptr(labels), float(p), ignore_index, len(ctx), seed, counter))
        if events is not None:
            events[1].record()
        out['next_sentence_labels'] = d_nsl
        out['labels'] = labels
        return out
    stm = labels = d_lab_off = d_pos = d_pos_off = None
    if pk.static:
        d_lab_off, d_pos_off, d_pos = staged[4:]
        labels = torch.empty(B, L, dtype=torch.long, device=dev)
    else:
        stm = torch.empty(B, L, dtype=torch.long, device=dev)
    if events is not None:
        events[0].record()
    check(lib.lddl_collate_encode(ctx.handle, _stream(), _ptr(d_blob), _ptr(d_a), _ptr(d_b),
                                  _ptr(d_na), _ptr(d_nb), B, L, _ptr(out['input_ids']),
                                  _ptr(out['token_type_ids']), _ptr(out['attention_mask']),
                                  _ptr(stm), _ptr(d_blob) if pk.static else None, _ptr(d_lab_off),
                                  _ptr(d_pos), _ptr(d_pos_off), _ptr(labels), ignore_index))
    if events is not None:
        events[1].record()
    out['next_sentence_labels'] = d_nsl
    if pk.static:
        out['labels'] = labels
    else:
        out['special_tokens_mask'] = stm
    return out


class _LazyContext:
    """The loader's HIP Context, created on first use: after the DataLoader workers of every bin
    have been started, so no worker is ever forked from a process holding this library's HIP
    state."""

    def __init__(self, vocab_file, do_lower_case):
        self._args = (vocab_file, do_lower_case)
        self.ctx = None

    def get(self):
        if self.ctx is None:
            self.ctx = Context(self._args[0], do_lower_case=self._args[1])
        return self.ctx


class GPUCollateLoader:
    """Iterates a torch DataLoader of PackedBatch and finishes the collate on the GPU."""

    def __init__(self, loader, ctx, mlm_probability, ignore_index, sequence_length_alignment,
                 extra_collate, seed, start_epoch=0, stager=None):
        self._loader = loader
        self._lazy = ctx if isinstance(ctx, _LazyContext) else None
        self._ctx_obj = None if self._lazy is not None else ctx
        self._mlm = mlm_probability
        self._ignore = ignore_index
        self._align = sequence_length_alignment
        self._extra = extra_collate
        self._seed = seed            # Philox key: distinct per (base_seed, rank, bin)
        self._epoch = start_epoch    # counter = epoch << 32 | batch: no stream repeats across
        self._counter = start_epoch << 32  # epochs, and a resumed run continues, not replays
        self._stager = stager
        self.stats = None  # dict(pack_s=[], blob_bytes=[], events=[], slots=[]): record timings

    @property
    def _ctx(self):
        return self._lazy.get() if self._lazy is not None else self._ctx_obj

    @property
    def dataset(self):
        return self._loader.dataset

    def __len__(self):
        return len(self._loader)

    def __getattr__(self, k):
        return getattr(self._loader, k)

    def __iter__(self):
        """Starts (or, persistent, resets) the DataLoader's workers NOW, before the first batch
        is asked for: `Binned` creates every bin's iterator before it draws from any, so all
        workers exist before the Context does."""
        self._counter = self._epoch << 32
        self._epoch += 1
        return self._batches(iter(self._loader))

    def _batches(self, it):
        for pk in it:
            ctx = self._ctx
            ev = None
            if self.stats is not None:
                self.stats['pack_s'].append(pk.pack_s)
                self.stats['blob_bytes'].append(len(pk.blob))
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            # the batch shape is known on the host (counted in the worker): nothing here waits
            # for the GPU, the collate kernel is queued behind the consumer's training step
            with torch.no_grad():  # dynamic masking: collate + _mask_tokens in one kernel
                enc = encode_packed(pk, ctx, self._align, self._ignore,
                                    mask=(self._mlm, self._seed, self._counter), events=ev,
                                    stager=self._stager)
            if not pk.static:
                self._counter += 1
            if self.stats is not None:
                self.stats['events'].append(ev)
                self.stats['slots'].append(enc['input_ids'].numel())
            yield self._extra(enc)


def mask_seed(base_seed, rank, bin_id=-1):
    """64-bit Philox key of one (rank, bin) loader's dynamic masking: independent streams per
    rank and per bin (the reference draws all of them from each worker's torch RNG)."""
    return ((int(base_seed) * 1000003 + int(rank)) * 65537 + int(bin_id) + 1) & ((1 << 64) - 1)


class BertPretrainBinned(Binned):
    def _get_batch_size(self, batch):
        if isinstance(batch, dict):
            return batch['input_ids'].size(0)
        return len(batch[0]) if isinstance(batch, (list, tuple)) else len(batch)


def get_bert_pretrain_data_loader(path, local_rank=0, shuffle_buffer_size=16384,
                                  shuffle_buffer_warmup_factor=16, tokenizer_class=None,
                                  vocab_file=None, tokenizer_kwargs={}, data_loader_class=DataLoader,
                                  data_loader_kwargs={}, mlm_probability=0.15, base_seed=12345,
                                  log_dir=None, log_level=logging.INFO, return_raw_samples=False,
                                  start_epoch=0, sequence_length_alignment=8, ignore_index=-1):
    """Same signature, arguments and yielded dicts as lddl.torch.get_bert_pretrain_data_loader
    (lddl/torch/bert.py:199-413); the tensors are on the current cuda device.

    tokenizer_class is accepted for compatibility (BertTokenizerFast / BertTokenizer or None):
    the vocab file is loaded into a lddl_amd Context (vocab hash in HBM). vocab_file must be a
    local path (no model-name download offline)."""
    assert isinstance(path, str)
    assert isinstance(local_rank, int) and local_rank >= 0
    assert isinstance(shuffle_buffer_size, int) and shuffle_buffer_size > 0
    assert isinstance(shuffle_buffer_warmup_factor, int) and shuffle_buffer_warmup_factor > 0
    if tokenizer_class is not None:
        assert getattr(tokenizer_class, '__name__', '') in {'BertTokenizerFast', 'BertTokenizer'}
    assert isinstance(vocab_file, str)
    assert isinstance(tokenizer_kwargs, dict)
    assert data_loader_class in {DataLoader}
    assert isinstance(data_loader_kwargs, dict)
    assert isinstance(mlm_probability, (int, float)) and 0 <= mlm_probability <= 1
    assert isinstance(base_seed, int)
    assert log_dir is None or isinstance(log_dir, str)
    assert log_level in {logging.NOTSET, logging.DEBUG, logging.INFO, logging.WARNING,
                         logging.ERROR, logging.CRITICAL}
    assert isinstance(return_raw_samples, bool)
    assert isinstance(start_epoch, int)
    if not os.path.isfile(vocab_file):
        raise FileNotFoundError('vocab_file {!r}: a local vocab.txt is required (offline)'.format(
            vocab_file))
    data_loader_kwargs = dict(data_loader_kwargs)
    logger = DatasetLogger(log_dir=log_dir,
                           node_rank=get_node_rank(nproc_per_node=get_nproc_per_node(local_rank)),
                           local_rank=local_rank, log_level=log_level)
    dataset_kwargs = dict(local_rank=local_rank, shuffle_buffer_size=shuffle_buffer_size,
                          shuffle_buffer_warmup_factor=shuffle_buffer_warmup_factor,
                          base_seed=base_seed, logger=logger, start_epoch=start_epoch)
    extra_collate = data_loader_kwargs.get('collate_fn', lambda x: x)
    ctx = stager = None
    if not return_raw_samples:  # the Context is created after the workers start (_LazyContext)
        ctx = _LazyContext(vocab_file, tokenizer_kwargs.get('do_lower_case', True))
        stager = HostStager()
        data_loader_kwargs['collate_fn'] = _pack_batch
    data_loader_kwargs['persistent_workers'] = True

    def make(paths, bin_id=-1):
        dl = data_loader_class(BertPretrainDataset(paths, **dataset_kwargs), **data_loader_kwargs)
        if return_raw_samples:
            return dl
        return GPUCollateLoader(dl, ctx, mlm_probability, ignore_index,
                                sequence_length_alignment, extra_collate,
                                mask_seed(base_seed, get_rank(), bin_id), start_epoch, stager)

    paths = get_all_parquets_under(path)
    bin_ids = get_all_bin_ids(paths)
    if bin_ids:
        return BertPretrainBinned([make(get_file_paths_for_bin_id(paths, b), b) for b in bin_ids],
                                  base_seed=base_seed, start_epoch=start_epoch, logger=logger)
    return make(paths)
