"""BERT pretraining loader — drop-in for lddl/torch/bert.py (`get_bert_pretrain_data_loader`,
199-413) with the collate on the GPU.

`_to_encoded_inputs` and `_mask_tokens` keep the reference's names, arguments and outputs, but
run as HIP kernels (lddl_collate_encode / lddl_mask_dynamic) and return cuda tensors (the
reference returns CPU tensors that the training loop then moves with `.to(device)`; on a cuda
tensor that call is a no-op).

Process split (SURVEY §7 "Fork + HIP"): the reference runs the whole collate inside forked
DataLoader workers. HIP must not be used there, so the workers only decode parquet record
batches, run the shuffle buffer and pack each batch into flat numpy buffers (`_pack_batch`);
the process that owns the GPU uploads the packed batch, runs the encode + masking kernels and
then the user's extra collate_fn. Sample order, bin choice and epoch logic are the reference's.
"""
import ctypes
import io
import logging
import os
import re
import time

import numpy as np
import torch

from .._native import lib, check
from ..context import Context, _ptr, _stream
from ..utils import get_all_bin_ids, get_all_parquets_under, get_file_paths_for_bin_id
from .dataloader import Binned, DataLoader
from .datasets import ParquetDataset
from .log import DatasetLogger
from .utils import get_node_rank, get_nproc_per_node, get_rank


def _decode_record_batch(b):
    """lddl/torch/bert.py:42-54: (A, B, is_random_next[, masked_lm_positions, labels])."""
    b = b.to_pydict()
    if 'masked_lm_positions' in b:
        assert 'masked_lm_labels' in b
    cols = tuple(b[k] for k in ('A', 'B', 'is_random_next', 'masked_lm_positions',
                                'masked_lm_labels') if k in b)
    for s in zip(*cols):
        yield s


class BertPretrainDataset(ParquetDataset):
    def _decode_record_batch(self, b):
        return _decode_record_batch(b)


def _npy_u16(b):
    """Decode `serialize_np_array` bytes (lddl/utils.py:98-102, np.save of uint16[k])."""
    if b[:6] == b'\x93NUMPY' and b[6] == 1:
        hl = int.from_bytes(b[8:10], 'little')
        hdr = b[10:10 + hl]
        if b"'<u2'" in hdr and b'False' in hdr:
            return np.frombuffer(b, np.uint16, offset=10 + hl)
    return np.load(io.BytesIO(b)).astype(np.uint16)


# whitespace of Python's str.split() (str.isspace()) that the kernel's ASCII splitter (space and
# \t-\r, the bytes.split() set) does not treat as a separator
_ODD_WS = re.compile('[\x1c-\x1f\x85\xa0\u1680\u2000-\u200a\u2028\u2029\u202f\u205f\u3000]')


# UTF-8 byte sequences that every string holding such whitespace contains (\xe2\x80 also
# starts common punctuation: those strings get the exact regex check)
_ODD_WS_SEQ = (b'\x1c', b'\x1d', b'\x1e', b'\x1f', b'\xc2\x85', b'\xc2\xa0', b'\xe1\x9a\x80',
               b'\xe2\x80', b'\xe2\x81\x9f', b'\xe3\x80\x80')


def _canon(s):
    """The string as the GPU splitter sees it, UTF-8 encoded: the reference splits with Python's
    str.split() (Unicode whitespace, bert.py:80-81); the kernel splits on ASCII space / \\t-\\r.
    Strings holding any other whitespace are re-joined with single spaces first (same tokens)."""
    b = s.encode('utf-8')
    if any(q in b for q in _ODD_WS_SEQ) and _ODD_WS.search(s):
        return ' '.join(s.split()).encode('utf-8')
    return b


def _ntok(b):
    """len(b.split()) (ASCII whitespace) without building the token list: a string of tokens
    joined by single spaces (what the preprocessor writes) has count(' ') + 1."""
    if not b:
        return 0
    if (b[0] == 32 or b[-1] == 32 or b'  ' in b or b'\t' in b or b'\n' in b or b'\r' in b or
            b'\x0b' in b or b'\x0c' in b):
        return len(b.split())
    return b.count(b' ') + 1


def _pack(batch, static):
    """Flat host buffers of a batch: A and B strings back to back (separators canonicalised to
    ASCII), their token counts (bytes.split() of the canonical strings = the reference's
    str.split(), bert.py:80-81) and offsets and, with static masking, the labels strings and
    decoded positions. Runs in the DataLoader workers, so the main process never has to wait for
    the batch's shape."""
    As = [_canon(s[0]) for s in batch]
    Bs = [_canon(s[1]) for s in batch]
    na = np.fromiter(map(_ntok, As), np.int32, len(batch))
    nb = np.fromiter(map(_ntok, Bs), np.int32, len(batch))
    la = np.fromiter(map(len, As), np.int64, len(batch))
    lb = np.fromiter(map(len, Bs), np.int64, len(batch))
    a_off = np.zeros(len(batch) + 1, np.int64)
    a_off[1:] = np.cumsum(la)
    b_off = a_off[-1] + np.concatenate([[0], np.cumsum(lb)])
    parts = As + Bs
    extra = None
    if static:
        labs = [_canon(s[4]) for s in batch]
        lab_off = np.zeros(len(batch) + 1, np.int64)
        lab_off[1:] = np.cumsum([len(x) for x in labs])
        lab_off += b_off[-1]
        pos = [_npy_u16(s[3]) for s in batch]
        pos_off = np.zeros(len(batch) + 1, np.int64)
        pos_off[1:] = np.cumsum([len(p) for p in pos])
        parts += labs
        extra = (lab_off, np.concatenate(pos) if pos else np.zeros(0, np.uint16), pos_off)
    blob = np.frombuffer(bytearray(b''.join(parts)), np.uint8)
    return blob, a_off, b_off, na, nb, extra


def _dev(a, device):
    """Host array -> device through a pinned staging copy: a copy from pageable memory would
    make the host wait for everything queued before it (the consumer's training step)."""
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(device, non_blocking=True)


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


class PackedBatch:
    """A collated batch as flat host buffers (built in a DataLoader worker, picklable)."""

    def __init__(self, batch):
        t0 = time.perf_counter()
        self.static = len(batch[0]) > 3
        self.blob, self.a_off, self.b_off, self.na, self.nb, self.extra = _pack(batch, self.static)
        self.nsl = np.asarray([s[2] for s in batch], np.int64)
        self.pack_s = time.perf_counter() - t0  # host time of the pack (in the worker)

    def __len__(self):
        return len(self.nsl)


def _pack_batch(batch):
    return PackedBatch(batch)


def encode_packed(pk, ctx, sequence_length_alignment=8, ignore_index=-1, mask=None, events=None):
    """`_to_encoded_inputs` on an already packed batch (main process, GPU).

    mask = (mlm_probability, seed, counter) on a dynamic-masking batch runs `_mask_tokens` fused
    into the same kernel (lddl_collate_encode_masked) and returns `labels` instead of
    `special_tokens_mask`. events: optional pair of torch.cuda.Event recorded around the
    encode kernel (timing)."""
    dev = ctx.device
    B = len(pk)
    seq = int((pk.na + pk.nb).max()) + 3  # the batch's shape (bert.py:91-96), known on the host
    L = ((seq - 1) // sequence_length_alignment + 1) * sequence_length_alignment
    d_blob = _dev(pk.blob, dev) if len(pk.blob) else torch.zeros(1, dtype=torch.uint8, device=dev)
    d_off = _dev(np.concatenate([pk.a_off, pk.b_off]), dev)
    d_a, d_b = d_off[:B + 1], d_off[B + 1:]
    d_cnt = _dev(np.concatenate([pk.na, pk.nb]), dev)
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
        out['next_sentence_labels'] = _dev(pk.nsl, dev)
        out['labels'] = labels
        return out
    stm = labels = d_lab_off = d_pos = d_pos_off = None
    if pk.static:
        lab_off, pos, pos_off = pk.extra
        if len(pos) and int(pos.max()) >= L:  # the reference's labels[i][positions] raises
            raise IndexError('masked_lm_positions holds {} >= sequence length {}'.format(
                int(pos.max()), L))
        d_lab_off, d_pos_off = _dev(lab_off, dev), _dev(pos_off, dev)
        d_pos = _dev(pos.view(np.int16), dev) if len(pos) else torch.zeros(1, dtype=torch.int16,
                                                                           device=dev)
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
    out['next_sentence_labels'] = _dev(pk.nsl, dev)
    if pk.static:
        out['labels'] = labels
    else:
        out['special_tokens_mask'] = stm
    return out


class GPUCollateLoader:
    """Iterates a torch DataLoader of PackedBatch and finishes the collate on the GPU."""

    def __init__(self, loader, ctx, mlm_probability, ignore_index, sequence_length_alignment,
                 extra_collate, seed, start_epoch=0):
        self._loader = loader
        self._ctx = ctx
        self._mlm = mlm_probability
        self._ignore = ignore_index
        self._align = sequence_length_alignment
        self._extra = extra_collate
        self._seed = seed            # Philox key: distinct per (base_seed, rank, bin)
        self._epoch = start_epoch    # counter = epoch << 32 | batch: no stream repeats across
        self._counter = start_epoch << 32  # epochs, and a resumed run continues, not replays
        self.stats = None  # dict(pack_s=[], blob_bytes=[], events=[], slots=[]): record timings

    @property
    def dataset(self):
        return self._loader.dataset

    def __len__(self):
        return len(self._loader)

    def __getattr__(self, k):
        return getattr(self._loader, k)

    def __iter__(self):
        self._counter = self._epoch << 32
        self._epoch += 1
        for pk in self._loader:
            ev = None
            if self.stats is not None:
                self.stats['pack_s'].append(pk.pack_s)
                self.stats['blob_bytes'].append(len(pk.blob))
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            # the batch shape is known on the host (counted in the worker): nothing here waits
            # for the GPU, the collate kernel is queued behind the consumer's training step
            with torch.no_grad():  # dynamic masking: collate + _mask_tokens in one kernel
                enc = encode_packed(pk, self._ctx, self._align, self._ignore,
                                    mask=(self._mlm, self._seed, self._counter), events=ev)
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
    ctx = None
    if not return_raw_samples:
        ctx = Context(vocab_file, do_lower_case=tokenizer_kwargs.get('do_lower_case', True))
        data_loader_kwargs['collate_fn'] = _pack_batch
    data_loader_kwargs['persistent_workers'] = True

    def make(paths, bin_id=-1):
        dl = data_loader_class(BertPretrainDataset(paths, **dataset_kwargs), **data_loader_kwargs)
        if return_raw_samples:
            return dl
        return GPUCollateLoader(dl, ctx, mlm_probability, ignore_index,
                                sequence_length_alignment, extra_collate,
                                mask_seed(base_seed, get_rank(), bin_id), start_epoch)

    paths = get_all_parquets_under(path)
    bin_ids = get_all_bin_ids(paths)
    if bin_ids:
        return BertPretrainBinned([make(get_file_paths_for_bin_id(paths, b), b) for b in bin_ids],
                                  base_seed=base_seed, start_epoch=start_epoch, logger=logger)
    return make(paths)
