"""GPU collate for the BERT loader — counterparts of lddl/torch/bert.py:69-196.

`_to_encoded_inputs` and `_mask_tokens` keep the reference's names, arguments and outputs, but
run as HIP kernels (lddl_collate_encode / lddl_mask_dynamic) and return cuda tensors (the
reference returns CPU tensors that the training loop then moves with `.to(device)`; on a cuda
tensor that call is a no-op).

HIP must not be initialised in forked DataLoader workers ("Fork + HIP"): these functions
run in the process that owns the GPU; the loader's workers only decode parquet into raw samples.
"""
import ctypes
import io

import numpy as np
import torch

from .._native import lib, check
from ..context import _ptr, _stream


def _npy_u16(b):
    """Decode `serialize_np_array` bytes (lddl/utils.py:98-102, np.save of uint16[k])."""
    if b[:6] == b'\x93NUMPY' and b[6] == 1:
        hl = int.from_bytes(b[8:10], 'little')
        hdr = b[10:10 + hl]
        if b"'<u2'" in hdr and b'False' in hdr:
            return np.frombuffer(b, np.uint16, offset=10 + hl)
    return np.load(io.BytesIO(b)).astype(np.uint16)


def _pack(batch, static):
    As = [s[0].encode('utf-8') for s in batch]
    Bs = [s[1].encode('utf-8') for s in batch]
    na = np.fromiter((len(s[0].split()) for s in batch), np.int32, len(batch))
    nb = np.fromiter((len(s[1].split()) for s in batch), np.int32, len(batch))
    la = np.fromiter(map(len, As), np.int64, len(batch))
    lb = np.fromiter(map(len, Bs), np.int64, len(batch))
    a_off = np.zeros(len(batch) + 1, np.int64)
    a_off[1:] = np.cumsum(la)
    b_off = a_off[-1] + np.concatenate([[0], np.cumsum(lb)])
    parts = As + Bs
    extra = None
    if static:
        labs = [s[4].encode('utf-8') for s in batch]
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
    return torch.from_numpy(np.ascontiguousarray(a)).to(device, non_blocking=True)


def _to_encoded_inputs(batch, tokenizer, sequence_length_alignment=8, ignore_index=-1):
    """lddl/torch/bert.py:69-149. `tokenizer` is a lddl_amd.context.Context."""
    ctx = tokenizer
    dev = ctx.device
    B = len(batch)
    static = len(batch[0]) > 3
    if static:
        assert len(batch[0]) == 5
    blob, a_off, b_off, na, nb, extra = _pack(batch, static)
    seq = int((na + nb).max()) + 3
    L = ((seq - 1) // sequence_length_alignment + 1) * sequence_length_alignment
    d_blob = _dev(blob, dev) if len(blob) else torch.zeros(1, dtype=torch.uint8, device=dev)
    d_a, d_b, d_na, d_nb = (_dev(x, dev) for x in (a_off, b_off, na, nb))
    out = {k: torch.empty(B, L, dtype=torch.long, device=dev)
           for k in ('input_ids', 'token_type_ids', 'attention_mask')}
    stm = labels = d_lab_off = d_pos = d_pos_off = None
    if static:
        lab_off, pos, pos_off = extra
        d_lab_off, d_pos_off = _dev(lab_off, dev), _dev(pos_off, dev)
        d_pos = _dev(pos.view(np.int16), dev) if len(pos) else torch.zeros(1, dtype=torch.int16,
                                                                           device=dev)
        labels = torch.empty(B, L, dtype=torch.long, device=dev)
    else:
        stm = torch.empty(B, L, dtype=torch.long, device=dev)
    check(lib.lddl_collate_encode(ctx.handle, _stream(), _ptr(d_blob), _ptr(d_a), _ptr(d_b),
                                  _ptr(d_na), _ptr(d_nb), B, L, _ptr(out['input_ids']),
                                  _ptr(out['token_type_ids']), _ptr(out['attention_mask']),
                                  _ptr(stm), _ptr(d_blob) if static else None, _ptr(d_lab_off),
                                  _ptr(d_pos), _ptr(d_pos_off), _ptr(labels), ignore_index))
    out['next_sentence_labels'] = torch.as_tensor([s[2] for s in batch], dtype=torch.long).to(dev)
    if static:
        out['labels'] = labels
    else:
        out['special_tokens_mask'] = stm
    return out


def _mask_tokens(inputs, special_tokens_mask=None, tokenizer=None, mlm_probability=0.15,
                 ignore_index=-1, seed=12345, counter=0, replay=None):
    """lddl/torch/bert.py:152-196 on the GPU; masks `inputs` in place and returns
    (inputs, labels).

    Native mode draws from Philox keyed by (seed, counter): pass a new counter per batch.
    replay = dict(masked=, replaced=, random=, words=) applies captured torch draws exactly.
    """
    ctx = tokenizer
    assert inputs.is_cuda and inputs.dtype == torch.long and inputs.is_contiguous()
    B, L = inputs.shape
    labels = torch.empty_like(inputs)
    stm = special_tokens_mask
    if stm is None:
        raise ValueError('special_tokens_mask is required (the GPU path has no per-id lookup)')
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
