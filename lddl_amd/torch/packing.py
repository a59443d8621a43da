"""Worker-side half of the BERT loader (lddl/torch/bert.py:42-149, host part): decoding parquet
record batches and packing a collated batch into flat numpy buffers.

This module is what DataLoader workers run. It imports neither the native library nor anything
that touches the GPU, so a worker started with `spawn` / `forkserver` never loads HIP, and a
forked one never calls it (the HIP context is never used across `fork()`)."""
import io
import re
import time

import numpy as np

from .datasets import ParquetDataset


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
