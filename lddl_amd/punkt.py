"""GPU Punkt sentence segmentation: the reference's `nltk.tokenize.sent_tokenize(text)` followed by
`strip()` and dropping empty sentences (lddl/dask/bert/pretrain.py:86-88), for a whole batch of
documents at once (csrc/segment.hip, C-ABI `lddl_segment_count` / `lddl_segment_fill`).

Parameters mirror nltk's `PunktParameters` (nltk/tokenize/punkt.py:333-369, nltk 3.6.5):
abbreviation types, collocations, frequent sentence starters and orthographic context. nltk's
English model is a run-time download the reference performs (`nltk.download('punkt')`); offline,
`sent_tokenize` has no model and the untrained `PunktSentenceTokenizer()` is what runs, which
is `PunktParams()` (empty). A trained model can be used through `PunktParams.from_nltk(tok)`
(an nltk `PunktSentenceTokenizer` the caller loaded) or `PunktParams.from_json(path)`.
"""
import json
import os
import struct

import numpy as np
import torch

from ._native import lib, check

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets')
KIND_ABBREV, KIND_STARTER, KIND_ORTHO, KIND_COLLOC = 1, 2, 3, 4


class PunktParams:
    """abbrev_types: set[str]; collocations: set[(str, str)]; sent_starters: set[str];
    ortho_context: dict[str, int] (nltk _ORTHO_* flags)."""

    def __init__(self, abbrev_types=(), collocations=(), sent_starters=(), ortho_context=None):
        self.abbrev_types = set(abbrev_types)
        self.collocations = set(tuple(c) for c in collocations)
        self.sent_starters = set(sent_starters)
        self.ortho_context = dict(ortho_context or {})

    @classmethod
    def from_dict(cls, d):
        return cls(d.get('abbrev_types', ()), d.get('collocations', ()),
                   d.get('sent_starters', ()), d.get('ortho_context', {}))

    @classmethod
    def from_json(cls, path):
        with open(path) as f:
            return cls.from_dict(json.load(f))

    @classmethod
    def from_nltk(cls, tokenizer):
        """From an nltk PunktSentenceTokenizer (or PunktParameters) already loaded by the caller."""
        p = getattr(tokenizer, '_params', tokenizer)
        return cls(p.abbrev_types, p.collocations, p.sent_starters,
                   {k: int(v) for k, v in p.ortho_context.items() if v})

    def records(self):
        """The C-ABI record blob (include/lddl_amd.h, lddl_punkt_set_params)."""
        out = []

        def rec(kind, value, a, b=''):
            a, b = a.encode('utf-8'), b.encode('utf-8')
            if len(a) > 255 or len(b) > 255:
                raise ValueError('Punkt parameter key longer than 255 bytes: {!r}'.format(a))
            out.append(struct.pack('<BBHH', kind, value, len(a), len(b)) + a + b)
        for t in sorted(self.abbrev_types):
            rec(KIND_ABBREV, 0, t)
        for t in sorted(self.sent_starters):
            rec(KIND_STARTER, 0, t)
        for t, v in sorted(self.ortho_context.items()):
            if not 0 <= int(v) < 256:
                raise ValueError('ortho_context flags out of range: {}={}'.format(t, v))
            rec(KIND_ORTHO, int(v), t)
        for a, b in sorted(self.collocations):
            rec(KIND_COLLOC, 0, a, b)
        return b''.join(out)


def set_params(ctx, params=None):
    table = np.fromfile(os.path.join(ASSETS, 'punkt_props.bin'), np.uint8)
    blob = (params or PunktParams()).records()
    buf = np.frombuffer(blob, np.uint8) if blob else np.zeros(1, np.uint8)
    check(lib.lddl_punkt_set_params(ctx._h, table.ctypes.data, len(table), buf.ctypes.data,
                                    len(blob)))
    ctx._punkt_params = params


def segment(ctx, text, doc_off):
    """Sentence offsets of every document of a device batch.

    text: uint8 cuda tensor; doc_off: int64 cuda tensor [n_doc+1] (document d's text, after its
    id, is text[doc_off[d]:doc_off[d+1]], documents contiguous). Returns (sent_off int64[n_sent+1],
    doc_sent_off int64[n_doc+1]) in the layout lddl_tokenize / make_pairs consume.
    """
    import ctypes
    from .context import _ptr, _stream
    assert text.dtype == torch.uint8 and text.is_cuda and doc_off.dtype == torch.int64
    if not hasattr(ctx, '_punkt_params'):
        set_params(ctx)
    n_doc = doc_off.numel() - 1
    if n_doc > 0:  # kernels index documents with int32 offsets and read text[doc_off[0]:doc_off[-1]]
        lim = torch.stack([(doc_off[1:] - doc_off[:-1]).max(), doc_off[0], doc_off[-1]]).cpu()
        if int(lim[0]) >= 1 << 31 or int(lim[1]) < 0 or int(lim[2]) > text.numel():
            raise ValueError('documents must lie inside the text and be < 2 GiB each')
    n_sent = ctypes.c_int64()
    check(lib.lddl_segment_count(ctx._h, _stream(), _ptr(text), text.numel(), _ptr(doc_off), n_doc,
                                 ctypes.byref(n_sent)))
    filled = False
    try:
        sent_off = torch.empty(n_sent.value + 1, dtype=torch.int64, device=ctx.device)
        doc_sent_off = torch.empty(n_doc + 1, dtype=torch.int64, device=ctx.device)
        check(lib.lddl_segment_fill(ctx._h, _stream(), _ptr(sent_off), _ptr(doc_sent_off)))
        filled = True
    finally:
        if not filled:  # e.g. an allocation failed: cancel, so the context stays usable
            lib.lddl_segment_fill(ctx._h, _stream(), None, None)
    return sent_off, doc_sent_off


def utf8_first_invalid(text):
    """Offset of the first malformed UTF-8 byte of a uint8 cuda tensor, or -1 (lddl_utf8_check)."""
    from .context import _ptr, _stream
    out = torch.empty(1, dtype=torch.int64, device=text.device)
    check(lib.lddl_utf8_check(_stream(), _ptr(text), text.numel(), _ptr(out)))
    v = int(out.item())
    return -1 if v >= text.numel() else v


def stripped_sentences(text, sent_off, doc_sent_off):
    """Host helper (tests, debugging): the sentences as the reference sees them, per document:
    decoded, strip()ped, empty ones dropped (pretrain.py:86-88)."""
    text = bytes(np.asarray(text, np.uint8))
    so, ds = np.asarray(sent_off), np.asarray(doc_sent_off)
    out = []
    for d in range(len(ds) - 1):
        ss = (text[so[k]:so[k + 1]].decode('utf-8').strip() for k in range(ds[d], ds[d + 1]))
        out.append([s for s in ss if s])
    return out
