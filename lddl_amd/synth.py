"""Synthetic corpus — thin wrapper over lddl_synth_corpus in the C library.

A corpus here is already sentence-segmented (the hot path starts after Punkt,
lddl/dask/bert/pretrain.py:86): `text` holds every sentence's UTF-8 bytes back to back,
`sent_off[i]:sent_off[i+1]` is sentence i, `doc_sent_off[d]:doc_sent_off[d+1]` are the
sentences of document d.
"""
import ctypes
from dataclasses import dataclass

import numpy as np

from ._native import lib, check


@dataclass
class Corpus:
    text: np.ndarray          # uint8 [n_bytes]
    sent_off: np.ndarray      # int64 [n_sent + 1]
    doc_sent_off: np.ndarray  # int64 [n_doc + 1]

    @property
    def n_sent(self):
        return len(self.sent_off) - 1

    @property
    def n_doc(self):
        return len(self.doc_sent_off) - 1

    def sentence(self, i):
        return bytes(self.text[self.sent_off[i]:self.sent_off[i + 1]]).decode('utf-8')

    def documents(self):
        """List of documents, each a list of sentence strings."""
        b = self.text.tobytes()
        so = self.sent_off.tolist()
        out = []
        for d in range(self.n_doc):
            s0, s1 = self.doc_sent_off[d], self.doc_sent_off[d + 1]
            out.append([b[so[i]:so[i + 1]].decode('utf-8') for i in range(s0, s1)])
        return out


def generate(seed=1234, n_bytes=1 << 20, doc_begin=0, nonascii_frac=0.01, threads=8):
    cap = n_bytes + (1 << 20)
    text = np.empty(cap, np.uint8)
    so = np.empty(n_bytes // 16 + 4096, np.int64)
    do = np.empty(n_bytes // 64 + 1024, np.int64)
    ns, nd = ctypes.c_int64(), ctypes.c_int64()
    n = check(lib.lddl_synth_corpus(seed, doc_begin, n_bytes, nonascii_frac, text.ctypes.data, cap,
                                    so.ctypes.data, len(so), do.ctypes.data, len(do),
                                    ctypes.byref(ns), ctypes.byref(nd), threads))
    return Corpus(text[:n], so[:ns.value + 1].copy(), do[:nd.value + 1].copy())


def generate_doc_text(seed=1234, n_bytes=1 << 20, doc_begin=0, nonascii_frac=0.01, threads=8):
    """The documents of `generate` as raw text (sentences joined by one space): (text uint8,
    doc_off int64[n_doc+1]) -- the input of sentence segmentation."""
    cap = n_bytes + (1 << 20)
    text = np.empty(cap, np.uint8)
    do = np.empty(n_bytes // 64 + 1024, np.int64)
    nd = ctypes.c_int64()
    n = check(lib.lddl_synth_doc_text(seed, doc_begin, n_bytes, nonascii_frac, text.ctypes.data,
                                      cap, do.ctypes.data, len(do), ctypes.byref(nd), threads))
    return text[:n], do[:nd.value + 1].copy()


def from_documents(docs):
    """Build a Corpus from a list of documents (lists of sentence strings)."""
    chunks, so, do = [], [0], [0]
    for d in docs:
        for s in d:
            b = s.encode('utf-8')
            chunks.append(b)
            so.append(so[-1] + len(b))
        do.append(len(so) - 1)
    text = np.frombuffer(b''.join(chunks), np.uint8).copy()
    return Corpus(text, np.asarray(so, np.int64), np.asarray(do, np.int64))
