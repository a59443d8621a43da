"""NSP pairs + static masking on the GPU — the device-resident replacement of
`_to_partition_pairs` / `create_pairs_from_document` / `create_masked_lm_predictions`
(lddl/dask/bert/pretrain.py:386-402, 241-365, 182-238).
"""
import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from ._native import lib, check, PairParams, RNG_REPLAY, RNG_NATIVE
from .context import _ptr, _stream


def _ids(t):
    """Host copy of an id tensor: int16 storage holds uint16 ids."""
    a = t.cpu().numpy()
    return a.view(np.uint16) if a.dtype == np.int16 else a


@dataclass
class PairBatch:
    """Pairs of one batch of partitions, in output order (partition order, then the reference's
    per-partition shuffle). Pair q: tokens[tok_off[q]:tok_off[q]+len_a[q]] is A (after masking),
    the rest up to tok_off[q+1] is B. With static masking, pos[pos_off[q]:pos_off[q+1]] are the
    masked positions in [CLS] A [SEP] B [SEP] coordinates (sorted) and labels the original ids.
    Token ids and labels are uint16 held in int16 tensors when the vocab fits (ctx.id_dtype),
    else int32; to_host() returns them as uint16 / int32 numpy arrays."""
    tokens: torch.Tensor
    tok_off: torch.Tensor
    len_a: torch.Tensor
    is_random_next: torch.Tensor
    pos: torch.Tensor = None      # int16 storage of uint16 positions
    labels: torch.Tensor = None
    pos_off: torch.Tensor = None
    n_kept_sentences: int = 0
    n_kept_documents: int = 0
    part_off: torch.Tensor = None  # int64 [n_part + 1]: pair range of each partition
    plan_ms: float = 0.0           # device time of the planner kernel (HIP events)
    n_masked: int = 0

    @property
    def n_pairs(self):
        return self.len_a.numel()

    @property
    def num_tokens(self):
        """len(A) + len(B) + 3 per pair (pretrain.py:352)."""
        return (self.tok_off[1:] - self.tok_off[:-1]) + 3

    def to_host(self):
        out = dict(tokens=_ids(self.tokens), tok_off=self.tok_off.cpu().numpy(),
                   len_a=self.len_a.cpu().numpy(),
                   is_random_next=self.is_random_next.cpu().numpy().astype(bool))
        out['num_tokens'] = np.diff(out['tok_off']) + 3
        if self.part_off is not None:
            out['part_off'] = self.part_off.cpu().numpy()
        if self.pos is not None:
            out['pos'] = self.pos.cpu().numpy().view(np.uint16)
            out['labels'] = _ids(self.labels)
            out['pos_off'] = self.pos_off.cpu().numpy()
        return out


def make_pairs(ctx, sent_off, ids, sent_len, doc_sent_off, part_doc_off, part_seed, seq=128,
               dup=5, masking=False, short_seq_prob=0.1, masked_lm_ratio=0.15, rng='replay',
               native_seed=12345):
    """All inputs are cuda tensors (int64 offsets / seeds; tokenizer output from Context.tokenize).

    rng='replay' reproduces CPython `random` after random.seed(part_seed[p]) per partition.
    """
    dev = ctx.device
    prm = PairParams(seq, dup, int(bool(masking)), RNG_REPLAY if rng == 'replay' else RNG_NATIVE,
                     short_seq_prob, masked_lm_ratio, native_seed)
    n_sent = sent_off.numel() - 1
    n_doc = doc_sent_off.numel() - 1
    n_part = part_doc_off.numel() - 1
    h = ctypes.c_void_p()
    counts = np.zeros(5, np.int64)
    st = _stream()
    check(lib.lddl_pairs_plan(ctx.handle, st, ctypes.byref(prm), _ptr(sent_off), _ptr(ids),
                              _ptr(sent_len), n_sent, _ptr(doc_sent_off), n_doc, _ptr(part_doc_off),
                              _ptr(part_seed), n_part, ctypes.byref(h), counts.ctypes.data))
    try:
        n_pairs, n_tok, n_mask = int(counts[0]), int(counts[1]), int(counts[2])
        tokens = torch.empty(max(n_tok, 1), dtype=ctx.id_dtype, device=dev)[:n_tok]
        tok_off = torch.empty(n_pairs + 1, dtype=torch.int64, device=dev)
        len_a = torch.empty(n_pairs, dtype=torch.int32, device=dev)
        is_rn = torch.empty(n_pairs, dtype=torch.uint8, device=dev)
        pos = labels = pos_off = None
        if masking:
            pos = torch.empty(max(n_mask, 1), dtype=torch.int16, device=dev)[:n_mask]
            labels = torch.empty(max(n_mask, 1), dtype=ctx.id_dtype, device=dev)[:n_mask]
            pos_off = torch.empty(n_pairs + 1, dtype=torch.int64, device=dev)
        check(lib.lddl_pairs_emit(h, st, _ptr(tokens), _ptr(tok_off), _ptr(len_a), _ptr(is_rn),
                                  _ptr(pos), _ptr(labels), _ptr(pos_off)))
        part_off = torch.empty(n_part + 1, dtype=torch.int64, device=dev)
        check(lib.lddl_pairs_part_offsets(h, st, _ptr(part_off)))
        ms = ctypes.c_float()
        check(lib.lddl_pairs_plan_ms(h, ctypes.byref(ms)))
    finally:
        lib.lddl_pairs_destroy(h, st)
    return PairBatch(tokens, tok_off, len_a, is_rn, pos, labels, pos_off, int(counts[3]),
                     int(counts[4]), part_off, float(ms.value), n_mask)


_SIDE = {}


def _side_stream(dev):
    """One persistent side stream per device: the caching allocator keeps per-stream pools, so
    a fresh stream per call would never reuse the previous call's blocks."""
    key = torch.device(dev).index
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


def tokenize_and_pair_chunked(ctx, text, sent_off, doc_sent_off, part_doc_off, part_seed,
                              n_chunks=2, max_pieces=512, tok_stream=None, **pair_kw):
    """tokenize + make_pairs over `n_chunks` partition-aligned chunks, pipelined on two streams:
    every chunk's tokenizer is queued on a side stream, each chunk's pair planner on the current
    stream waits only for its own chunk's tokens, so chunk k+1 is tokenized while chunk k is
    planned and gathered. Partitions are independent (per-partition seeds), so the result is
    bit-identical to one call over all partitions. Returns the chunks' PairBatch list in
    partition order."""
    n_part = part_doc_off.numel() - 1
    cuts = [round(k * n_part / n_chunks) for k in range(n_chunks + 1)]
    pc = torch.tensor(cuts, dtype=torch.int64, device=part_doc_off.device)
    d_cut = part_doc_off.index_select(0, pc)
    s_cut = doc_sent_off.index_select(0, d_cut)
    b_cut = sent_off.index_select(0, s_cut)
    d_cut, s_cut, b_cut = d_cut.tolist(), s_cut.tolist(), b_cut.tolist()
    main = torch.cuda.current_stream()
    side = tok_stream or _side_stream(text.device)
    side.wait_stream(main)
    toks = []
    with torch.cuda.stream(side):
        for k in range(n_chunks):
            t = text[b_cut[k]:b_cut[k + 1]]
            so = sent_off[s_cut[k]:s_cut[k + 1] + 1] - b_cut[k]
            ids, sl = ctx.tokenize(t, so, max_pieces)
            ev = torch.cuda.Event()
            ev.record(side)
            toks.append((so, ids, sl, ev))
    out = []
    for k, (so, ids, sl, ev) in enumerate(toks):
        main.wait_event(ev)
        for x in (so, ids, sl):
            x.record_stream(main)
        pb = make_pairs(ctx, so, ids, sl, doc_sent_off[d_cut[k]:d_cut[k + 1] + 1] - s_cut[k],
                        part_doc_off[cuts[k]:cuts[k + 1] + 1] - d_cut[k],
                        part_seed[cuts[k]:cuts[k + 1]], **pair_kw)
        del ids
        out.append(pb)
    return out
