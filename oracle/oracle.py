"""ctypes binding of the oracle (oracle/_build/liblddl_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the lddl_amd package.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, '_build', 'liblddl_oracle.so')
ASSETS = os.path.join(os.path.dirname(HERE), 'lddl_amd', 'assets')

P = ctypes.c_void_p
i64, i32, u32, dbl = ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_double


class PairParams(ctypes.Structure):
    _fields_ = [('dup', i32), ('seq', i32), ('masking', i32), ('vocab_size', i32),
                ('cls_id', i32), ('sep_id', i32), ('mask_id', i32),
                ('short_seq_prob', dbl), ('masked_lm_ratio', dbl)]


def _load():
    if not os.path.exists(LIB_PATH):
        from lddl_amd.build import build_oracle
        build_oracle()
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        'orc_mt_seed_i64': (None, [P, i64]),
        'orc_mt_u32': (u32, [P]),
        'orc_mt_random': (dbl, [P]),
        'orc_mt_randint': (i64, [P, i64, i64]),
        'orc_mt_shuffle_i32': (None, [P, P, i64]),
        'orc_mt_get_state': (None, [P, P]),
        'orc_tok_create': (P, [P, i64, P, i64]),
        'orc_tok_destroy': (None, [P]),
        'orc_tok_vocab_size': (i32, [P]),
        'orc_tok_token_id': (i32, [P, ctypes.c_char_p, i32]),
        'orc_tokenize': (i64, [P, P, P, i64, i32, P, i64, P]),
        'orc_partition_pairs': (i64, [ctypes.POINTER(PairParams), i64, P, i64, P, P, P, i64, P, P,
                                      P, i64, P, P, i64, P]),
        'orc_partition_pairs_native': (i64, [ctypes.POINTER(PairParams), ctypes.c_uint64, i64, P,
                                             i64, P, P, P, i64, P, P, P, i64, P, P, i64, P]),
        'orc_bin': (None, [P, i64, i32, i32, P, P, P]),
        'orc_punkt_create': (P, [P, i64, P, i64]),
        'orc_punkt_destroy': (None, [P]),
        'orc_punkt_spans': (i64, [P, P, P, i64, P, P, P]),
    }
    for k, (r, a) in sig.items():
        f = getattr(lib, k)
        f.restype = r
        f.argtypes = a
    return lib


lib = _load()


def _p(a):
    return a.ctypes.data if a is not None else None


class MT:
    """CPython `random.Random` restated (seeded like random.seed(int))."""

    def __init__(self, seed):
        self._buf = ctypes.create_string_buffer(625 * 4 + 8)
        lib.orc_mt_seed_i64(self._buf, seed)

    def u32(self):
        return lib.orc_mt_u32(self._buf)

    def random(self):
        return lib.orc_mt_random(self._buf)

    def randint(self, a, b):
        return lib.orc_mt_randint(self._buf, a, b)

    def shuffle(self, x):
        a = np.ascontiguousarray(x, np.int32)
        lib.orc_mt_shuffle_i32(self._buf, _p(a), len(a))
        return a

    def state(self):
        st = np.zeros(625, np.uint32)
        lib.orc_mt_get_state(self._buf, _p(st))
        return st


class Tokenizer:
    def __init__(self, vocab_file, lowercase=True):
        name = 'uncased' if lowercase else 'cased'
        self._table = np.fromfile(os.path.join(ASSETS, 'bert_norm_{}.bin'.format(name)), np.uint8)
        self._vocab = np.fromfile(vocab_file, np.uint8)
        self._h = lib.orc_tok_create(_p(self._table), len(self._table), _p(self._vocab),
                                     len(self._vocab))
        if not self._h:
            raise RuntimeError('bad tokenizer tables')
        self.vocab_size = lib.orc_tok_vocab_size(self._h)

    def __del__(self):
        if getattr(self, '_h', None):
            lib.orc_tok_destroy(self._h)

    def token_id(self, s):
        b = s.encode()
        return lib.orc_tok_token_id(self._h, b, len(b))

    def tokenize(self, text, sent_off, max_pieces=512):
        text = np.ascontiguousarray(text, np.uint8)
        sent_off = np.ascontiguousarray(sent_off, np.int64)
        n = len(sent_off) - 1
        cap = max(64, len(text) + 16)
        ids = np.empty(cap, np.int32)
        off = np.empty(n + 1, np.int64)
        total = lib.orc_tokenize(self._h, _p(text), _p(sent_off), n, max_pieces, _p(ids), cap,
                                 _p(off))
        assert total >= 0
        return ids[:total], off


def partition_pairs(doc_sent, tok_off, ids, seed, dup, seq, masking, vocab_size, cls_id, sep_id,
                    mask_id, short_seq_prob=0.1, masked_lm_ratio=0.15):
    """One partition through the reference algorithm; returns a dict of numpy arrays."""
    doc_sent = np.ascontiguousarray(doc_sent, np.int64)
    tok_off = np.ascontiguousarray(tok_off, np.int64)
    ids = np.ascontiguousarray(ids, np.int32)
    n_docs = len(doc_sent) - 1
    n_sent = int(doc_sent[-1] - doc_sent[0])
    pp = PairParams(dup, seq, int(masking), vocab_size, cls_id, sep_id, mask_id, short_seq_prob,
                    masked_lm_ratio)
    pair_cap = dup * max(n_sent, 1) + 16
    tok_cap = pair_cap * (seq - 3)
    pos_cap = pair_cap * seq if masking else 0
    out_tok = np.empty(tok_cap, np.int32)
    out_off = np.empty(pair_cap + 1, np.int64)
    len_a = np.empty(pair_cap, np.int32)
    is_rn = np.empty(pair_cap, np.uint8)
    pos = np.empty(max(pos_cap, 1), np.uint16)
    lab = np.empty(max(pos_cap, 1), np.int32)
    pos_off = np.empty(pair_cap + 1, np.int64)
    n = lib.orc_partition_pairs(ctypes.byref(pp), seed, _p(doc_sent), n_docs, _p(tok_off), _p(ids),
                                _p(out_tok), tok_cap, _p(out_off), _p(len_a), _p(is_rn), pair_cap,
                                _p(pos), _p(lab), pos_cap, _p(pos_off) if masking else None)
    assert n >= 0
    out = dict(tokens=out_tok[:out_off[n]].copy(), tok_off=out_off[:n + 1].copy(),
               len_a=len_a[:n].copy(), is_random_next=is_rn[:n].astype(bool))
    out['num_tokens'] = np.diff(out['tok_off']) + 3
    if masking:
        out['pos'] = pos[:pos_off[n]].copy()
        out['labels'] = lab[:pos_off[n]].copy()
        out['pos_off'] = pos_off[:n + 1].copy()
    return out


def partition_pairs_native(doc_sent, tok_off, ids, native_seed, part_seed, dup, seq, masking,
                           vocab_size, cls_id, sep_id, mask_id, short_seq_prob=0.1,
                           masked_lm_ratio=0.15):
    """One partition through lddl_amd's native-RNG mode (oracle/native_oracle.c): the reference's
    algorithm on Philox streams keyed by (native_seed, part_seed); a dict as partition_pairs."""
    doc_sent = np.ascontiguousarray(doc_sent, np.int64)
    tok_off = np.ascontiguousarray(tok_off, np.int64)
    ids = np.ascontiguousarray(ids, np.int32)
    n_docs = len(doc_sent) - 1
    n_sent = int(doc_sent[-1] - doc_sent[0])
    pp = PairParams(dup, seq, int(masking), vocab_size, cls_id, sep_id, mask_id, short_seq_prob,
                    masked_lm_ratio)
    pair_cap = dup * max(n_sent, 1) + 16
    tok_cap = pair_cap * (seq - 3)
    pos_cap = pair_cap * seq if masking else 0
    out_tok = np.empty(tok_cap, np.int32)
    out_off = np.empty(pair_cap + 1, np.int64)
    len_a = np.empty(pair_cap, np.int32)
    is_rn = np.empty(pair_cap, np.uint8)
    pos = np.empty(max(pos_cap, 1), np.uint16)
    lab = np.empty(max(pos_cap, 1), np.int32)
    pos_off = np.empty(pair_cap + 1, np.int64)
    n = lib.orc_partition_pairs_native(
        ctypes.byref(pp), native_seed & ((1 << 64) - 1), part_seed, _p(doc_sent), n_docs,
        _p(tok_off), _p(ids), _p(out_tok), tok_cap, _p(out_off), _p(len_a), _p(is_rn), pair_cap,
        _p(pos), _p(lab), pos_cap, _p(pos_off) if masking else None)
    assert n >= 0
    out = dict(tokens=out_tok[:out_off[n]].copy(), tok_off=out_off[:n + 1].copy(),
               len_a=len_a[:n].copy(), is_random_next=is_rn[:n].astype(bool))
    out['num_tokens'] = np.diff(out['tok_off']) + 3
    if masking:
        out['pos'] = pos[:pos_off[n]].copy()
        out['labels'] = lab[:pos_off[n]].copy()
        out['pos_off'] = pos_off[:n + 1].copy()
    return out


def bin_samples(num_tokens, bin_size, nbins):
    nt = np.ascontiguousarray(num_tokens, np.int32)
    n = len(nt)
    bin_id = np.empty(n, np.int32)
    order = np.empty(n, np.int64)
    counts = np.empty(nbins, np.int64)
    lib.orc_bin(_p(nt), n, bin_size, nbins, _p(bin_id), _p(order), _p(counts))
    return bin_id, order, counts


def punkt_params_blob(params):
    """Records of a Punkt parameter dict {abbrev_types, sent_starters, ortho_context,
    collocations} in the oracle's layout (lddl_oracle.h)."""
    import struct
    out = []

    def rec(kind, value, a, b=''):
        a, b = a.encode('utf-8'), b.encode('utf-8')
        out.append(struct.pack('<BBHH', kind, value, len(a), len(b)) + a + b)
    for t in (params or {}).get('abbrev_types', []):
        rec(1, 0, t)
    for t in (params or {}).get('sent_starters', []):
        rec(2, 0, t)
    for t, v in (params or {}).get('ortho_context', {}).items():
        rec(3, int(v), t)
    for a, b in (params or {}).get('collocations', []):
        rec(4, 0, a, b)
    return b''.join(out)


class Punkt:
    """nltk PunktSentenceTokenizer(params) spans, per document (byte offsets)."""

    def __init__(self, params=None):
        table = np.fromfile(os.path.join(ASSETS, 'punkt_props.bin'), np.uint8)
        blob = np.frombuffer(punkt_params_blob(params) or b'\0', np.uint8)
        self._keep = (table, blob)
        self.h = lib.orc_punkt_create(_p(table), len(table), _p(blob),
                                      len(punkt_params_blob(params)))
        assert self.h

    def __del__(self):
        if getattr(self, 'h', None):
            lib.orc_punkt_destroy(self.h)

    def spans(self, text, doc_off):
        text = np.ascontiguousarray(text, np.uint8)
        doc_off = np.ascontiguousarray(doc_off, np.int64)
        n_doc = len(doc_off) - 1
        cap = int(doc_off[-1] - doc_off[0]) + n_doc + 1
        st = np.empty(cap, np.int64)
        en = np.empty(cap, np.int64)
        cnt = np.empty(max(n_doc, 1), np.int64)
        n = lib.orc_punkt_spans(self.h, _p(text), _p(doc_off), n_doc, _p(st), _p(en), _p(cnt))
        return st[:n].copy(), en[:n].copy(), cnt[:n_doc].copy()
