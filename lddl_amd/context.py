"""Device context: the GPU-resident equivalent of `transformers.BertTokenizerFast(vocab_file)`
as the reference builds it (lddl/dask/bert/pretrain.py:584-587, lddl/torch/bert.py:343-346).

All device buffers are torch.cuda tensors; kernels run on torch's current stream.
"""
import ctypes
import os

import numpy as np
import torch

from ._native import lib, check

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'assets')
SPECIALS = ('[PAD]', '[UNK]', '[CLS]', '[SEP]', '[MASK]')
LEN_HAS_CLS_SEP = 1 << 30
LEN_MASK = (1 << 30) - 1


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# The library's temporaries come from PyTorch's caching allocator (lddl_ctx_set_allocator), so
# one pool owns HBM: no second cache of hipMalloc blocks beside torch's. `user` carries the
# device index. LDDL_ARENA=own keeps the library's own block cache instead (A/B only).
_ALLOC_FN = ctypes.CFUNCTYPE(ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p)
_FREE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p)


def _torch_alloc(nbytes, stream, user):
    try:
        return torch.cuda.caching_allocator_alloc(int(nbytes), device=int(user or 0),
                                                  stream=int(stream or 0))
    except Exception:  # out of memory: the library reports hipErrorOutOfMemory
        return None


def _torch_free(p, stream, user):
    torch.cuda.caching_allocator_delete(int(p))


_TORCH_ALLOC, _TORCH_FREE = _ALLOC_FN(_torch_alloc), _FREE_FN(_torch_free)


class Context:
    """Tokenizer tables resident in HBM.

    do_lower_case follows BertTokenizerFast's default (True), which the reference keeps even for
    cased vocabularies.
    """

    def __init__(self, vocab_file, do_lower_case=True, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError('lddl_amd needs a ROCm GPU; there is no CPU fallback')
        self.device = torch.device('cuda', torch.cuda.current_device() if device is None else device)
        name = 'uncased' if do_lower_case else 'cased'
        table = np.fromfile(os.path.join(ASSETS, 'bert_norm_{}.bin'.format(name)), np.uint8)
        with open(vocab_file, 'rb') as f:
            vocab = f.read()
        self.tokens = vocab.decode('utf-8').split('\n')
        if self.tokens and self.tokens[-1] == '':
            self.tokens.pop()
        self.vocab = {}
        for i, t in enumerate(self.tokens):
            self.vocab[t.rstrip('\r')] = i
        h = ctypes.c_void_p()
        check(lib.lddl_ctx_create(self.device.index, table.ctypes.data, len(table), vocab,
                                  len(vocab), ctypes.byref(h)))
        self._h = h
        if os.environ.get('LDDL_ARENA') != 'own':
            check(lib.lddl_ctx_set_allocator(h, _TORCH_ALLOC, _TORCH_FREE,
                                             ctypes.c_void_p(self.device.index)))
        vs = ctypes.c_int32()
        sp = (ctypes.c_int32 * 5)()
        mp = ctypes.c_int32()
        check(lib.lddl_ctx_info(h, ctypes.byref(vs), sp, ctypes.byref(mp)))
        self.vocab_size = vs.value
        self.special_ids = dict(zip(SPECIALS, list(sp)))
        self.max_piece_bytes = mp.value
        # token ids of the pair tables (PairBatch.tokens / labels): uint16 when the vocab fits
        # (held in int16 tensors), else int32 (lddl_ctx_id_bytes)
        self.id_bytes = lib.lddl_ctx_id_bytes(h)
        self.id_dtype = torch.int16 if self.id_bytes == 2 else torch.int32

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, '_h', None):
            lib.lddl_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.vocab_size

    # ---- the tokenizer duck-type the reference's hot path uses -----------------
    # pretrain.py:79-80, 384; lddl/torch/bert.py:111, 123, 169-171, 185-186, 191
    mask_token = '[MASK]'
    cls_token = '[CLS]'
    sep_token = '[SEP]'
    pad_token = '[PAD]'
    unk_token = '[UNK]'

    @property
    def all_special_tokens(self):
        return [t for t in ('[UNK]', '[SEP]', '[PAD]', '[CLS]', '[MASK]') if self.special_ids[t] >= 0]

    @property
    def all_special_ids(self):
        return [self.special_ids[t] for t in self.all_special_tokens]

    def convert_tokens_to_ids(self, tokens):
        """A token -> its id, a list of tokens -> list of ids ([UNK] for unknown tokens)."""
        unk = self.special_ids['[UNK]']
        if isinstance(tokens, str):
            return self.vocab.get(tokens, unk)
        return [self.vocab.get(t, unk) for t in tokens]

    def convert_ids_to_tokens(self, ids):
        if isinstance(ids, int):
            return self.tokens[ids]
        return [self.tokens[int(i)] for i in ids]

    def get_special_tokens_mask(self, token_ids_0, token_ids_1=None,
                                already_has_special_tokens=False):
        """BertTokenizerFast.get_special_tokens_mask: with already_has_special_tokens, 1 for
        every id in all_special_ids; else the [CLS] A [SEP] (B [SEP]) layout."""
        if already_has_special_tokens:
            if token_ids_1 is not None:
                raise ValueError('You should not supply a second sequence if the provided '
                                 'sequence of ids is already formatted with special tokens '
                                 'for the model.')
            sp = set(self.all_special_ids)
            return [1 if int(t) in sp else 0 for t in token_ids_0]
        out = [1] + [0] * len(token_ids_0) + [1]
        if token_ids_1 is not None:
            out += [0] * len(token_ids_1) + [1]
        return out

    # ------------------------------------------------------------------------------------------
    def tokenize(self, text, sent_off=None, max_pieces=512, max_length=None, truncation=False):
        """Two forms.

        tokenize(str, max_length=None, truncation=False) -> list of WordPiece strings: the
        reference's per-sentence call `tokenizer.tokenize(s, max_length=512, truncation=True)`
        (pretrain.py:79-80), as a host convenience over the same GPU kernel.

        tokenize(text, sent_off, max_pieces=512): WordPiece-tokenize device-resident sentences
        (the product path). text: uint8 cuda tensor; sent_off: int64 cuda tensor [n_sent+1].
        Returns (ids int32[n_bytes], sent_len int32[n_sent]): sentence s's pieces are
        ids[sent_off[s] : sent_off[s] + (sent_len[s] & LEN_MASK)].
        """
        if isinstance(text, str):
            return self._tokenize_str(text, max_length if truncation and max_length else None)
        assert text.dtype == torch.uint8 and text.is_cuda and sent_off.dtype == torch.int64
        n_sent = sent_off.numel() - 1
        ids = torch.empty(max(text.numel(), 1), dtype=torch.int32, device=self.device)
        sent_len = torch.empty(max(n_sent, 0), dtype=torch.int32, device=self.device)
        check(lib.lddl_tokenize(self._h, _stream(), _ptr(text), text.numel(), _ptr(sent_off),
                                n_sent, max_pieces, _ptr(ids), _ptr(sent_len)))
        return ids, sent_len

    def _tokenize_str(self, s, max_length=None):
        b = np.array(bytearray(s.encode('utf-8')), np.uint8)
        if len(b) == 0:
            return []
        cap = min(len(b), 1 << 24) if max_length is None else int(max_length)
        ids, off = self.tokenize_host(b, np.asarray([0, len(b)], np.int64), cap)
        return [self.tokens[i] for i in ids[off[0]:off[1]]]

    def tokenize_host(self, text, sent_off, max_pieces=512):
        """Convenience: numpy in, ragged numpy (ids, offsets) out."""
        t = torch.from_numpy(np.ascontiguousarray(text, np.uint8)).to(self.device)
        o = torch.from_numpy(np.ascontiguousarray(sent_off, np.int64)).to(self.device)
        ids, sl = self.tokenize(t, o, max_pieces)
        ids, sl = ids.cpu().numpy(), (sl.cpu().numpy() & LEN_MASK).astype(np.int64)
        so = np.asarray(sent_off, np.int64)
        out_off = np.zeros(len(sl) + 1, np.int64)
        out_off[1:] = np.cumsum(sl)
        flat = np.concatenate([ids[so[i]:so[i] + sl[i]] for i in range(len(sl))]) if len(sl) else \
            np.zeros(0, np.int32)
        return flat, out_off
