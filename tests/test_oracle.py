"""Pin the oracle (CPU restatement) against the reference-generated golden fixtures.

Every fixture in tests/golden/ was produced by tests/golden/make_goldens.py from the reference's
own functions (see that file's header). If these pass, the oracle is a faithful checker for the
GPU path.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, VOCAB_CASED, VOCAB_UNCASED
from oracle import oracle as O


def load(name):
    with np.load(os.path.join(GOLDEN, name)) as z:  # NpzFile decompresses on every access
        return dict(z)


@pytest.fixture(scope='module')
def tok_u():
    return O.Tokenizer(VOCAB_UNCASED, lowercase=True)


@pytest.fixture(scope='module')
def tok_c():
    return O.Tokenizer(VOCAB_CASED, lowercase=False)


def test_mt19937_stream():
    for rec in json.load(open(os.path.join(GOLDEN, 'mt19937.json'))):
        seed = int(rec['seed'])
        if seed >= 2 ** 63:
            continue
        m = O.MT(seed)
        assert list(m.state()[:8]) == rec['state_head']
        assert [m.u32() for _ in range(64)] == rec['u32']
        assert [m.random().hex() for _ in range(32)] == rec['random_hex']
        assert [m.randint(a, b) for a, b, _ in rec['randint']] == [v for _, _, v in rec['randint']]
        assert m.shuffle(np.arange(50)).tolist() == rec['shuffle50']


@pytest.mark.parametrize('case', ['uncased', 'cased'])
def test_tokenize_golden(case, tok_u, tok_c):
    g = load('tokenize.npz')
    tok = tok_u if case == 'uncased' else tok_c
    ids, off = tok.tokenize(g['text'], g['sent_off'])
    exp, exp_off = g['ids_' + case], g['off_' + case]
    bad = [i for i in range(len(off) - 1)
           if not np.array_equal(ids[off[i]:off[i + 1]], exp[exp_off[i]:exp_off[i + 1]])]
    assert not bad, 'mismatching sentences: {}'.format(bad[:10])


@pytest.mark.parametrize('case', ['uncased', 'cased'])
def test_documents_golden(case, tok_u, tok_c):
    """_get_documents (pretrain.py:77-97): drop sentences with no pieces, then empty docs."""
    g = load('documents_{}.npz'.format(case))
    tok = tok_u if case == 'uncased' else tok_c
    ids, off = tok.tokenize(g['text'], g['sent_off'])
    lens = np.diff(off)
    keep_sent = lens > 0
    line_off = g['line_sent_off']
    doc_nsent = np.asarray([keep_sent[line_off[i]:line_off[i + 1]].sum()
                            for i in range(len(line_off) - 1)])
    np.testing.assert_array_equal(doc_nsent[doc_nsent > 0], g['doc_nsent'])
    kept = [ids[off[i]:off[i + 1]] for i in range(len(lens)) if keep_sent[i]]
    flat = np.concatenate(kept)
    np.testing.assert_array_equal(flat, g['ids'])
    np.testing.assert_array_equal(np.cumsum([0] + [len(k) for k in kept]), g['ids_off'])


def golden_documents():
    g = load('documents_uncased.npz')
    return np.concatenate([[0], np.cumsum(g['doc_nsent'])]), g['ids_off'], g['ids']


PAIR_CASES = ['s128_mask', 's128_nomask', 's512_mask', 's512_nomask_short', 's64_mask_ratio']


@pytest.mark.parametrize('name', PAIR_CASES)
def test_pairs_golden(name, tok_u):
    g = load('pairs_{}.npz'.format(name))
    doc_sent, tok_off, ids = golden_documents()
    dup, seq, masking = g['params'].tolist()
    cls_id, sep_id, mask_id = (tok_u.token_id(t) for t in ('[CLS]', '[SEP]', '[MASK]'))
    d0 = 0
    for p, ndoc in enumerate(g['part_doc_sizes']):
        ds = doc_sent[d0:d0 + ndoc + 1]
        out = O.partition_pairs(ds, tok_off, ids, int(g['seeds'][p]), dup, seq, masking,
                                tok_u.vocab_size, cls_id, sep_id, mask_id,
                                float(g['short_seq_prob']), float(g['ratio']))
        q0, q1 = g['part_pair_off'][p], g['part_pair_off'][p + 1]
        assert len(out['len_a']) == q1 - q0
        np.testing.assert_array_equal(out['is_random_next'], g['is_random_next'][q0:q1])
        np.testing.assert_array_equal(out['num_tokens'], g['num_tokens'][q0:q1])
        for k in range(q1 - q0):
            a = g['a'][g['a_off'][q0 + k]:g['a_off'][q0 + k + 1]]
            b = g['b'][g['b_off'][q0 + k]:g['b_off'][q0 + k + 1]]
            t = out['tokens'][out['tok_off'][k]:out['tok_off'][k + 1]]
            assert out['len_a'][k] == len(a)
            np.testing.assert_array_equal(t, np.concatenate([a, b]))
            if masking:
                pe = g['pos'][g['pos_off'][q0 + k]:g['pos_off'][q0 + k + 1]]
                le = g['labels'][g['labels_off'][q0 + k]:g['labels_off'][q0 + k + 1]]
                sl = slice(out['pos_off'][k], out['pos_off'][k + 1])
                np.testing.assert_array_equal(out['pos'][sl], pe)
                np.testing.assert_array_equal(out['labels'][sl], le)
        d0 += ndoc


def test_binning_golden():
    for c in json.load(open(os.path.join(GOLDEN, 'binning.json'))):
        nbins = c['seq'] // c['bin_size']
        bin_id, order, counts = O.bin_samples(c['num_tokens'], c['bin_size'], nbins)
        assert order.tolist() == c['uid_order']
        assert bin_id[order].tolist() == c['bin_id']
