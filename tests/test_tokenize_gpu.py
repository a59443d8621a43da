"""GPU tokenizer parity: lddl_tokenize (HIP) vs the reference goldens and the oracle."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, VOCAB_CASED, VOCAB_UNCASED

pytestmark = pytest.mark.gpu


def load(name):
    with np.load(os.path.join(GOLDEN, name)) as z:
        return dict(z)


@pytest.fixture(scope='module')
def ctxs():
    from lddl_amd.context import Context
    return {'uncased': Context(VOCAB_UNCASED, True), 'cased': Context(VOCAB_CASED, False)}


@pytest.mark.parametrize('case', ['uncased', 'cased'])
def test_tokenize_golden_gpu(case, ctxs):
    g = load('tokenize.npz')
    ids, off = ctxs[case].tokenize_host(g['text'], g['sent_off'])
    exp, exp_off = g['ids_' + case], g['off_' + case]
    np.testing.assert_array_equal(off, exp_off)
    np.testing.assert_array_equal(ids, exp)


@pytest.mark.parametrize('case', ['uncased', 'cased'])
def test_tokenize_documents_gpu(case, ctxs):
    g = load('documents_{}.npz'.format(case))
    ids, off = ctxs[case].tokenize_host(g['text'], g['sent_off'])
    lens = np.diff(off)
    kept = np.concatenate([ids[off[i]:off[i + 1]] for i in range(len(lens)) if lens[i] > 0])
    np.testing.assert_array_equal(kept, g['ids'])


def test_tokenize_synthetic_vs_oracle(ctxs):
    from lddl_amd import synth
    from oracle import oracle as O
    corp = synth.generate(seed=31337, n_bytes=4 << 20, nonascii_frac=0.05)
    ids, off = ctxs['uncased'].tokenize_host(corp.text, corp.sent_off)
    tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
    e_ids, e_off = tok.tokenize(corp.text, corp.sent_off)
    np.testing.assert_array_equal(off, e_off)
    np.testing.assert_array_equal(ids, e_ids)


def test_tokenize_max_pieces_gpu(ctxs):
    """Truncation to max_pieces (4.16.2 truncation=True), including mid-word cuts."""
    s = ' '.join(['strommeth'] * 300) + ' ' + 'x' * 150
    text = np.frombuffer(s.encode(), np.uint8)
    off = np.asarray([0, len(text)], np.int64)
    from oracle import oracle as O
    tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
    for mp in (1, 7, 128, 511, 512, 513, 4096):
        ids, o = ctxs['uncased'].tokenize_host(text, off, max_pieces=mp)
        e, eo = tok.tokenize(text, off, max_pieces=mp)
        np.testing.assert_array_equal(ids, e)
