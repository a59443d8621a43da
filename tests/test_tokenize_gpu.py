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


def _adversarial_corpus(seed=7, n=6000):
    """Sentences built to hit every branch of the wave tokenizer: literal special tokens and
    multi-byte code points straddling 64-byte windows, invalid UTF-8, control chars inside words,
    words of 16/17/64/65/150/500 bytes, many-piece words, CJK, separator code points beyond ASCII,
    empty and whitespace-only sentences."""
    rng = np.random.default_rng(seed)
    frags = [b'the', b'Strommeth', b'[MASK]', b'[CLS]', b'[SEP]', b'[PAD]', b'[UNK]', b'[MAS', b'[[SEP]]',
             b'x[MASK]y', 'café'.encode(), 'ÉCOLE'.encode(), '中文'.encode(),
             '　'.encode(), ' '.encode(), ' '.encode(), b'\x01', b'ab\x00cd', b'\x7f',
             b'\xe2\x82', b'\xff', b'\xc3', b'\x80\x80', '𝐀'.encode('utf-8', 'surrogatepass'),
             '\U0001d400\U0001d401'.encode(), 'ﬃn'.encode(), 'İstanbul'.encode(),
             'ȺȺ'.encode(), b'1234567890123456789012345', b'a' * 16, b'b' * 17, b'c' * 63,
             b'd' * 64, b'e' * 65, b'f' * 150, b'g' * 500, ('hé' * 40).encode(), b'(', b')', b'...', b"don't", b'U.S.A.', b'\t', b'\n', b'  ',
             ('ß' * 30).encode(), ('ΑΒ' * 12).encode()]
    sents = []
    for _ in range(n):
        k = int(rng.integers(0, 24))
        parts = []
        for _ in range(k):
            f = frags[int(rng.integers(0, len(frags)))]
            sep = [b' ', b'', b'  ', b'-', b'\t'][int(rng.integers(0, 5))]
            parts.append(f + sep)
        sents.append(b''.join(parts))
    text = np.frombuffer(b''.join(sents), np.uint8).copy()
    off = np.zeros(len(sents) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in sents])
    return text, off


def _assert_same(ids, o, e, eo, text, off):
    """ids / offsets against the oracle's; on a difference, name the first sentence that differs
    (its text and both piece lists)."""
    if np.array_equal(o, eo) and np.array_equal(ids, e):
        return
    for k in range(len(off) - 1):
        a, b = ids[o[k]:o[k + 1]], e[eo[k]:eo[k + 1]]
        if not np.array_equal(a, b):
            raise AssertionError('sentence {} of {} ({!r}): got {} expected {}'.format(
                k, len(off) - 1, bytes(text[off[k]:off[k + 1]])[:300], a.tolist()[:60],
                b.tolist()[:60]))
    raise AssertionError('outputs differ')


@pytest.mark.parametrize('case', ['uncased', 'cased'])
def test_tokenize_adversarial_vs_oracle(case, ctxs):
    from oracle import oracle as O
    text, off = _adversarial_corpus()
    vocab = VOCAB_UNCASED if case == 'uncased' else VOCAB_CASED
    tok = O.Tokenizer(vocab, lowercase=case == 'uncased')
    for mp in (512, 9):
        ids, o = ctxs[case].tokenize_host(text, off, max_pieces=mp)
        e, eo = tok.tokenize(text, off, max_pieces=mp)
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(ids, e)


@pytest.mark.parametrize('path', ['lane', 'wave', 'fused', 'plain'])
def test_tokenize_paths_vs_oracle(ctxs, monkeypatch, path):
    """Every LDDL_TOKENIZE_PATH (the lane kernel alone, the unbatched wave kernel, the streaming
    kernel by name and without the word memo) against the oracle, on the synthetic corpus and on
    the adversarial one."""
    from lddl_amd import synth
    from oracle import oracle as O
    tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
    corp = synth.generate(seed=99, n_bytes=1 << 20, nonascii_frac=0.05)
    monkeypatch.setenv('LDDL_TOKENIZE_PATH', path)
    for text, off in ((corp.text, corp.sent_off), _adversarial_corpus(seed=21, n=3000)):
        ids, o = ctxs['uncased'].tokenize_host(text, off)
        e, eo = tok.tokenize(text, off)
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(ids, e)


def test_tokenize_path_unknown_raises(ctxs, monkeypatch):
    monkeypatch.setenv('LDDL_TOKENIZE_PATH', 'cp')
    text = np.frombuffer(b'hello world', np.uint8)
    with pytest.raises(Exception, match='LDDL_TOKENIZE_PATH'):
        ctxs['uncased'].tokenize_host(text, np.asarray([0, len(text)], np.int64))


def test_tokenize_long_and_empty_sentences(ctxs):
    """Sentences far beyond 512 pieces (early stop), runs of empty sentences (ring retirement),
    and one sentence per wave's stream position."""
    from oracle import oracle as O
    parts = [b'', b'', b'word ' * 3000, b'', b'a', b'  ', b'[SEP] x ' * 400, b''] * 50
    text = np.frombuffer(b''.join(parts), np.uint8).copy()
    off = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
    tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
    for mp in (512, 3):
        ids, o = ctxs['uncased'].tokenize_host(text, off, max_pieces=mp)
        e, eo = tok.tokenize(text, off, max_pieces=mp)
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(ids, e)


@pytest.mark.parametrize('grid', ['1', '3'])
def test_tokenize_dynamic_chunks_vs_oracle(ctxs, monkeypatch, grid):
    """With a grid of 1 or 3 workgroups (LDDL_TOKENIZE_GRID) most sentences are claimed through
    the batch kernel's atomic chunk counter, in chunks of consecutive (adjacent) sentences; the
    output is the oracle's, with runs of empty sentences at chunk boundaries included."""
    from oracle import oracle as O
    monkeypatch.setenv('LDDL_TOKENIZE_GRID', grid)
    text, off = _adversarial_corpus(seed=31, n=9000)
    tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
    for mp in (512, 9):
        ids, o = ctxs['uncased'].tokenize_host(text, off, max_pieces=mp)
        e, eo = tok.tokenize(text, off, max_pieces=mp)
        np.testing.assert_array_equal(o, eo)
        np.testing.assert_array_equal(ids, e)


@pytest.mark.parametrize('case', ['uncased', 'cased'])
@pytest.mark.parametrize('sample', ['1', '64', '1000'])
def test_tokenize_word_memo_vs_oracle(ctxs, monkeypatch, case, sample):
    """The word memo (a sample pass stores each multi-piece word's pieces, the rest of the call
    reads them; on by default for inputs of >= 64 K sentences): forced onto small inputs with a
    sample of 1 / 64 / 1000 sentences (LDDL_TOKENIZE_MEMO_SAMPLE), the output is the oracle's on
    the synthetic corpus (repeated words: memo hits), the adversarial one (non-ASCII words
    normalised before the lookup, [UNK], > 8 pieces, dropped characters) and with the dynamic
    chunk claims of a one-workgroup grid."""
    from lddl_amd import synth
    from oracle import oracle as O
    vocab = VOCAB_UNCASED if case == 'uncased' else VOCAB_CASED
    tok = O.Tokenizer(vocab, lowercase=case == 'uncased')
    monkeypatch.setenv('LDDL_TOKENIZE_MEMO_SAMPLE', sample)
    corp = synth.generate(seed=77, n_bytes=1 << 20, nonascii_frac=0.05)
    for text, off in ((corp.text, corp.sent_off), _adversarial_corpus(seed=5, n=4000)):
        for grid in (None, '1'):
            if grid:
                monkeypatch.setenv('LDDL_TOKENIZE_GRID', grid)
            for mp in (512, 9):
                ids, o = ctxs[case].tokenize_host(text, off, max_pieces=mp)
                e, eo = tok.tokenize(text, off, max_pieces=mp)
                _assert_same(ids, o, e, eo, text, off)
            monkeypatch.delenv('LDDL_TOKENIZE_GRID', raising=False)
