"""GPU Punkt segmentation parity (csrc/segment.hip through lddl_segment_count/_fill) against
nltk's spans (tests/golden/punkt.npz) and the oracle, and the segmented path end to end
(segment -> tokenize -> NSP pairs + static masking) against the oracle."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, VOCAB_UNCASED

pytestmark = pytest.mark.gpu


def reference_sentences(text, doc_off, st, en, cnt):
    """sent_tokenize + strip + drop empty (pretrain.py:86-88) from (nltk / oracle) spans."""
    out, k = [], 0
    for d in range(len(doc_off) - 1):
        b0 = int(doc_off[d])
        ss = [bytes(text[b0 + st[j]:b0 + en[j]]).decode('utf-8').strip()
              for j in range(k, k + int(cnt[d]))]
        out.append([s for s in ss if s])
        k += int(cnt[d])
    return out


@pytest.fixture(scope='module')
def ctx():
    from lddl_amd.context import Context
    return Context(VOCAB_UNCASED, True)


@pytest.fixture(scope='module')
def golden():
    with np.load(os.path.join(GOLDEN, 'punkt.npz')) as z:
        g = dict(z)
    with open(os.path.join(GOLDEN, 'punkt_params.json')) as f:
        g['params'] = json.load(f)
    return g


def gpu_sentences(ctx, text, doc_off, params=None):
    import torch
    from lddl_amd import punkt
    punkt.set_params(ctx, punkt.PunktParams.from_dict(params) if params else None)
    t = torch.from_numpy(np.ascontiguousarray(text)).cuda()
    do = torch.from_numpy(np.ascontiguousarray(doc_off, np.int64)).cuda()
    so, ds = punkt.segment(ctx, t, do)
    so, ds = so.cpu().numpy(), ds.cpu().numpy()
    # layout invariants: contiguous, monotone, covering the batch, 1+ sentence per document
    assert so[0] == doc_off[0] and so[-1] == doc_off[-1]
    assert (np.diff(so) >= 0).all()
    assert np.array_equal(so[ds[:-1]], doc_off[:-1])
    assert (np.diff(ds) >= 1).all()
    return punkt.stripped_sentences(text, so, ds)


@pytest.mark.parametrize('name', ['untrained', 'trained'])
def test_segment_matches_nltk(ctx, golden, name):
    prm = golden['params'] if name == 'trained' else None
    got = gpu_sentences(ctx, golden['text'], golden['doc_off'], prm)
    exp = reference_sentences(golden['text'], golden['doc_off'], golden[name + '_start'],
                              golden[name + '_end'], golden[name + '_count'])
    assert len(got) == len(exp)
    bad = [d for d in range(len(exp)) if got[d] != exp[d]]
    assert not bad, (len(bad), bad[:5], [(got[d], exp[d]) for d in bad[:2]])


def test_segment_synthetic_vs_oracle(ctx):
    from lddl_amd import synth
    from oracle import oracle as O
    text, doc_off = synth.generate_doc_text(seed=31, n_bytes=8 << 20, nonascii_frac=0.05, threads=8)
    got = gpu_sentences(ctx, text, doc_off)
    st, en, cnt = O.Punkt().spans(text, doc_off)
    assert got == reference_sentences(text, doc_off, st, en, cnt)


def test_segment_dense_enders_vs_oracle(ctx):
    """Runs of sentence enders (every byte a qualified ender: "?!?!?! x") and long runs that
    cross the 4-KB slab and the 64-byte context windows; documents back to back, so a write
    outside a document's candidate slots would corrupt its neighbour."""
    from oracle import oracle as O
    import random
    rng = random.Random(5)
    docs = ['?!' * 40 + ' x', '?' * 301 + ' Y', '.!?' * 50 + ') Z. ' + '!' * 7, 'a.)' * 100,
            ('word' * 300 + '. Next. ') * 3, '"' * 70 + 'x.' + ')' * 70 + ' Y',
            ' '.join('w{}?!'.format(i) for i in range(700)), 'x' * 5000 + '. A ' + 'b' * 4500 + '.']
    docs += [''.join(rng.choice('?!.) "ab') for _ in range(rng.randint(1, 200))) for _ in range(300)]
    enc = [d.encode() for d in docs]
    doc_off = np.concatenate([[0], np.cumsum([len(e) for e in enc])]).astype(np.int64)
    text = np.frombuffer(b''.join(enc), np.uint8)
    got = gpu_sentences(ctx, text, doc_off)
    st, en, cnt = O.Punkt().spans(text, doc_off)
    exp = reference_sentences(text, doc_off, st, en, cnt)
    bad = [d for d in range(len(exp)) if got[d] != exp[d]]
    assert not bad, (bad[:5], [(got[d][:3], exp[d][:3]) for d in bad[:2]])


def test_segment_empty_and_whitespace_documents(ctx):
    docs = ['', '   ', 'One. Two.', '　', 'x', 'End.) ', '']
    enc = [d.encode() for d in docs]
    doc_off = np.concatenate([[0], np.cumsum([len(e) for e in enc])]).astype(np.int64)
    text = np.frombuffer(b''.join(enc), np.uint8)
    got = gpu_sentences(ctx, text, doc_off)
    assert got == [[], [], ['One.', 'Two.'], [], ['x'], ['End.)'], []]


def test_segmented_path_end_to_end(ctx):
    """GPU segment -> tokenize -> pairs (whitespace kept between sentences) equals the oracle
    on the reference's stripped sentences."""
    import torch
    from lddl_amd import punkt, synth
    from lddl_amd.pairs import make_pairs
    from oracle import oracle as O
    text, doc_off = synth.generate_doc_text(seed=77, n_bytes=1 << 20, nonascii_frac=0.05, threads=8)
    punkt.set_params(ctx, None)
    t = torch.from_numpy(text).cuda()
    so, ds = punkt.segment(ctx, t, torch.from_numpy(doc_off).cuda())
    ids, sl = ctx.tokenize(t, so)
    n_doc = len(doc_off) - 1
    part = np.asarray([0, n_doc // 3, n_doc], np.int64)
    seeds = np.asarray([5, 6], np.int64)
    pb = make_pairs(ctx, so, ids, sl, ds, torch.from_numpy(part).cuda(),
                    torch.from_numpy(seeds).cuda(), seq=128, dup=2, masking=True).to_host()
    # oracle: nltk-equivalent spans -> stripped sentences -> compact corpus -> tokenize -> pairs
    st, en, cnt = O.Punkt().spans(text, doc_off)
    docs = reference_sentences(text, doc_off, st, en, cnt)
    corp = synth.from_documents(docs)
    tok = O.Tokenizer(VOCAB_UNCASED)
    e_ids, e_off = tok.tokenize(corp.text, corp.sent_off)
    lens = np.diff(e_off)
    keep = lens > 0
    k_off = np.concatenate([[0], np.cumsum(lens[keep])])
    kept_pos = np.concatenate([[0], np.cumsum(keep)])
    ds_h = np.concatenate([[0], np.cumsum([len(d) for d in docs])])
    toks, nts = [], []
    for p in range(2):
        kd = kept_pos[ds_h[part[p]:part[p + 1] + 1]]
        kd = np.concatenate([kd[:1], kd[1:][np.diff(kd) > 0]])
        out = O.partition_pairs(kd, k_off, e_ids, int(seeds[p]), 2, 128, True, tok.vocab_size,
                                *(tok.token_id(x) for x in ('[CLS]', '[SEP]', '[MASK]')))
        toks.append(out['tokens'])
        nts.append(out['num_tokens'])
    np.testing.assert_array_equal(pb['num_tokens'], np.concatenate(nts))
    np.testing.assert_array_equal(pb['tokens'], np.concatenate(toks))
