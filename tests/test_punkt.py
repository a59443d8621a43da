"""Punkt sentence segmentation, CPU side: the oracle (oracle/punkt_oracle.c) against nltk's own
spans (tests/golden/punkt.npz, tests/golden/make_punkt_golden.py), and the host parameter
records of lddl_amd.punkt."""
import json
import os
import struct

import numpy as np
import pytest

from conftest import ASSETS, GOLDEN


@pytest.fixture(scope='module')
def golden():
    with np.load(os.path.join(GOLDEN, 'punkt.npz')) as z:
        g = dict(z)
    with open(os.path.join(GOLDEN, 'punkt_params.json')) as f:
        g['params'] = json.load(f)
    return g


@pytest.mark.parametrize('name', ['untrained', 'trained'])
def test_oracle_matches_nltk_spans(golden, name):
    from oracle import oracle as O
    st, en, cnt = O.Punkt(golden['params'] if name == 'trained' else None).spans(
        golden['text'], golden['doc_off'])
    np.testing.assert_array_equal(cnt, golden[name + '_count'])
    np.testing.assert_array_equal(st, golden[name + '_start'])
    np.testing.assert_array_equal(en, golden[name + '_end'])


def test_golden_covers_the_parameter_paths(golden):
    # the trained parameters change decisions (abbreviations, collocations, starters, ortho)
    assert golden['untrained_count'].sum() != golden['trained_count'].sum()
    assert (golden['untrained_count'] > 1).sum() > 1000


def test_props_table_matches_python():
    import re
    t = np.fromfile(os.path.join(ASSETS, 'punkt_props.bin'), np.uint8)
    assert bytes(t[:4]) == b'LDPK'
    _, n_pages, n_lower = struct.unpack('<III', bytes(t[4:16]))
    l1 = t[16:16 + 0x2200].view(np.uint16)
    pages = t[16 + 0x2200:16 + 0x2200 + 256 * n_pages]
    sp, alnod, dig = re.compile(r'\s'), re.compile(r'[^\W\d]'), re.compile(r'\d')
    for cp in list(range(0, 0x3100, 7)) + [0x85, 0xA0, 0x130, 0x1680, 0x2028, 0x3000, 0x660, 0xB2]:
        ch = chr(cp)
        b = (bool(sp.match(ch)) | ch.isupper() << 1 | ch.islower() << 2 | bool(alnod.match(ch)) << 3
             | bool(dig.match(ch)) << 4)
        assert pages[int(l1[cp >> 8]) * 256 + (cp & 255)] == b, hex(cp)


def test_param_records_roundtrip(golden):
    from lddl_amd.punkt import PunktParams
    p = PunktParams.from_dict(golden['params'])
    blob, recs, i = p.records(), [], 0
    while i < len(blob):
        kind, val, la, lb = struct.unpack('<BBHH', blob[i:i + 6])
        a = blob[i + 6:i + 6 + la].decode()
        b = blob[i + 6 + la:i + 6 + la + lb].decode()
        recs.append((kind, val, a, b))
        i += 6 + la + lb
    assert {a for k, _, a, _ in recs if k == 1} == set(golden['params']['abbrev_types'])
    assert {a for k, _, a, _ in recs if k == 2} == set(golden['params']['sent_starters'])
    assert {(a, b) for k, _, a, b in recs if k == 4} == {tuple(c) for c in
                                                          golden['params']['collocations']}
    assert {a: v for k, v, a, _ in recs if k == 3} == \
        {k: v for k, v in golden['params']['ortho_context'].items()}
    with pytest.raises(ValueError):
        PunktParams(abbrev_types=['x' * 300]).records()


def test_synth_doc_text_matches_sentence_corpus():
    from lddl_amd import synth
    corp = synth.generate(seed=5, n_bytes=200_000, nonascii_frac=0.05, threads=2)
    text, doc_off = synth.generate_doc_text(seed=5, n_bytes=200_000, nonascii_frac=0.05, threads=2)
    docs = corp.documents()
    n = min(len(docs), len(doc_off) - 1) - 1
    for d in range(n):
        assert bytes(text[doc_off[d]:doc_off[d + 1]]).decode() == ' '.join(docs[d])
