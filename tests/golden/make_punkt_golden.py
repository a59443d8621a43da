"""Golden fixtures for sentence segmentation (tests/golden/punkt.npz + punkt_params.json), made by
nltk itself in the dev container (nltk is not on the GPU box).

The reference segments each document with `nltk.tokenize.sent_tokenize(text)`
(lddl/dask/bert/pretrain.py:86), then strips every sentence and drops the empty ones (87-88).
nltk is a third-party dependency, not vendored in the reference (pinned version in this image:
nltk 3.6.5 under /opt/conda/lib/python3.9/site-packages). Its English Punkt model is a run-time
download (absent offline), so two parameter sets are recorded:

  untrained  PunktSentenceTokenizer()            (what sent_tokenize degrades to here)
  trained    PunktSentenceTokenizer(params)      hand-made PunktParameters exercising every
             parameter lookup: abbreviations (incl. hyphen suffix rule), collocations, frequent
             sentence starters, orthographic context flags

Documents: synthetic corpus documents (sentences joined by assorted whitespace), hand-written
edge cases, and seeded fuzz strings over the characters the Punkt regular expressions treat
specially (sentence enders, closing brackets/quotes, hyphens, commas, Unicode whitespace, cased
and uncased letters, Unicode digits). Expected output: nltk's `span_tokenize` spans as UTF-8 byte
offsets relative to each document. Only data is written.

    python tests/golden/make_punkt_golden.py
"""
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

EDGE = [
    '', ' ', 'Hello.', 'Hello. World.', 'Hello Mr. Smith. (Sent1.) Sent2! J. Bach lived in 12. '
    'century... x.)y. z? a', 'A.  B.', 'end.) Next one.', 'Quote." Next?" Really!\' ok.',
    'He said "Go." Then left.', 'Wait... what?', 'Stop.--not', 'x.--Y', 'a. . . b', 'a . . . b',
    'U.S. Army. The end', 'e.g. this', 'no. 5 is here. No. 6 too', '3.5 is. 4. Then',
    'Mr. Smith met Dr. Who. The end.', 'x. Y', 'x. Y', 'x.\x1cY', 'x.\x0bY z.\x85W',
    'É. Élan. é. élan.', 'İ. İstanbul. ı. x', 'A.B. C.', '...', '. . .', '?!', 'Hi?! Yo.',
    'word.)', 'word.)  ', '  lead. trail.  ', 'nums 1,000. 2 things. -4. Z', 'a,. b', 'a,) b',
    'x.(y) z. W', 'tab.\tTab', 'x.\rY', 'one.\n two', 'Ünal. ünal. ß. SS.', 'x.　Y.',
    '(a.) (b.) c.', 'He lied." she said.', 'J. Bach. j. bach.', '٣. A. ²x. B', '_. A',
    'end.]} x', 'end."\' x', 'end.)-- x', 'end.)--x', 'a.--b. C', 'etc. and so. on',
    'Prof. X. Fig. 3 shows. the', 'jan. 12 was. Jan. 13', 'st.-louis. St. Louis',
    'fig.-1. F', 'dort. Dort. but. But. the. The',
]

ALPHABET = (list('..........??!!!)))"""\'\'\']]}}(([{{----,,,;;::**@@&&##``') +
            [' '] * 30 + ['\t', ' ', ' ', '\x1c', '　', '\x0b'] +
            list('aAbBxXjJzZ') + ['é', 'É', 'ß', 'İ', 'ı', '_', '²', '٣', '5', '0', '9'])
WORDS = ['Mr', 'mr', 'Dr', 'dr', 'who', 'Who', 'the', 'The', 'century', 'J', 'j', 'x', 'A', 'É',
         'é', 'ß', '12', '3.5', '1,000', '-4', 'İstanbul', 'Ünal', 'ünal', '_x', '²', '٣', 'e.g',
         'U.S', 'u.s', 'etc', 'vs', 'jan', 'Jan', 'no', 'No', 'St', 'ms', 'Prof', 'fig', 'dort',
         'Dort', 'But', 'but', 'However', 'however', 'st-louis', 'fig-1', 'Wait', 'go', 'GO']
PUNCT = ['.', '.', '.', '?', '!', '...', '.)', '."', '?"', ".'", '.)]', ',', ';', ':', '--', '-',
         '(', ')', '"', "'", '.--', '..', '?!']
SPACES = [' ', ' ', ' ', ' ', '  ', '\t', ' ', ' ', '\x1c', ' 　 ', '\x85', '\r']


def fuzz_docs(rng, n):
    docs = []
    for _ in range(n):
        if rng.random() < 0.35:
            docs.append(''.join(rng.choice(ALPHABET) for _ in range(rng.randint(1, 60))))
            continue
        parts = []
        for _ in range(rng.randint(1, 14)):
            w = rng.choice(WORDS)
            if rng.random() < 0.15:
                w = rng.choice(PUNCT[12:]) + w
            parts.append(w)
            if rng.random() < 0.45:
                parts.append(rng.choice(PUNCT))
            parts.append(rng.choice(SPACES) if rng.random() < 0.9 else '')
        docs.append(''.join(parts))
    return docs


def synth_docs(n_bytes=200_000):
    from lddl_amd import synth
    rng = random.Random(7)
    corp = synth.generate(seed=99, n_bytes=n_bytes, nonascii_frac=0.05, threads=4)
    out = []
    for d in range(corp.n_doc):
        s0, s1 = corp.doc_sent_off[d], corp.doc_sent_off[d + 1]
        sents = [corp.sentence(i) for i in range(s0, s1)]
        out.append(''.join(s + (rng.choice([' ', ' ', ' ', '  ', '\t']) if i + 1 < len(sents)
                                else '') for i, s in enumerate(sents)))
    return out


def trained_params():
    return {
        'abbrev_types': ['mr', 'dr', 'e.g', 'u.s', 'etc', 'vs', 'jan', 'no', 'st', 'ms', 'prof',
                         'fig', 'louis', 'é', 'ünal', '1'],
        'collocations': [['##number##', 'century'], ['dr', 'who'], ['jan', '##number##'],
                         ['mr', 'j'], ['x', 'y']],
        'sent_starters': ['the', 'but', 'however', 'dort', 'j', 'é'],
        'ortho_context': {},
    }


def main():
    sys.path.append('/opt/conda/lib/python3.9/site-packages')
    from nltk.tokenize.punkt import PunktParameters, PunktSentenceTokenizer
    rng = random.Random(2024)
    docs = EDGE + synth_docs() + fuzz_docs(rng, 6000)
    prm = trained_params()
    # orthographic flags (nltk's _ORTHO_* bits 2..64) for every word type the fuzz can produce
    types = set()
    for w in WORDS + ['y', 'x', 'b', 'a', 'z', 'ss', 'i̇stanbul', 'louis', 'go', 'wait', '##number##']:
        types.add(w.lower())
    for t in sorted(types):
        prm['ortho_context'][t] = rng.choice([0, 2, 4, 8, 16, 32, 64, 2 | 16, 4 | 32, 8 | 64,
                                              2 | 4 | 8, 16 | 32 | 64, 126, 2 | 32, 4 | 16])
    p = PunktParameters()
    p.abbrev_types = set(prm['abbrev_types'])
    p.collocations = set(tuple(c) for c in prm['collocations'])
    p.sent_starters = set(prm['sent_starters'])
    for k, v in prm['ortho_context'].items():
        p.ortho_context[k] = v
    toks = {'untrained': PunktSentenceTokenizer(), 'trained': PunktSentenceTokenizer(p)}
    enc = [d.encode('utf-8') for d in docs]
    doc_off = np.zeros(len(enc) + 1, np.int64)
    np.cumsum([len(e) for e in enc], out=doc_off[1:])
    out = {'text': np.frombuffer(b''.join(enc), np.uint8), 'doc_off': doc_off}
    for name, tok in toks.items():
        starts, ends, counts = [], [], []
        for d in docs:
            # code-point index -> byte offset
            cum = np.zeros(len(d) + 1, np.int64)
            np.cumsum([len(c.encode('utf-8')) for c in d], out=cum[1:])
            sp = list(tok.span_tokenize(d))
            counts.append(len(sp))
            starts += [int(cum[a]) for a, _ in sp]
            ends += [int(cum[b]) for _, b in sp]
        out[name + '_start'] = np.asarray(starts, np.int64)
        out[name + '_end'] = np.asarray(ends, np.int64)
        out[name + '_count'] = np.asarray(counts, np.int64)
    np.savez_compressed(os.path.join(HERE, 'punkt.npz'), **out)
    with open(os.path.join(HERE, 'punkt_params.json'), 'w') as f:
        json.dump(prm, f, ensure_ascii=False, indent=0, sort_keys=True)
    print('{} documents, {} bytes; untrained {} / trained {} sentences'.format(
        len(docs), int(doc_off[-1]), int(out['untrained_count'].sum()),
        int(out['trained_count'].sum())))


if __name__ == '__main__':
    main()
