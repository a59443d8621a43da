"""Sentence segmentation at the host boundary (the reference's `nltk.tokenize.sent_tokenize`,
lddl/dask/bert/pretrain.py:86, 583).

The reference needs NLTK's pre-trained English Punkt model, which is downloaded at run time
(`nltk.download('punkt')`); this environment has no network and no model. Order of preference:
  1. `nltk.tokenize.sent_tokenize` when nltk and its English Punkt model load;
  2. nltk's untrained `PunktSentenceTokenizer()` when nltk imports but the model is absent;
  3. the built-in rule splitter below (an approximation of untrained Punkt: break after
     [.?!] plus closing quotes/brackets when whitespace follows, except after an ellipsis or a
     single-letter initial followed by a capitalised word).
A GPU Punkt is SURVEY.md §8(f1) ("next"); this module is the host fallback until then.
"""
import re

_splitter = None
KIND = None

_BREAK = re.compile(r'''(?<=[.?!])(?:["')\]}']*)(?=\s+\S)''')


def _rule_split(text):
    out, start = [], 0
    for m in _BREAK.finditer(text):
        end = m.end()
        head = text[start:end].rstrip()
        # token that carries the terminator
        tok = head.split()[-1] if head.split() else ''
        core = tok.rstrip('"\')]}\'')
        if core.endswith('...'):
            continue
        nxt = text[end:].lstrip()[:1]
        word = core[:-1]
        if len(word) == 1 and word.isalpha() and core.endswith('.') and nxt.isupper():
            continue  # an initial ("J. Smith")
        out.append(text[start:end])
        start = end
    out.append(text[start:])
    return out


def _init():
    global _splitter, KIND
    if _splitter is not None:
        return
    try:
        import nltk
        try:
            nltk.data.find('tokenizers/punkt')
            _splitter, KIND = nltk.tokenize.sent_tokenize, 'nltk-punkt-english'
        except LookupError:
            from nltk.tokenize.punkt import PunktSentenceTokenizer
            _splitter, KIND = PunktSentenceTokenizer().tokenize, 'nltk-punkt-untrained'
    except ImportError:
        _splitter, KIND = _rule_split, 'rules'


def sent_tokenize(text):
    _init()
    return _splitter(text)


def document_sentences(raw_line):
    """`_to_document` up to tokenization (pretrain.py:82-88): id / text split, sentences,
    strip, drop empty."""
    from ..readers import split_id_text
    doc_id, text = split_id_text(raw_line)
    return doc_id, [s for s in (x.strip() for x in sent_tokenize(text)) if s]
