"""Host sentence segmentation (`--sentence-splitter host`): the reference's own
`nltk.tokenize.sent_tokenize` (lddl/dask/bert/pretrain.py:86, 583), for debugging and A/B runs
against the GPU Punkt (lddl_amd/punkt.py + csrc/segment.hip, the default).

The reference needs nltk and downloads its English Punkt model at run time
(`nltk.download('punkt')`). Here, with nltk importable:
  1. `nltk.tokenize.sent_tokenize` when the English Punkt model loads locally;
  2. nltk's untrained `PunktSentenceTokenizer()` otherwise (what offline nltk degrades to).
Without nltk this splitter refuses to run: an approximation would silently produce other
sentences than the reference. Use the GPU splitter, which restates nltk's Punkt exactly.
"""
_splitter = None
KIND = None


def _init():
    global _splitter, KIND
    if _splitter is not None:
        return
    try:
        import nltk
    except ImportError as e:
        raise RuntimeError(
            "--sentence-splitter host needs nltk (the reference's sent_tokenize), which is not "
            "importable here; use the default --sentence-splitter gpu (exact nltk Punkt on the "
            "GPU)") from e
    try:
        nltk.data.find('tokenizers/punkt')
        _splitter, KIND = nltk.tokenize.sent_tokenize, 'nltk-punkt-english'
    except LookupError:
        from nltk.tokenize.punkt import PunktSentenceTokenizer
        _splitter, KIND = PunktSentenceTokenizer().tokenize, 'nltk-punkt-untrained'


def sent_tokenize(text):
    _init()
    return _splitter(text)


def document_sentences(raw_line):
    """`_to_document` up to tokenization (pretrain.py:82-88): id / text split, sentences,
    strip, drop empty."""
    from ..readers import split_id_text
    doc_id, text = split_id_text(raw_line)
    return doc_id, [s for s in (x.strip() for x in sent_tokenize(text)) if s]
