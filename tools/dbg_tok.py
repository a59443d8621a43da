"""Debug helper: first sentences where the GPU tokenizer and the oracle disagree (adversarial corpus)."""
import sys
import numpy as np
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
from test_tokenize_gpu import _adversarial_corpus, VOCAB_UNCASED
from lddl_amd.context import Context
from oracle import oracle as O
text, off = _adversarial_corpus()
ctx = Context(VOCAB_UNCASED)
tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
ids, o = ctx.tokenize_host(text, off, max_pieces=512)
e, eo = tok.tokenize(text, off, max_pieces=512)
lg, le = np.diff(o), np.diff(eo)
bad = np.nonzero(lg != le)[0]
print('mismatched sentences', len(bad), 'of', len(lg), 'first', bad[:20])
for s in bad[:6]:
    print('--- sentence', s, 'mod32', s % 32, 'len', off[s + 1] - off[s], 'got', lg[s], 'want', le[s])
    for t in (s - 1, s, s + 1):
        if 0 <= t < len(lg):
            print('  s', t, bytes(text[off[t]:off[t + 1]]))
    print('  got ', ids[o[s]:o[s + 1]].tolist())
    print('  want', e[eo[s]:eo[s + 1]].tolist())
