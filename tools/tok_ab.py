"""Tokenizer A/B (diagnostic): time lddl_tokenize over one synthetic batch with each
LDDL_TOKENIZE_PATH value and library given, and check every variant's ids / sent_len bit for bit
against the first one's.

    python tools/tok_ab.py <bytes> <variant>...   variant = [path][@lib-dir], e.g. batch  cp
    cp@lddl_amd/_lib_x  (path '' or batch = the default kernel)
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from lddl_amd import synth  # noqa: E402
from lddl_amd.context import Context  # noqa: E402

nbytes = int(float(sys.argv[1]))
variants = sys.argv[2:] or ['batch']
corp = synth.generate(seed=1234, n_bytes=nbytes, nonascii_frac=0.01, threads=16)
ctx = Context(os.path.join(REPO, 'lddl_amd', 'assets', 'vocab_synth_uncased_30522.txt'))
text = torch.from_numpy(corp.text).cuda()
off = torch.from_numpy(corp.sent_off).cuda()
ref = None
for v in variants:
    path = v.split('@')[0]
    if path in ('', 'batch'):
        os.environ.pop('LDDL_TOKENIZE_PATH', None)
    else:
        os.environ['LDDL_TOKENIZE_PATH'] = path
    for _ in range(2):
        ids, sl = ctx.tokenize(text, off)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 5
    e0.record()
    for _ in range(n):
        ids, sl = ctx.tokenize(text, off)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    pieces = int((sl & ((1 << 30) - 1)).sum())
    same = None
    if ref is None:
        ref = (ids, sl)
    else:
        # the sparse ids layout: compare only each sentence's kept pieces
        same = bool(torch.equal(sl, ref[1]))
        if same:
            L = (sl & ((1 << 30) - 1)).to(torch.int64)
            so = off[:-1]
            mx = int(L.max())
            k = torch.arange(mx, device=L.device)
            for c0 in range(0, len(L), 1 << 20):
                Lc, sc = L[c0:c0 + (1 << 20)], so[c0:c0 + (1 << 20)]
                m = k[None, :] < Lc[:, None]
                idx = (sc[:, None] + k[None, :])[m]
                if not torch.equal(ids[idx], ref[0][idx]):
                    same = False
                    break
    print('[{}] {:.3f} ms per {:.2f} GB, {:.2f} GB/s text, pieces {} bit-exact vs first: {}'.format(
        v, ms, nbytes / 1e9, nbytes / ms / 1e6, pieces, same), flush=True)
