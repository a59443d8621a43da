"""Quick tokenizer throughput probe (not the bench): time lddl_tokenize over a synthetic batch."""
import sys
import time

import torch

sys.path.insert(0, '.')
from lddl_amd import synth
from lddl_amd.context import Context

nbytes = int(float(sys.argv[1])) if len(sys.argv) > 1 else 256 << 20
t0 = time.time()
corp = synth.generate(seed=1234, n_bytes=nbytes, threads=16)
print('gen {:.2f}s {} bytes {} sents'.format(time.time() - t0, len(corp.text), corp.n_sent), flush=True)
ctx = Context('lddl_amd/assets/vocab_synth_uncased_30522.txt')
text = torch.from_numpy(corp.text).cuda()
off = torch.from_numpy(corp.sent_off).cuda()
for _ in range(2):
    ids, sl = ctx.tokenize(text, off)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
n = 5
for _ in range(n):
    ids, sl = ctx.tokenize(text, off)
ev1.record()
torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1) / n
pieces = int((sl & ((1 << 30) - 1)).sum())
import os
fb = os.environ.get('LDDL_TOKENIZE_PATH', 'batch')
print('[{}] tokenize: {:.3f} ms/iter, {:.2f} GB/s text, {:.3f} G pieces/s, pieces={}'.format(
    fb, ms, len(corp.text) / ms / 1e6, pieces / ms / 1e6, pieces), flush=True)
