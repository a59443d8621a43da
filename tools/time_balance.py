"""Per-phase wall times of lddl_amd.balance.balance on a bench-sized C4 batch (diagnostics)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
from bench import make_batch, VOCAB  # noqa: E402
from lddl_amd.balance import balance  # noqa: E402
from lddl_amd.context import Context  # noqa: E402
from lddl_amd.pairs import make_pairs  # noqa: E402


class A:
    seed = 1234
    batch_bytes = int(float(sys.argv[1])) if len(sys.argv) > 1 else 4 << 30
    partition_bytes = 1 << 20
    gen_threads = 16


corp, part, seeds = make_batch(0, A)
ctx = Context(VOCAB)
d = lambda x: torch.from_numpy(x).cuda()  # noqa: E731
so = d(corp.sent_off)
ids, sl = ctx.tokenize(d(corp.text), so)
for it in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pb = make_pairs(ctx, so, ids, sl, d(corp.doc_sent_off), d(part), d(seeds), seq=512, dup=5,
                    masking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    tm = {}
    bb = balance(ctx, pb, 8, 64, timings=tm)
    keys = list(tm)
    print('pairs {:.1f} ms; balance: {}'.format((t1 - t0) * 1e3, ', '.join(
        '{} {:.1f} ms'.format(k, (tm[k] - tm[p]) * 1e3) for p, k in zip(keys, keys[1:]))),
        flush=True)
    del pb, bb
