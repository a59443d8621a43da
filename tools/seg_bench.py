"""Time GPU Punkt segmentation alone (HIP events around lddl_segment_count + fill) on synthetic
raw documents. python tools/seg_bench.py [GiB]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lddl_amd import punkt, synth  # noqa: E402
from lddl_amd.context import Context  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
text, doc_off = synth.generate_doc_text(seed=1234, n_bytes=int(gib * (1 << 30)), nonascii_frac=0.01,
                                        threads=16)
ctx = Context(os.path.join(os.path.dirname(punkt.__file__), 'assets', 'vocab_synth_uncased_30522.txt'))
t = torch.from_numpy(text).cuda()
d = torch.from_numpy(doc_off).cuda()
punkt.set_params(ctx, None)
for _ in range(2):
    so, ds = punkt.segment(ctx, t, d)
torch.cuda.synchronize()
ms = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    so, ds = punkt.segment(ctx, t, d)
    e1.record()
    torch.cuda.synchronize()
    ms.append(e0.elapsed_time(e1))
print('segment: {:.1f} MB, {} docs, {} sentences, {:.2f} ms (min {:.2f}), {:.1f} GB/s'.format(
    len(text) / 1e6, len(doc_off) - 1, so.numel() - 1, np.mean(ms), min(ms),
    len(text) / (min(ms) * 1e-3) / 1e9), flush=True)
