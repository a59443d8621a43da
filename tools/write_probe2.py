"""Parquet write throughput on the GPU box, 16 threads x 256 files of ~10 MB, for tables built
like the CLI's (Array.from_buffers over numpy views) from pageable vs pinned host memory."""
import os
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import torch

N = 10000
rng = np.random.default_rng(0)
nb = N * 500
src = rng.integers(97, 122, nb, dtype=np.uint8)
off = (np.arange(N + 1, dtype=np.int64) * 500).astype(np.int32)
sch = pa.schema([('A', pa.string()), ('B', pa.string()), ('is_random_next', pa.bool_()),
                 ('num_tokens', pa.uint16())])
d = tempfile.mkdtemp(dir=os.environ.get('TMPDIR', '/tmp'))
torch.cuda.init()
for kind in ('pageable', 'pinned'):
    if kind == 'pinned':
        buf = torch.empty(nb, dtype=torch.uint8, pin_memory=True).numpy()
    else:
        buf = np.empty(nb, np.uint8)
    buf[:] = src

    def mk():
        a = pa.Array.from_buffers(pa.string(), N, [None, pa.py_buffer(off), pa.py_buffer(buf)])
        return pa.Table.from_arrays([a, a, pa.array(np.zeros(N, bool)),
                                     pa.array(np.zeros(N, np.uint16))], schema=sch)
    for threads in (1, 16):
        n = 16 * threads
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(lambda i: pq.write_table(mk(), os.path.join(d, 'f%d.parquet' % i),
                                                 compression=None), range(n)))
        dt = time.perf_counter() - t0
        print('%s %2d threads: %.2f GB/s, %.1f ms per file' % (kind, threads, 2 * nb * n / dt / 1e9,
                                                               dt / n * threads * 1e3))
        for i in range(n):
            os.remove(os.path.join(d, 'f%d.parquet' % i))
