"""Host write-throughput probe of the GPU box: the CLI's parquet writes (pyarrow, 16 threads,
~10 MB files of token strings) without the GPU, plus where TMPDIR lives."""
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

print(subprocess.run(['df', '-h', os.environ.get('TMPDIR', '/tmp')], capture_output=True,
                     text=True).stdout)
print('cpus', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))
import io

rng = np.random.default_rng(0)
voc = ['w%d' % i for i in range(30000)]
N = 20000


def s(k):
    return ' '.join(voc[j] for j in rng.integers(0, 30000, k))


def npy(k):
    b = io.BytesIO()
    np.save(b, np.sort(rng.integers(0, 128, k)).astype(np.uint16))
    return b.getvalue()


# the seq-128 masked schema and row shape of the CLI's part files
t = pa.table({'A': pa.array([s(55) for _ in range(N)]), 'B': pa.array([s(52) for _ in range(N)]),
              'is_random_next': pa.array(rng.integers(0, 2, N).astype(bool)),
              'num_tokens': pa.array(rng.integers(0, 128, N).astype(np.uint16)),
              'masked_lm_positions': pa.array([npy(17) for _ in range(N)], pa.binary()),
              'masked_lm_labels': pa.array([s(17) for _ in range(N)])})
nb = t.nbytes
d = tempfile.mkdtemp(dir=os.environ.get('TMPDIR', '/tmp'))
for threads in (1, 4, 8, 16):
    n_files = 16 * threads
    t0 = time.perf_counter()
    c0 = time.process_time()
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda i: pq.write_table(t, os.path.join(d, 'f%d.parquet' % i),
                                             compression=None), range(n_files)))
    dt = time.perf_counter() - t0
    cpu = time.process_time() - c0
    print('threads %d: %.2f GB in %.2f s = %.2f GB/s (cpu %.1f s)' % (threads, nb * n_files / 1e9,
                                                                     dt, nb * n_files / dt / 1e9,
                                                                     cpu))
    for i in range(n_files):
        os.remove(os.path.join(d, 'f%d.parquet' % i))
sys.stdout.flush()
