"""Host read bandwidth of torch pinned memory vs pageable numpy memory (the CLI's writers read
the rendered strings from the D2H staging buffers)."""
import time

import numpy as np
import torch

n = 1 << 30
torch.cuda.init()
for kind in ('pageable', 'pinned'):
    if kind == 'pinned':
        h = torch.empty(n, dtype=torch.uint8, pin_memory=True).numpy()
    else:
        h = np.empty(n, np.uint8)
    h[:] = 7
    t0 = time.perf_counter()
    for _ in range(3):
        x = h.copy()
    dt = (time.perf_counter() - t0) / 3
    print('%s: host read+copy %.2f GB/s' % (kind, n / dt / 1e9))
    d = torch.empty(n, dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if kind == 'pinned':
        ht = torch.from_numpy(h)
        ht.copy_(d, non_blocking=True)
    else:
        torch.from_numpy(h).copy_(d)
    torch.cuda.synchronize()
    print('%s: D2H %.2f GB/s' % (kind, n / (time.perf_counter() - t0) / 1e9))
t0 = time.perf_counter()
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
print('pin alloc 1 GiB: %.3f s' % (time.perf_counter() - t0))
