"""Host-side cost of getting rendered batches off the GPU (diagnostic; the CLI's tail): pinned
allocation (torch's host allocator, fresh and cached), device-to-host copy into pinned and into
pageable memory, for a few sizes.

    python tools/d2h_probe.py
"""
import time

import torch


def t(f):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, r


for gb in (1, 4):
    n = gb << 30
    d = torch.empty(n, dtype=torch.uint8, device='cuda').fill_(7)
    ta, h = t(lambda: torch.empty(n, dtype=torch.uint8, pin_memory=True))
    tc, _ = t(lambda: h.copy_(d, non_blocking=True))
    tc2, _ = t(lambda: h.copy_(d, non_blocking=True))
    del h
    tr, h2 = t(lambda: torch.empty(n, dtype=torch.uint8, pin_memory=True))  # cached block
    del h2
    p = torch.empty(n, dtype=torch.uint8)
    p.numpy()[::4096] = 1  # touch the pages
    tp, _ = t(lambda: p.copy_(d))
    tp2, _ = t(lambda: p.copy_(d))
    print('{} GiB: pinned alloc {:.3f} s ({:.1f} GB/s), D2H into it {:.3f} s ({:.1f} GB/s; again '
          '{:.1f} GB/s), cached re-alloc {:.4f} s; pageable D2H {:.3f} s ({:.1f} GB/s; again {:.1f} GB/s)'
          .format(gb, ta, n / ta / 1e9, tc, n / tc / 1e9, n / tc2 / 1e9, tr, tp, n / tp / 1e9,
                  n / tp2 / 1e9), flush=True)
    del d, p
