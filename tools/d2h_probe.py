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


# Does a pinned allocation stall the other host threads? A ticker thread records its longest
# gap while the main thread allocates 4 GiB pinned, through torch and through hipHostMalloc
# (ctypes releases the GIL during the foreign call); then a 512 MiB pageable H2D copy is timed
# while another thread makes the same allocation.
import ctypes  # noqa: E402
import threading  # noqa: E402

hip = ctypes.CDLL('libamdhip64.so')
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipHostFree.argtypes = [ctypes.c_void_p]


def alloc_torch(n):
    return torch.empty(n, dtype=torch.uint8, pin_memory=True)


def alloc_hip(n):
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), n, 0) == 0
    return p


def free_hip(p):
    hip.hipHostFree(p)


def ticker_gap(fn):
    stop, gaps = [False], []

    def tick():
        last = time.perf_counter()
        while not stop[0]:
            time.sleep(0.0005)
            now = time.perf_counter()
            gaps.append(now - last)
            last = now
    th = threading.Thread(target=tick)
    th.start()
    time.sleep(0.05)
    t0 = time.perf_counter()
    r = fn()
    ta = time.perf_counter() - t0
    time.sleep(0.05)
    stop[0] = True
    th.join()
    return ta, max(gaps), r


n = 4 << 30
ta, gap, h = ticker_gap(lambda: alloc_torch(n))
print('torch pinned 4 GiB: {:.3f} s, longest gap of another Python thread {:.3f} s'.format(ta, gap),
      flush=True)
del h
ta, gap, p = ticker_gap(lambda: alloc_hip(n))
print('hipHostMalloc 4 GiB (ctypes): {:.3f} s, longest gap of another Python thread {:.3f} s'.format(
    ta, gap), flush=True)
free_hip(p)
src = torch.empty(512 << 20, dtype=torch.uint8)
src.numpy()[::4096] = 1
t(lambda: src.to('cuda'))
t_alone, _ = t(lambda: src.to('cuda'))
for name, fn, fr in (('torch', alloc_torch, lambda r: None), ('hipHostMalloc', alloc_hip, free_hip)):
    box = []
    th = threading.Thread(target=lambda: box.append(fn(n)))
    th.start()
    time.sleep(0.005)
    tb, _ = t(lambda: src.to('cuda'))
    th.join()
    fr(box[0])
    del box
    print('512 MiB pageable H2D: alone {:.3f} s, beside a 4 GiB {} allocation {:.3f} s'.format(
        t_alone, name, tb), flush=True)

# ... and other HIP work beside such an allocation: 100 small kernel launches + sync, and a
# 512 MiB H2D copy from pinned memory
dev = torch.ones(1 << 20, device='cuda')
pin_src = torch.empty(512 << 20, dtype=torch.uint8, pin_memory=True)
t(lambda: pin_src.to('cuda', non_blocking=True))


def launches():
    for _ in range(100):
        dev.add_(1.0)


tl_alone, _ = t(launches)
tp_alone, _ = t(lambda: pin_src.to('cuda', non_blocking=True))
for name, fn in (('100 launches', launches), ('512 MiB pinned H2D', lambda: pin_src.to('cuda', non_blocking=True))):
    box = []
    th = threading.Thread(target=lambda: box.append(alloc_hip(n)))
    th.start()
    time.sleep(0.005)
    tb, _ = t(fn)
    th.join()
    free_hip(box[0])
    print('{}: alone {:.4f} s, beside a 4 GiB hipHostMalloc {:.4f} s'.format(
        name, tl_alone if name.startswith('100') else tp_alone, tb), flush=True)
