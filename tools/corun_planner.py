"""Co-residency of the replay planner with VALU work (diagnostic, not product).

The planner (plan_replay_kernel) is a chain of wave-uniform scalar steps; the issue model that
fits its time adds SALU and VALU cycles. tools/ubench/issue_rate corun shows that the CU's scalar
unit and the SIMDs' vector pipes do serve different waves in the same cycles (86-97 % overlap of a
SALU-only and a VALU-only kernel). This asks the same of the real planner: a VALU-only filler
(tools/ubench/libfiller.so, one wave per SIMD, launched first on a side stream) runs beside
make_pairs on a C2-shaped batch; if the planner keeps its own time while the filler retires its
work at its own rate, the additive model describes the planner's dependency chains, not a pipe
bound, and a VALU-heavy stage (the tokenizer) could run beside it.

    python tools/corun_planner.py [batch_bytes=2e9]

A SALU-only filler is run the same way: if the planner slowed beside it, the CU's scalar unit
(shared by the waves of its four SIMDs) would be what the planner waits on.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from lddl_amd import synth  # noqa: E402
from lddl_amd.context import Context  # noqa: E402
from lddl_amd.pairs import make_pairs  # noqa: E402


def main():
    nbytes = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(2e9)
    corp = synth.generate(seed=1234, n_bytes=nbytes, nonascii_frac=0.01, threads=16)
    part = bench.partition_docs(corp, 1 << 20)
    seeds = np.arange(len(part) - 1, dtype=np.int64) * 7919 + 1234
    ctx = Context(bench.VOCAB, do_lower_case=True)
    dev = ctx.device
    text = torch.from_numpy(corp.text).to(dev)
    so = torch.from_numpy(corp.sent_off).to(dev)
    dso = torch.from_numpy(corp.doc_sent_off).to(dev)
    po = torch.from_numpy(part).to(dev)
    ps = torch.from_numpy(seeds).to(dev)
    ids, sl = ctx.tokenize(text, so)
    lib = ctypes.CDLL(os.path.join(REPO, 'tools', 'ubench', 'libfiller.so'))
    sink = torch.zeros(1, dtype=torch.int32, device=dev)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    fs = torch.cuda.Stream()

    def pairs():
        pb = make_pairs(ctx, so, ids, sl, dso, po, ps, seq=128, dup=5, masking=True,
                        short_seq_prob=0.1, masked_lm_ratio=0.15)
        return pb.plan_ms

    def filler(iters, kind):
        fn = lib.ubench_valu_filler if kind == 'valu' else lib.ubench_salu_filler
        with torch.cuda.stream(fs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(fs)
            assert fn(ctypes.c_void_p(fs.cuda_stream), n_cu, iters, ctypes.c_void_p(sink.data_ptr())) == 0
            e1.record(fs)
        return e0, e1

    for _ in range(2):
        pairs()
    torch.cuda.synchronize()
    plan_alone = float(np.mean([pairs() for _ in range(3)]))
    out = {'batch_bytes': nbytes, 'planner_ms_alone': plan_alone}
    for kind in ('valu', 'salu'):
        # calibrate the filler to about the planner's time alone
        e0, e1 = filler(2000, kind)
        torch.cuda.synchronize()
        per_iter = e0.elapsed_time(e1) / 2000
        iters = max(1, int(plan_alone / per_iter))
        e0, e1 = filler(iters, kind)
        torch.cuda.synchronize()
        fill_alone = e0.elapsed_time(e1)
        # together: the filler first (one wave per SIMD on every CU), then the pair stage
        res = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0, e1 = filler(iters, kind)
            p = pairs()
            torch.cuda.synchronize()
            res.append((p, e0.elapsed_time(e1), (time.perf_counter() - t0) * 1e3))
        p_t, f_t, wall = (float(np.mean(x)) for x in zip(*res))
        out[kind] = {'filler_ms_alone': fill_alone, 'filler_iters': iters,
                     'filler_waves_per_simd': 1,
                     'together': {'planner_ms': p_t, 'filler_ms': f_t,
                                  'wall_ms_incl_pair_stage': wall},
                     'planner_slowdown': p_t / plan_alone, 'filler_slowdown': f_t / fill_alone}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
