"""End-to-end `preprocess_bert_pretrain` timing (SURVEY 8f2 / BASELINE C1): synthetic
`<id> <text>` documents written as the reference's source layout, then the CLI with
--profile-stages (device-synchronised seconds per stage: read = host file read + decode + line
split + doc corpus build, h2d, segment (GPU Punkt), tokenize, pairs, render, write (pyarrow)).

    python tools/cli_e2e.py --bytes 100e6 [--seq 128] [--bin-size N] [--num-blocks 128]
"""
import argparse
import json
import os
import shutil
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--bytes', type=float, default=100e6)
    ap.add_argument('--seq', type=int, default=128)
    ap.add_argument('--bin-size', type=int, default=None)
    ap.add_argument('--num-blocks', type=int, default=128)
    ap.add_argument('--masking', action='store_true', default=True)
    ap.add_argument('--files', type=int, default=16)
    ap.add_argument('--num-shards', type=int, default=None)
    ap.add_argument('--switch-interval', type=float, default=None,
                    help='sys.setswitchinterval for the run (GIL hand-off experiments)')
    a, extra = ap.parse_known_args()  # extra: passed to preprocess_bert_pretrain
    if a.switch_interval:
        sys.setswitchinterval(a.switch_interval)
    from lddl_amd import synth
    from lddl_amd.dask.bert import pretrain as P
    root = tempfile.mkdtemp(prefix='lddl_e2e_', dir=os.environ.get('TMPDIR', '/tmp'))
    try:
        t0 = time.perf_counter()
        text, doc_off = synth.generate_doc_text(seed=1234, n_bytes=int(a.bytes), nonascii_frac=0.01,
                                                threads=16)
        src = os.path.join(root, 'source', 'en')
        os.makedirs(src)
        n_doc = len(doc_off) - 1
        per = (n_doc + a.files - 1) // a.files
        for f in range(a.files):
            with open(os.path.join(src, 'wiki_{}.txt'.format(f)), 'wb') as fh:
                for d in range(f * per, min(n_doc, (f + 1) * per)):
                    fh.write(b'wiki-%d ' % d + text[doc_off[d]:doc_off[d + 1]].tobytes() + b'\n')
        gen_s = time.perf_counter() - t0
        src_bytes = sum(os.path.getsize(os.path.join(src, x)) for x in os.listdir(src))
        argv = ['--schedule', 'local', '--wikipedia', os.path.join(root, 'source'), '--sink',
                os.path.join(root, 'out'), '--target-seq-length', str(a.seq), '--num-blocks',
                str(a.num_blocks), '--vocab-file',
                os.path.join(REPO, 'lddl_amd', 'assets', 'vocab_synth_uncased_30522.txt'),
                '--profile-stages'] + (['--masking'] if a.masking else []) + (
                    ['--bin-size', str(a.bin_size)] if a.bin_size else []) + (
                    ['--num-shards', str(a.num_shards)] if a.num_shards else [])
        import torch  # noqa: F401  (first import outside the clock)
        import resource
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t1 = time.perf_counter()
        P.main(P.attach_args().parse_args(argv + extra))
        wall = time.perf_counter() - t1
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        out = os.path.join(root, 'out')
        out_bytes = sum(os.path.getsize(os.path.join(out, x)) for x in os.listdir(out))
        shards = None
        if a.num_shards:  # the balancer's contract: every bin's shards hold N or N+1 samples
            import pyarrow.parquet as pq
            with open(os.path.join(out, '.num_samples.json')) as f:
                ns = json.load(f)
            per_bin = {}
            for k, v in ns.items():
                assert pq.read_metadata(os.path.join(out, k)).num_rows == v, k
                per_bin.setdefault(k.rsplit('_', 1)[-1] if a.bin_size else '', []).append(v)
            spread = max(max(v) - min(v) for v in per_bin.values())
            assert spread <= 1 and all(len(v) == a.num_shards for v in per_bin.values())
            shards = {'files': len(ns), 'bins': len(per_bin), 'samples': sum(ns.values()),
                      'max_spread_per_bin': spread}
        print(json.dumps({'source_bytes': src_bytes, 'documents': n_doc, 'cli_wall_s': wall,
                          'source_MB_per_s': src_bytes / wall / 1e6, 'output_bytes': out_bytes,
                          'generate_s': gen_s, 'cpu_s': cpu_s, 'cpu_per_wall': cpu_s / wall,
                          'shards': shards,
                          'hbm_peak_reserved_gb': torch.cuda.max_memory_reserved() / 1e9,
                          'hbm_peak_allocated_gb': torch.cuda.max_memory_allocated() / 1e9,
                          'argv': argv[argv.index('--target-seq-length'):] + extra}))
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == '__main__':
    main()
