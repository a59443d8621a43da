"""Benchmark of the hot path on BASELINE.json's metric config (configs[1], "C2"):
synthetic English-like corpus, seq 128, static masking, no binning, on MI355X.
`--workload c4` runs configs[2]/[3] instead (seq 512 phase 2, static masking, 64 bins of 8
tokens, HBM load balance: at N > 1 an RCCL all-gather of per-bin counts and an all-to-all-v
sample exchange over xGMI, lddl_amd/balance.py).

One step = one pass of the hot path over one batch of synthetic input already resident in HBM:
WordPiece tokenization of the batch's (Punkt-segmented) sentences, then NSP pair construction with
duplicate_factor 5 and static MLM masking (CPython-exact `random` replay per partition), producing
the device-resident sample table (A/B token ids, num_tokens, is_random_next, masked positions and
labels). Every step recomputes everything from the text; nothing is cached between steps.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)

Multi-GPU: documents are sharded across ranks (each rank owns disjoint documents of the corpus and
its own partitions); the path has no data-path collective for C2, so `scaling` is "weak". At N > 1
the line also carries `c4_exchange`: one C4-style step per rank (seq 512, 64 bins, 8 x N shards)
through the load balance, i.e. the RCCL bin-count all-gather and all-to-all-v exchange.
value = sum over ranks of output tokens (sum of num_tokens, [CLS]/[SEP] included) / max rank time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

VOCAB = os.path.join(REPO, 'lddl_amd', 'assets', 'vocab_synth_uncased_30522.txt')
HBM_PEAK_GBS = 8000.0
BASELINE_ANCHOR_PER_CORE = 0.667e6  # reference functions, seq 128 + static masking  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def partition_docs(corp, partition_bytes):
    """Group consecutive documents into partitions of ~partition_bytes of text (the reference's
    Dask blocks, readers.py:48-67)."""
    doc_bytes = corp.sent_off[corp.doc_sent_off]
    cuts = np.searchsorted(doc_bytes, np.arange(0, doc_bytes[-1], partition_bytes), 'left')
    cuts = np.unique(np.concatenate([cuts, [corp.n_doc]]))
    if cuts[0] != 0:
        cuts = np.concatenate([[0], cuts])
    return cuts.astype(np.int64)


# LDDL_BENCH_SHARE_DEVICE=1: every rank on cuda:0 with gloo collectives (CPU tensors) - a rehearsal
# of the N > 1 bench logic on a one-GPU box; the driver's N > 1 runs use one GPU per rank + RCCL
SHARE_DEVICE = os.environ.get('LDDL_BENCH_SHARE_DEVICE') == '1'
RED_DEV = 'cpu' if SHARE_DEVICE else None


def launch_command(argv, env, n_devices, gpus):
    """`python bench.py --gpus N` with N > 1 and no launcher around it: the command that starts N
    fresh one-GPU ranks (torch.distributed.run, the reference's `mpirun -np` launch model,
    examples/local_example.sh:56-70). None when this process is already a rank (WORLD_SIZE set) or
    N == 1. Raises SystemExit when N exceeds the visible devices (unless LDDL_BENCH_SHARE_DEVICE=1,
    the one-GPU rehearsal) or disagrees with an outer launcher's WORLD_SIZE.

    Called before anything touches the GPU: the parent only counts devices (no HIP init on this
    image) and waits for the child; it never re-execs itself."""
    if 'WORLD_SIZE' in env:
        if int(env['WORLD_SIZE']) != gpus and gpus != 1:
            raise SystemExit('bench.py: --gpus {} but WORLD_SIZE={}'.format(gpus, env['WORLD_SIZE']))
        return None
    if gpus <= 1:
        return None
    if env.get('LDDL_BENCH_SHARE_DEVICE') != '1' and gpus > n_devices:
        raise SystemExit('bench.py: --gpus {} but only {} GPU(s) are visible'.format(gpus, n_devices))
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
            '--nproc-per-node', str(gpus), '--master-addr', '127.0.0.1', '--master-port', str(port),
            os.path.abspath(__file__)] + list(argv)


def make_batch(rank, args):
    from lddl_amd import synth
    corp = synth.generate(seed=args.seed, n_bytes=args.batch_bytes, doc_begin=rank * 50_000_000,
                          nonascii_frac=0.01, threads=args.gen_threads)
    part = partition_docs(corp, args.partition_bytes)
    # per-partition seeds for random.seed(); the reference leaves the worker RNG unseeded (H1)
    seeds = (np.arange(len(part) - 1, dtype=np.int64) + rank * 10_000_000) * 7919 + args.seed
    return corp, part, seeds


def st_moved_sum(x, world, dev):
    """Sum of a per-rank count over all ranks (gloo on the host in the shared-device
    rehearsal, RCCL otherwise)."""
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.int64, device=RED_DEV or dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return int(t.item())


def st_max(x, world, dev):
    """Max of a per-rank float over all ranks."""
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=RED_DEV or dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def partition_prefix(corp, part, max_bytes):
    """The number of leading whole partitions of `part` that hold at most max_bytes of text (at
    least one)."""
    doc_b = corp.sent_off[corp.doc_sent_off[part]]  # text byte at each partition boundary
    p1 = int(np.searchsorted(doc_b, doc_b[0] + max_bytes, 'right')) - 1
    return int(min(max(p1, 1), len(part) - 1))


def c4_exchange(args, ctx, dev, corp, part, seeds, text, world):
    """N > 1 beside the C2 headline (which has no data-path collective): one C4-style step on
    every rank — the rank's first ~args.exchange_bytes of text, seq 512, 64 bins of 8 tokens,
    balanced into 8 x N shards by StreamBalancer — so that a scaling run also measures the two
    collectives north_star names: the per-bin count all-gather and the all-to-all-v of the rows
    over each rank's shard quota (RCCL over xGMI; gloo through host tensors in the one-GPU
    rehearsal). One warm-up step, then one measured step; times are the max over ranks."""
    from lddl_amd.balance import StreamBalancer
    from lddl_amd.pairs import make_pairs
    p1 = partition_prefix(corp, part, args.exchange_bytes)
    d1 = int(part[p1])
    s1 = int(corp.doc_sent_off[d1])
    b1 = int(corp.sent_off[s1])
    up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    sent_off, doc_off = up(corp.sent_off[:s1 + 1]), up(corp.doc_sent_off[:d1 + 1])
    part_off, part_seed = up(part[:p1 + 1]), up(seeds[:p1])
    S = 8 * world
    out = None
    for it in range(2):
        ids, sl = ctx.tokenize(text[:b1], sent_off)
        pb = make_pairs(ctx, sent_off, ids, sl, doc_off, part_off, part_seed, seq=512, dup=5,
                        masking=True, short_seq_prob=0.1, masked_lm_ratio=0.15)
        del ids, sl
        sb = StreamBalancer(ctx, 8, 64, num_shards=S)
        tm = {}
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        bb = sb.step(pb, timings=tm)
        if it == 1:
            out = {
                'workload': 'C4-style exchange step beside the C2 headline: each rank\'s first '
                            'partitions (~{} MB of text), seq 512, duplicate_factor 5, static '
                            'masking, 64 bins of 8 tokens, StreamBalancer into {} shards'.format(
                                args.exchange_bytes // 10 ** 6, S),
                'backend': dist.get_backend() if world > 1 else None,
                'text_bytes_per_rank_max': int(st_max(float(b1), world, dev)),
                'rows': st_moved_sum(int(pb.n_pairs), world, dev),
                'moved_rows': st_moved_sum(int(bb.moved_rows), world, dev),
                'counts_allgather_and_plan_ms': st_max((tm['plan'] - tm['bin']) * 1e3, world, dev),
                'exchange_ms': st_max((tm['exchange'] - tm['plan']) * 1e3, world, dev),
                'balance_ms': st_max((tm['regroup'] - tm['start']) * 1e3, world, dev),
                'num_shards': S,
                'shard_counts_spread': int((sb.all_shard_counts.max(0) -
                                            sb.all_shard_counts.min(0)).max()),
                'note': 'moved_rows: rows received from other ranks (only the per-bin surplus over '
                        'each rank\'s shard quota moves, balance.py); exchange_ms: the all-to-all-v '
                        'of row metadata and the token / position / label columns; not part of '
                        'value'}
        del bb, pb, sb
    return out


def granted_cores():
    """Host cores this process may actually use: the CPU affinity mask, capped by the cgroup CPU
    quota (cgroup v2 cpu.max, else v1 cfs_quota_us / cfs_period_us). os.cpu_count() reports the
    whole machine. Returns (cores, derivation string)."""
    import math
    aff = len(os.sched_getaffinity(0))
    quota, src = None, 'none'
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, p = f.read().split()[:2]
        if q != 'max':
            quota, src = int(q) / int(p), 'cgroup v2 cpu.max {}/{}'.format(q, p)
    except (OSError, ValueError):
        try:
            with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as f:
                q = int(f.read())
            with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as f:
                p = int(f.read())
            if q > 0:
                quota, src = q / p, 'cgroup v1 cfs quota {}/{}'.format(q, p)
        except (OSError, ValueError):
            pass
    cores = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    return cores, 'sched_getaffinity = {}, CPU quota = {} ({}), os.cpu_count() = {}'.format(
        aff, 'none' if quota is None else '{:g}'.format(quota), src, os.cpu_count())


def load_pmc(batch_sizes):
    """Per-kernel counters per launch from the committed PMC passes (profiles/pmc_*.json, made by
    tools/prof_counters.sh + tools/make_pmc_json.py) taken on one of `batch_sizes` (requested or
    actual bytes); the last such file in name order wins. Returns (kernels, file name, the pass's
    build id and git head)."""
    import glob
    kernels, src, meta = {}, None, {}
    for pmc in sorted(glob.glob(os.path.join(REPO, 'profiles', 'pmc_*.json'))):
        try:
            with open(pmc) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if rec.get('batch_bytes') in batch_sizes:
            kernels, src = rec.get('kernels', {}), os.path.basename(pmc)
            meta = {k: rec.get(k) for k in ('build_id', 'git_head')}
    return kernels, src, meta


def pmc_entry(kernels, kernel):
    """A kernel's counters per step by name: template instantiations (`name<...>`) match their base
    name and are summed (the tokenizer runs as a memo-building and a memo-reading launch per
    call, tokenize_batch_kernel<1> and <2>)."""
    out = {}
    for k, v in kernels.items():
        if k == kernel or k.startswith(kernel + '<'):
            for n, x in v.items():
                if isinstance(x, (int, float)) and not isinstance(x, bool):
                    out[n] = out.get(n, 0) + x
                else:
                    out.setdefault(n, x)
    return out


def cgroup_cpu_stat():
    """cgroup v2 cpu.stat counters (usage_usec, nr_throttled, throttled_usec, ...) or {}."""
    try:
        with open('/sys/fs/cgroup/cpu.stat') as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return {}


def cpu_baseline(corp, part, seeds, args):
    """The oracle (C restatement of the reference algorithm) on a bounded sample of the same
    workload, one single-threaded process per granted host core (the reference's
    Dask/mpi4py pipeline runs one single-threaded worker per core): worker w takes its own run
    of ~cpu_sample_bytes of consecutive partitions. value = all workers' output tokens / wall."""
    import multiprocessing as mp
    from oracle.cpu_worker import cpu_worker
    cores, derivation = granted_cores()
    n_proc = max(1, cores if args.cpu_procs is None else min(args.cpu_procs, cores))
    doc_bytes = corp.sent_off[corp.doc_sent_off]
    jobs, p0 = [], 0
    for _ in range(n_proc):
        p1 = int(np.searchsorted(doc_bytes[part], doc_bytes[part[p0]] + args.cpu_sample_bytes))
        p1 = min(max(p1, p0 + 1), len(part) - 1)
        if p1 <= p0:
            break
        d0, d1 = part[p0], part[p1]
        s0, s1 = corp.doc_sent_off[d0], corp.doc_sent_off[d1]
        b0, b1 = corp.sent_off[s0], corp.sent_off[s1]
        jobs.append((corp.text[b0:b1].copy(), corp.sent_off[s0:s1 + 1] - b0,
                     corp.doc_sent_off[d0:d1 + 1] - s0, part[p0:p1 + 1] - d0, seeds[p0:p1].copy(),
                     args.seq, VOCAB))
        p0 = p1
    with mp.get_context('spawn').Pool(len(jobs)) as pool:  # workers import numpy + oracle only
        warm = [(j[0][:1 << 16], j[1][:2], j[2][:2], j[3][:1] * 0, j[4][:0], j[5], j[6])
                for j in jobs]
        pool.map(cpu_worker, warm, chunksize=1)  # imports and vocab load before the clock
        t0 = time.perf_counter()
        res = pool.map(cpu_worker, jobs)
        wall = time.perf_counter() - t0
    n_out = sum(r[0] for r in res)
    mb = sum(len(j[0]) for j in jobs) / 1e6
    model = None
    try:
        with open('/proc/cpuinfo') as f:
            model = next((l.split(':', 1)[1].strip() for l in f if l.startswith('model name')),
                         None)
    except OSError:
        pass
    per_core = n_out / wall / len(jobs)
    return {'value': n_out / wall, 'unit': 'output tokens/s', 'cores': len(jobs), 'kind': 'port',
            'per_core': per_core, 'cpu_model': model,
            'vs_anchor': per_core / BASELINE_ANCHOR_PER_CORE,
            'anchor_note': ('BASELINE.md anchor: the reference\'s own functions (HF tokenizers, '
                            'Python pairs/masking) at 0.667 M output tokens/s/core, seq 128 + '
                            'static masking. This port (C, -O2) is {:.0f}x faster per core, far '
                            'outside the +-25% band SURVEY 8d asks for: it is a stronger baseline '
                            'than the reference, not a timing of it (the reference cannot run on '
                            'the GPU box)').format(per_core / BASELINE_ANCHOR_PER_CORE),
            'granted_cores': cores, 'os_cpu_count': os.cpu_count(),
            'sample': '{} single-threaded processes (one per granted core: {}) x ~{:.0f} MB of '
                      'consecutive partitions = {:.1f} MB of the same synthetic batch (tokenize + '
                      'pairs + static masking, oracle/lddl_oracle.c), {:.1f} s wall'.format(
                          len(jobs), derivation, args.cpu_sample_bytes / 1e6, mb, wall)}


def timed_segmented(args, rank, world, ctx, dev, params=None):
    """The step from raw document text (what the reference hands to sent_tokenize,
    pretrain.py:86): GPU Punkt segmentation -> WordPiece -> pairs + static masking, same
    synthetic documents (sentences joined by spaces). params None: the untrained parameters
    (what offline nltk runs, segment_eval_kernel<false>); else a PunktParams (trained model:
    abbreviations, collocations, sentence starters, orthographic context — the English-model
    configuration of the reference, segment_eval_kernel<true>)."""
    from lddl_amd import punkt, synth
    from lddl_amd.pairs import make_pairs
    text, doc_off = synth.generate_doc_text(seed=args.seed, n_bytes=args.batch_bytes,
                                            doc_begin=rank * 50_000_000, nonascii_frac=0.01,
                                            threads=args.gen_threads)
    cuts = np.searchsorted(doc_off, np.arange(0, doc_off[-1], args.partition_bytes), 'left')
    part = np.unique(np.concatenate([[0], cuts, [len(doc_off) - 1]])).astype(np.int64)
    seeds = (np.arange(len(part) - 1, dtype=np.int64) + rank * 10_000_000) * 7919 + args.seed
    d_text = torch.from_numpy(text).to(dev)
    d_doc = torch.from_numpy(doc_off).to(dev)
    d_part = torch.from_numpy(part).to(dev)
    d_seed = torch.from_numpy(seeds).to(dev)
    punkt.set_params(ctx, params)
    info = {}

    def step(ev=None):
        if ev is not None:
            ev[0].record()
        so, ds = punkt.segment(ctx, d_text, d_doc)
        if ev is not None:
            ev[1].record()
        ids, sl = ctx.tokenize(d_text, so)
        pb = make_pairs(ctx, so, ids, sl, ds, d_part, d_seed, seq=args.seq, dup=5, masking=True,
                        short_seq_prob=0.1, masked_lm_ratio=0.15, rng=args.rng)
        del ids, sl
        if args.workload in ('c3', 'c4'):
            from lddl_amd.balance import balance
            bb = balance(ctx, pb, 8, args.seq // 8, num_shards=args.num_shards or 8)
            n = bb.n_tokens + 3 * bb.n_rows
            del bb
        else:
            n = int(pb.tokens.numel()) + 3 * pb.n_pairs
        info['sentences'] = int(so.numel()) - 1
        del pb, so, ds
        return n
    for _ in range(args.warmup):
        step()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n_tok = 0
    for k in range(args.steps):
        n_tok += step(evs[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt, float(n_tok)], dtype=torch.float64, device=RED_DEV or dev)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dt, n_tok = float(t[0].item()), int(t[1].item())
    seg_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    # segmentation algorithmic bytes: text read once + document offsets read + sentence offsets
    # and document sentence offsets written
    n_doc = len(doc_off) - 1
    seg_bytes = len(text) + 8 * (n_doc + 1) + 8 * (info['sentences'] + 1) + 8 * (n_doc + 1)
    seg_gbs = seg_bytes / (seg_ms * 1e-3) / 1e9
    return {'value': n_tok / dt, 'unit': 'output tokens/s', 'ms_per_step': dt / args.steps * 1e3,
            'segment_ms': seg_ms, 'segment_text_gbs': len(text) / (seg_ms * 1e-3) / 1e9,
            'roofline_segment': {'kernel': 'segment_classify + segment_eval + flatten + fill (HIP '
                                            'events around lddl_segment_count/fill, 2 host syncs)',
                                 'bound': 'hbm', 'achieved': seg_gbs, 'peak': HBM_PEAK_GBS,
                                 'unit': 'GB/s', 'frac': seg_gbs / HBM_PEAK_GBS,
                                 'algorithmic_bytes_per_launch': seg_bytes},
            'documents': int(len(doc_off) - 1), 'sentences': info['sentences'],
            'batch_bytes': int(len(text)),
            'note': 'input = raw document text; segment_ms includes the host sync for the '
                    'sentence count (lddl_segment_count)'}


VOCAB_CASED = os.path.join(REPO, 'lddl_amd', 'assets', 'vocab_synth_cased_28996.txt')


def c5_dataset(args, root):
    """C3-style binned, balanced parquet output (seq 512, bins of --c5-bin-size, no static
    masking) made by the product CLI (preprocess_bert_pretrain --num-shards) from synthetic
    documents, cased 28,996-piece vocab: the input of get_bert_pretrain_data_loader."""
    from lddl_amd import synth
    from lddl_amd.dask.bert import pretrain as P
    text, doc_off = synth.generate_doc_text(seed=args.seed, n_bytes=args.c5_corpus_bytes,
                                            nonascii_frac=0.01, threads=args.gen_threads)
    src = os.path.join(root, 'source', 'en')
    os.makedirs(src)
    n_doc = len(doc_off) - 1
    per = (n_doc + 7) // 8
    for f in range(8):
        with open(os.path.join(src, 'wiki_{}.txt'.format(f)), 'wb') as fh:
            for d in range(f * per, min(n_doc, (f + 1) * per)):
                fh.write(b'wiki-%d ' % d + text[doc_off[d]:doc_off[d + 1]].tobytes() + b'\n')
    sink = os.path.join(root, 'out')
    argv = ['--schedule', 'local', '--wikipedia', os.path.join(root, 'source'), '--sink', sink,
            '--target-seq-length', '512', '--bin-size', str(args.c5_bin_size), '--num-blocks', '64',
            '--vocab-file', VOCAB_CASED, '--num-shards', str(max(1, args.c5_workers)),
            '--sample-ratio', '1.0']
    P.main(P.attach_args().parse_args(argv))
    return sink


class TinyBert(torch.nn.Module):
    """A small BERT-shaped model for the C5 training step (the reference's harness only iterates
    the loader, benchmarks/torch_train.py:146-184; north_star config 5 feeds a training step):
    token + type + position embeddings, LayerNorm, one MLP block, MLM head on the masked slots
    (labels != ignore_index), NSP head on [CLS]."""

    def __init__(self, vocab, hidden=768, seq=512):
        super().__init__()
        self.tok = torch.nn.Embedding(vocab, hidden)
        self.typ = torch.nn.Embedding(2, hidden)
        self.pos = torch.nn.Embedding(seq, hidden)
        self.norm = torch.nn.LayerNorm(hidden)
        self.mlp = torch.nn.Sequential(torch.nn.Linear(hidden, 4 * hidden), torch.nn.GELU(),
                                       torch.nn.Linear(4 * hidden, hidden))
        self.mlm = torch.nn.Linear(hidden, vocab)
        self.nsp = torch.nn.Linear(hidden, 2)

    def forward(self, b, ignore_index=-1, mlm_cap=0.2):
        """No host syncs: the MLM head runs on a fixed number of slots (mlm_cap of the batch,
        above the 0.15 masking rate), the masked ones first (stable sort of the label mask);
        unmasked slots among them carry ignore_index and drop out of the loss."""
        ids = b['input_ids']
        L = ids.size(1)
        h = self.tok(ids) + self.typ(b['token_type_ids']) + self.pos.weight[:L][None]
        h = self.norm(h) * b['attention_mask'][..., None]
        h = h + self.mlp(h)
        lab = b['labels'].reshape(-1)
        k = max(1, int(mlm_cap * lab.numel()))
        idx = torch.sort((lab != ignore_index).to(torch.int8), descending=True,
                         stable=True).indices[:k]
        hs = h.reshape(-1, h.size(-1)).index_select(0, idx)
        mlm = torch.nn.functional.cross_entropy(self.mlm(hs).float(), lab.index_select(0, idx),
                                                ignore_index=ignore_index)
        nsp = torch.nn.functional.cross_entropy(self.nsp(h[:, 0]).float(),
                                                b['next_sentence_labels'])
        return mlm + nsp


def run_c5(args):
    """C5: online dynamic masking in get_bert_pretrain_data_loader's collate, batch 256 x seq
    512, cased vocab, fed to a PyTorch-ROCm training step. value = real (attended) token slots
    per second through loader + collate + masking + training step."""
    import logging
    import shutil
    import tempfile
    from lddl_amd.torch import get_bert_pretrain_data_loader
    root = tempfile.mkdtemp(prefix='lddl_c5_', dir=os.environ.get('TMPDIR', '/tmp'))
    try:
        t0 = time.perf_counter()
        path = c5_dataset(args, root)
        prep_s = time.perf_counter() - t0
        dl = get_bert_pretrain_data_loader(
            path, local_rank=0, vocab_file=VOCAB_CASED,
            data_loader_kwargs=dict({'batch_size': 256, 'num_workers': args.c5_workers},
                                    **({'prefetch_factor': 4} if args.c5_workers else {}),
                                    **({'multiprocessing_context': args.c5_mp}
                                       if args.c5_workers and args.c5_mp != 'fork' else {})),
            mlm_probability=0.15, base_seed=args.seed, log_level=logging.WARNING,
            sequence_length_alignment=8, ignore_index=-1)
        loaders = getattr(dl, '_dataloaders', [dl])

        def batches():
            while True:
                for b in dl:
                    yield b
        it = batches()
        dev = torch.device('cuda', 0)
        if args.c5_blas != 'default':  # ('cublas' selects rocBLAS on ROCm)
            torch.backends.cuda.preferred_blas_library('cublas' if args.c5_blas == 'rocblas' else 'cublaslt')
        with open(VOCAB_CASED, 'rb') as f:  # (not loaders[0]._ctx: that would create the
            n_vocab = sum(1 for _ in f)        # loader's Context before its workers start)
        model = TinyBert(n_vocab).to(dev)
        params = list(model.parameters())

        def sgd_step(lr=1e-4):
            # plain SGD as one fused foreach update (torch.optim.SGD spent ~150 ms of host time
            # per step here: profiles/r03c5_workers_train_step.txt)
            with torch.no_grad():
                torch._foreach_add_(params, [q.grad for q in params], alpha=-lr)
            for q in params:
                q.grad = None

        phase_s = [0.0, 0.0, 0.0]  # host seconds in forward / backward / optimizer (no syncs)

        pad_mult = 64

        def padded(b):
            # the step's input padded to a multiple of 64 positions (the loader's batches come in
            # up to 64 lengths; every new length loads new GEMM code objects - 40-135 ms of
            # hipModuleLoad each, profiles/r03h_c5_hip_api.txt - and 8 shapes are warmed up below)
            L = b['input_ids'].size(1)
            Lp = -(-L // pad_mult) * pad_mult
            if Lp == L:
                return b
            out = dict(b)
            for k_ in ('input_ids', 'token_type_ids', 'attention_mask'):
                out[k_] = torch.nn.functional.pad(b[k_], (0, Lp - L), value=0)
            out['labels'] = torch.nn.functional.pad(b['labels'], (0, Lp - L), value=-1)
            return out

        def train(b):
            b = padded(b)
            p0 = time.perf_counter()
            with torch.autocast('cuda', dtype=torch.bfloat16):
                loss = model(b)
            p1 = time.perf_counter()
            loss.backward()
            p2 = time.perf_counter()
            sgd_step()
            p3 = time.perf_counter()
            phase_s[0] += p1 - p0
            phase_s[1] += p2 - p1
            phase_s[2] += p3 - p2
            return loss

        def timed(k_steps, with_train):
            for x in loaders:
                x.stats = dict(pack_s=[], blob_bytes=[], events=[], slots=[])
            torch.cuda.synchronize()
            real = torch.zeros((), dtype=torch.int64, device=dev)
            slots = 0
            t = time.perf_counter()
            tw = tn = 0.0
            gev = []
            timed.kept = []
            for _ in range(k_steps):
                n0 = time.perf_counter()
                b = next(it)
                tn += time.perf_counter() - n0
                if with_train:  # the same batches are replayed by train_step_alone
                    timed.kept.append(b)
                real += b['attention_mask'].sum()
                slots += b['input_ids'].numel()
                if with_train:
                    w0 = time.perf_counter()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    train(b)
                    e1.record()
                    gev.append((e0, e1))
                    tw += time.perf_counter() - w0
            torch.cuda.synchronize()
            gms = [a.elapsed_time(z) for a, z in gev]
            timed.gpu_ms = float(np.mean(gms)) if gev else None
            timed.gpu_ms_pct = ([round(float(np.percentile(gms, q)), 2) for q in (50, 90, 100)]
                                if gev else None)
            dt = time.perf_counter() - t
            st = {k: sum((x.stats[k] for x in loaders), []) for k in loaders[0].stats}
            for x in loaders:
                x.stats = None
            return dt, int(real.item()), slots, st, tw, tn

        for Lp in range(pad_mult, 512 + 1, pad_mult):  # every padded shape, before timing
            z = torch.zeros(256, Lp, dtype=torch.long, device=dev)
            lab = torch.full((256, Lp), -1, dtype=torch.long, device=dev)
            lab[:, 1::7] = 5
            for _ in range(2):
                train({'input_ids': z, 'token_type_ids': z, 'attention_mask': z + 1, 'labels': lab,
                       'next_sentence_labels': torch.zeros(256, dtype=torch.long, device=dev)})
        for _ in range(args.warmup):
            train(next(it))
        phase_s[:] = [0.0, 0.0, 0.0]
        import gc
        gc_t = {'s': 0.0, 'n': 0, 't0': 0.0}

        def gc_cb(phase, info):  # time the main process spends in Python's garbage collector
            if phase == 'start':
                gc_t['t0'] = time.perf_counter()
            else:
                gc_t['s'] += time.perf_counter() - gc_t['t0']
                gc_t['n'] += 1
        gc.callbacks.append(gc_cb)
        m0 = torch.cuda.memory_stats()
        c0 = cgroup_cpu_stat()
        dt, real, slots, st, tw, tn = timed(args.steps, True)
        c1 = cgroup_cpu_stat()
        gc.callbacks.remove(gc_cb)
        m1 = torch.cuda.memory_stats()
        cg = {k: c1[k] - c0.get(k, 0) for k in ('usage_usec', 'nr_periods', 'nr_throttled',
                                                  'throttled_usec') if k in c1}
        train_gpu_ms, train_gpu_pct = timed.gpu_ms, timed.gpu_ms_pct
        # the same training step alone: the timed loop's own batches (same shapes, same order),
        # already resident in HBM, no loader in the loop - what the step costs when nothing else
        # runs beside it. (Round 4 replayed 8 other batches: their padded lengths, not the loader,
        # made that figure differ from the in-loop step.)
        res_b = timed.kept
        timed.kept = []
        torch.cuda.synchronize()
        ra = []
        t_alone = time.perf_counter()
        for i in range(args.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            train(res_b[i % len(res_b)])
            e1.record()
            ra.append((e0, e1))
        torch.cuda.synchronize()
        t_alone = time.perf_counter() - t_alone
        alone_gms = [a.elapsed_time(z) for a, z in ra]
        padded_len_mean = float(np.mean([-(-x['input_ids'].size(1) // pad_mult) * pad_mult
                                         for x in res_b]))
        del res_b
        host_phases = {k: round(v / args.steps * 1e3, 3) for k, v in
                       zip(('forward', 'backward', 'optimizer'), phase_s)}
        dev_allocs = int(m1.get('num_device_alloc', 0) - m0.get('num_device_alloc', 0))
        dev_frees = int(m1.get('num_device_free', 0) - m0.get('num_device_free', 0))
        ldt, lreal, lslots, lst, _, _ = timed(args.steps, False)
        kern_ms = [e[0].elapsed_time(e[1]) for e in lst['events']]
        # algorithmic bytes of the fused collate kernel per launch: the A/B strings read once +
        # input_ids, token_type_ids, attention_mask, labels written once (4 x 8 B per slot)
        alg = [bb + 32 * n for bb, n in zip(lst['blob_bytes'], lst['slots'])]
        k_ms = float(np.mean(kern_ms))
        ach = float(np.mean(alg)) / (k_ms * 1e-3) / 1e9
        return {
            'metric': 'WordPiece+MLM tokens/sec (1/2/4/8 MI355X) and % of HBM roofline',
            'value': lreal / ldt,
            'unit': 'real token slots/s (attention_mask = 1) delivered by get_bert_pretrain_data_'
                    'loader (parquet decode + shuffle buffer + collate + dynamic masking)',
            'n_gpus': 1, 'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': ldt / args.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': None, 'dtype': 'int64', 'data': 'synthetic',
            'config': {'workload': 'C5: get_bert_pretrain_data_loader, batch 256 x seq 512 '
                                   '(sequence_length_alignment 8), dynamic masking 0.15, cased '
                                   '28,996 vocab, {} bins of {} tokens, {} workers per bin; input '
                                   '= preprocess_bert_pretrain --num-shards output of {} MiB of '
                                   'synthetic documents'.format(
                                       512 // args.c5_bin_size, args.c5_bin_size,
                                       args.c5_workers, args.c5_corpus_bytes >> 20),
                       'global_batch': 256, 'seq_len': 512, 'parallelism': 'dp1 (replicas)'},
            'padded_slots_per_s': lslots / ldt,
            'with_training_step': {
                'value': real / dt, 'ms_per_step': dt / args.steps * 1e3,
                'padded_slots_per_s': slots / dt,
                'loader_wait_ms_per_step': tn / args.steps * 1e3,
                'train_step_host_ms': tw / args.steps * 1e3,
                'train_step_gpu_ms': train_gpu_ms,
                'train_step_gpu_ms_p50_p90_max': train_gpu_pct,
                'train_step_alone': {
                    'ms_per_step': t_alone / args.steps * 1e3,
                    'gpu_ms': float(np.mean(alone_gms)),
                    'gpu_ms_p50_p90_max': [round(float(np.percentile(alone_gms, q)), 2)
                                           for q in (50, 90, 100)],
                    'padded_len_mean': padded_len_mean,
                    'note': 'the same step replayed on the timed loop\'s own batches (same '
                            'shapes and order), HBM-resident, no loader in the loop'},
                'worker_start_method': args.c5_mp,
                'pinned_stager_allocations': loaders[0]._stager.allocations,
                'train_step_host_ms_by_phase': host_phases,
                'device_mallocs_frees_in_timed_steps': [dev_allocs, dev_frees],
                'cgroup_cpu_stat_delta': cg,  # CPU quota throttling of the container while timed
                'python_gc_ms_per_step': round(gc_t['s'] / args.steps * 1e3, 3),
                'python_gc_collections': gc_t['n'],
                'host_cpus_granted': granted_cores()[0],
                'dataloader_processes': len(loaders) * args.c5_workers,
                'note': 'each batch feeds a bf16 TinyBert training step (embeddings + LayerNorm + '
                        'MLP + MLM/NSP heads, SGD) with no host sync inside the step: the '
                        'pipeline runs at the step\'s GPU pace (train_step_gpu_ms, HIP events '
                        'around the step; the host launches run ahead until the queue fills, '
                        'so train_step_host_ms follows it); loader_wait_ms_per_step is the host '
                        'time the training loop spends in next(loader) (the data stall)'},
            'host_pack_ms_per_batch': float(np.mean(lst['pack_s'])) * 1e3,
            'collate_kernel_us': k_ms * 1e3,
            'roofline': {'kernel': 'encode_kernel (lddl_collate_encode_masked: collate + '
                                   'dynamic masking fused)', 'bound': 'hbm', 'achieved': ach,
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': ach / HBM_PEAK_GBS,
                         'traffic': None,
                         'algorithmic_bytes_per_launch': float(np.mean(alg)),
                         'note': 'A/B string bytes + 32 B per [B, L] slot (SURVEY 8d: 36 B/slot '
                                 'with 4-B ids); a ~5 MB launch is latency-bound, not HBM-bound'},
            'dataset_prep_s': prep_s,
        }
    finally:
        shutil.rmtree(root, ignore_errors=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=None,
                    help='timed steps (default 5; c5: 200 batches, so that the 8 bin loaders\' '
                         'worker start-up and shuffle-buffer fill stay outside the rate)')
    ap.add_argument('--warmup', type=int, default=None, help='untimed steps (default 1; c5: 20)')
    ap.add_argument('--batch-bytes', type=int, default=None,
                    help='sentence text per GPU per step (default: the 10 GB corpus of C2 in one '
                         'step, HBM-resident; 4 GiB for c4, for HBM headroom of the balance)')
    ap.add_argument('--partition-bytes', type=int, default=1 << 20)
    ap.add_argument('--seq', type=int, default=None)
    ap.add_argument('--workload', choices=['c2', 'c3', 'c4', 'c5'], default='c2')
    ap.add_argument('--sub-batch-bytes', type=int, default=10_000_000_000,
                    help='c3/c4: the resident corpus streams through tokenize -> pairs -> balance '
                         'in sub-batches of about this many text bytes (one batch\'s tables in '
                         'HBM at a time; balance state carried across them)')
    ap.add_argument('--num-shards', type=int, default=None,
                    help='c3/c4: balanced shards (default 8 per rank)')
    ap.add_argument('--c5-corpus-bytes', type=int, default=96 << 20)
    ap.add_argument('--c5-bin-size', type=int, default=64,
                    help='C5 loader bins (64 -> 8 bins, the reference example local_example.sh)')
    ap.add_argument('--c5-blas', choices=('default', 'rocblas', 'hipblaslt'), default='default',
                    help='c5: GEMM library of the training step (torch preferred_blas_library)')
    ap.add_argument('--c5-workers', type=int, default=2,
                    help='DataLoader workers per bin (= shards per bin of the C5 dataset)')
    ap.add_argument('--c5-mp', choices=('fork', 'forkserver', 'spawn'), default='fork',
                    help='c5: start method of the DataLoader workers (multiprocessing_context)')
    ap.add_argument('--chunks', type=int, default=1,
                    help='c2: split the step into partition-aligned chunks, tokenizing chunk k+1 '
                         'on a side stream under chunk k\'s pair planner')
    ap.add_argument('--seed', type=int, default=1234)
    ap.add_argument('--gen-threads', type=int, default=16)
    ap.add_argument('--cpu-sample-bytes', type=int, default=48 << 20)
    ap.add_argument('--cpu-procs', type=int, default=None,
                    help='CPU baseline processes (default: one per granted host core, '
                         'granted_cores(); a value above the grant is capped to it)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-alt-rng', dest='alt_rng', action='store_false',
                    help='skip timing the other RNG mode (reported as alt_rng)')
    ap.add_argument('--no-extra-lines', dest='extra_lines', action='store_false',
                    help='skip the PCIe-inclusive and reference-partitioning lines (c2)')
    ap.add_argument('--no-segmented-line', dest='segmented_line', action='store_false',
                    help='skip timing the raw-document input (GPU Punkt segmentation in the step)')
    ap.add_argument('--punkt-params', default=os.path.join(REPO, 'tests', 'golden',
                                                           'punkt_params.json'),
                    help='PunktParameters JSON for the trained-model segmentation line '
                         '(with_segmentation.trained); empty string skips it')
    ap.add_argument('--exchange-bytes', type=int, default=3_000_000_000,
                    help='c2 at N > 1: text per rank of the c4_exchange sub-line (one C4-style '
                         'balance step over RCCL beside the headline)')
    ap.add_argument('--no-exchange-line', dest='exchange_line', action='store_false',
                    help='c2 at N > 1: skip the c4_exchange sub-line')
    ap.add_argument('--rng', choices=['replay', 'native'], default='replay',
                    help='replay: CPython MT19937 per partition, bit-exact with the reference; '
                         'native: Philox counter RNG, documents and pairs in parallel')
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 200 if args.workload == 'c5' else 5
    if args.warmup is None:
        args.warmup = 20 if args.workload == 'c5' else 1
    if args.seq is None:
        args.seq = 128 if args.workload == 'c2' else 512
    if args.batch_bytes is None:
        # C2 / C3: the whole 10 GB corpus of BASELINE configs[1] / configs[2] per step; C4: the
        # 200 GB corpus of configs[3] over 8 GPUs = 25 GB of text per GPU
        args.batch_bytes = 25_000_000_000 if args.workload == 'c4' else 10_000_000_000
        if SHARE_DEVICE and args.gpus > 1:  # all ranks share one GPU's HBM in the rehearsal
            args.batch_bytes = min(args.batch_bytes, 2 << 30)
    args.exchange_bytes = min(args.exchange_bytes, args.batch_bytes)

    if args.workload == 'c5' and args.gpus > 1:
        raise SystemExit('C5 is measured per replica (--gpus 1)')
    cmd = launch_command(sys.argv[1:], os.environ, torch.cuda.device_count(), args.gpus)
    if cmd is not None:  # N fresh one-GPU ranks; rank 0 prints the JSON line
        import subprocess
        sys.stdout.flush()
        raise SystemExit(subprocess.call(cmd, env=dict(os.environ)))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.workload == 'c5':
        print(json.dumps(run_c5(args)), flush=True)
        return
    if world > 1:
        if SHARE_DEVICE:  # rehearsal of the multi-rank path on a one-GPU box (never the driver's run)
            torch.cuda.set_device(0)
            dist.init_process_group('gloo')
        else:
            torch.cuda.set_device(local)
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    from lddl_amd._native import lib
    from lddl_amd.context import Context
    from lddl_amd.pairs import make_pairs
    from lddl_amd.balance import balance

    corp, part, seeds = make_batch(rank, args)
    ctx = Context(VOCAB, do_lower_case=True)
    dev = ctx.device
    text = torch.from_numpy(corp.text).to(dev)
    sent_off = torch.from_numpy(corp.sent_off).to(dev)
    doc_off = torch.from_numpy(corp.doc_sent_off).to(dev)
    base = dict(text=text, sent_off=sent_off, part_off=torch.from_numpy(part).to(dev),
                part_seed=torch.from_numpy(seeds).to(dev))

    diag = {}  # {'balance': {}}: balance() records synchronised phase times (untimed step only)
    stream = args.workload in ('c3', 'c4')
    n_shards = args.num_shards or 8 * world
    subs = None
    if stream:  # the resident corpus in K sub-batches of whole partitions (offsets rebased once)
        K = max(1, -(-args.batch_bytes // args.sub_batch_bytes))
        doc_b = corp.sent_off[corp.doc_sent_off[part]]
        pc = np.unique(np.searchsorted(doc_b, np.arange(K + 1) * doc_b[-1] / K, 'left'))
        pc[-1] = len(part) - 1
        subs = []
        for p0, p1 in zip(pc[:-1], pc[1:]):
            d0, d1 = part[p0], part[p1]
            s0, s1 = corp.doc_sent_off[d0], corp.doc_sent_off[d1]
            b0, b1 = corp.sent_off[s0], corp.sent_off[s1]
            up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
            subs.append(dict(text=text[b0:b1], sent_off=up(corp.sent_off[s0:s1 + 1] - b0),
                             doc_off=up(corp.doc_sent_off[d0:d1 + 1] - s0),
                             part_off=up(part[p0:p1 + 1] - d0), part_seed=up(seeds[p0:p1])))

    def record(ev, i):
        if ev is not None:
            if i == 0:
                ev.append([torch.cuda.Event(enable_timing=True) for _ in range(3)])
            ev[-1][i].record()

    def step(ev=None, rng=args.rng, b=None):
        """ev: list that collects one (start, tokenized, paired) event triple per (sub-)batch."""
        b = base if b is None else b
        if args.chunks > 1 and args.workload == 'c2':
            return step_chunked(ev, rng, b)
        sb = None
        if stream:
            from lddl_amd.balance import StreamBalancer
            sb = StreamBalancer(ctx, 8, args.seq // 8, num_shards=n_shards)
        n_tok = 0
        st = {'pairs': 0, 'masked': 0, 'plan_ms': 0.0, 'tokens': 0, 'kept_sent': 0,
              'kept_doc': 0, 'moved_rows': 0}
        sent_lens = []
        for sub in (subs if stream else [dict(b, doc_off=doc_off)]):
            record(ev, 0)
            ids, sent_len = ctx.tokenize(sub['text'], sub['sent_off'])
            sent_lens.append(sent_len)
            record(ev, 1)
            pb = make_pairs(ctx, sub['sent_off'], ids, sent_len, sub['doc_off'], sub['part_off'],
                            sub['part_seed'], seq=args.seq, dup=5, masking=True,
                            short_seq_prob=0.1, masked_lm_ratio=0.15, rng=rng)
            del ids
            if sb is not None:
                tm = None
                if 'balance' in diag:
                    tm = {}
                bb = sb.step(pb, timings=tm)
                if tm is not None:
                    keys = list(tm)
                    for p_, k_ in zip(keys, keys[1:]):
                        diag['balance'][k_] = diag['balance'].get(k_, 0.0) + (tm[k_] - tm[p_]) * 1e3
                n = bb.n_tokens + 3 * bb.n_rows
                st['moved_rows'] += bb.moved_rows
                del bb
            else:
                n = int(pb.tokens.numel()) + 3 * pb.n_pairs
            record(ev, 2)
            n_tok += n
            for k_, v_ in (('pairs', pb.n_pairs), ('masked', pb.n_masked), ('plan_ms', pb.plan_ms),
                           ('tokens', n), ('kept_sent', pb.n_kept_sentences),
                           ('kept_doc', pb.n_kept_documents)):
                st[k_] += v_
            del pb  # nothing of a step outlives it (HBM is reused by the next step)
        if sb is not None:
            st['shard_counts_spread'] = int((sb.all_shard_counts.max(0) -
                                             sb.all_shard_counts.min(0)).max())
        return n_tok, st, sent_lens

    def step_chunked(ev, rng, b):
        """The same step with tokenization of chunk k+1 pipelined under the pairs of chunk k
        (lddl_amd.pairs.tokenize_and_pair_chunked); tokenize_ms then spans only chunk 0."""
        from lddl_amd.pairs import tokenize_and_pair_chunked
        record(ev, 0)
        record(ev, 1)
        pbs = tokenize_and_pair_chunked(ctx, b['text'], b['sent_off'], doc_off, b['part_off'],
                                        b['part_seed'], n_chunks=args.chunks, seq=args.seq, dup=5,
                                        masking=True, short_seq_prob=0.1, masked_lm_ratio=0.15,
                                        rng=rng)
        record(ev, 2)
        n_tok = sum(int(p.tokens.numel()) + 3 * p.n_pairs for p in pbs)
        st = {'pairs': sum(p.n_pairs for p in pbs), 'masked': sum(p.n_masked for p in pbs),
              'plan_ms': sum(p.plan_ms for p in pbs), 'tokens': n_tok,
              'kept_sent': sum(p.n_kept_sentences for p in pbs),
              'kept_doc': sum(p.n_kept_documents for p in pbs)}
        del pbs
        return n_tok, st, None

    def timed(rng, b=None, pcie=None):
        """W untimed steps, then exactly K steps between barrier + synchronize; max over ranks.
        pcie: host-resident mode — every step first copies its text + sentence offsets from
        pinned host memory (H2D on a copy stream, double-buffered: step k+1's copy overlaps step
        k's compute); the timed region holds all K copies."""
        for _ in range(args.warmup):
            step(rng=rng, b=b)
        torch.cuda.synchronize()
        evs = [[] for _ in range(args.steps)]
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out_tokens = 0
        stats = []
        sent_len = None
        if pcie is not None:
            pcie['issue'](0)
        for k in range(args.steps):
            if pcie is not None:
                bk = pcie['wait'](k)
                if k + 1 < args.steps:
                    pcie['issue'](k + 1)
            n, st, sent_len = step(evs[k], rng=rng, b=bk if pcie is not None else b)
            if pcie is not None:
                pcie['release'](k)
            out_tokens += n
            stats.append(st)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=RED_DEV or dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
            n = torch.tensor([out_tokens], dtype=torch.float64, device=RED_DEV or dev)
            dist.all_reduce(n, op=dist.ReduceOp.SUM)
            out_tokens = int(n.item())
        return dt, out_tokens, evs, stats, sent_len

    dt, out_tokens, evs, stats, sent_len = timed(args.rng)
    mem_head = torch.cuda.memory_stats()  # the headline's own allocator record
    pcie_line = ref_part = None
    if world == 1 and args.workload == 'c2' and args.extra_lines:
        torch.cuda.empty_cache()  # (between lines, untimed) each line starts from an empty pool
        # the same step with the text arriving over PCIe (never `value`)
        h_text = torch.from_numpy(corp.text).pin_memory()
        h_so = torch.from_numpy(corp.sent_off).pin_memory()
        bufs = [dict(base), dict(base, text=torch.empty_like(text), sent_off=torch.empty_like(sent_off))]
        cs = torch.cuda.Stream()
        ready = [torch.cuda.Event(), torch.cuda.Event()]
        free = [None, None]

        def issue(k):
            bk = bufs[k % 2]
            with torch.cuda.stream(cs):
                if free[k % 2] is not None:
                    cs.wait_event(free[k % 2])
                bk['text'].copy_(h_text, non_blocking=True)
                bk['sent_off'].copy_(h_so, non_blocking=True)
                ready[k % 2].record(cs)

        def wait(k):
            torch.cuda.current_stream().wait_event(ready[k % 2])
            return bufs[k % 2]

        def release(k):
            free[k % 2] = torch.cuda.Event()
            free[k % 2].record()
        pdt, ptok, _, _, _ = timed(args.rng, pcie=dict(issue=issue, wait=wait, release=release))
        h2d_gb = (corp.text.nbytes + corp.sent_off.nbytes) / 1e9
        pcie_line = {'value': ptok / pdt, 'ms_per_step': pdt / args.steps * 1e3,
                     'h2d_gb_per_step': h2d_gb,
                     'note': 'text + sentence offsets copied from pinned host memory every step '
                             '(copy stream, double-buffered: the next step\'s copy overlaps this '
                             'step\'s compute), all copies inside the timed region'}
        del bufs, h_text, h_so
        # the reference's example partitioning: --num-blocks 4096 (examples/local_example.sh),
        # i.e. multi-MB partitions, in both RNG modes
        ref_pb = max(1, corp.text.nbytes // 4096)
        rpart = partition_docs(corp, ref_pb)
        rseeds = np.arange(len(rpart) - 1, dtype=np.int64) * 7919 + args.seed
        rb = dict(base, part_off=torch.from_numpy(rpart).to(dev),
                  part_seed=torch.from_numpy(rseeds).to(dev))
        ref_part = {'partition_bytes': int(ref_pb), 'partitions': int(len(rpart) - 1),
                    'note': 'reference example partitioning: --num-blocks 4096 over the batch'}
        for r in ('replay', 'native'):
            torch.cuda.empty_cache()
            rdt, rtok, _, rst, _ = timed(r, b=rb)
            ref_part[r] = {'value': rtok / rdt, 'ms_per_step': rdt / args.steps * 1e3,
                           'plan_ms': float(np.mean([x['plan_ms'] for x in rst]))}
        del rb
    tok_ms = float(np.mean([sum(e[0].elapsed_time(e[1]) for e in ev) for ev in evs]))
    pair_ms = float(np.mean([sum(e[1].elapsed_time(e[2]) for e in ev) for ev in evs]))
    plan_ms = float(np.mean([s['plan_ms'] for s in stats]))
    st = stats[-1]
    n_pairs = st['pairs']
    if sent_len is None:  # chunked step: the tokenizer's own launch, timed once more (untimed step)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _, sl = ctx.tokenize(text, sent_off)
        e1.record()
        torch.cuda.synchronize()
        tok_ms = e0.elapsed_time(e1)
        sent_len = [sl]
    pieces = sum(int((sl.cpu().numpy() & ((1 << 30) - 1)).sum(dtype=np.int64)) for sl in sent_len)
    bal_ms = None
    moved_all = rows_all = None
    if stream:  # one more, untimed step with the balance phases timed (summed over sub-batches)
        diag['balance'] = {}
        step()
        bal_ms = diag.pop('balance')
        # rows that crossed ranks in one timed step, summed over ranks (the imbalance only)
        moved_all = int(st_moved_sum(stats[-1]['moved_rows'], world, dev))
        rows_all = int(st_moved_sum(stats[-1]['pairs'], world, dev))
    alt = None
    if args.alt_rng:  # the other RNG mode on the same batch, reported beside the headline
        other = 'native' if args.rng == 'replay' else 'replay'
        torch.cuda.empty_cache()
        adt, atok, _, astats, _ = timed(other)
        alt = {'rng': other, 'value': atok / adt, 'ms_per_step': adt / args.steps * 1e3,
               'plan_ms': float(np.mean([x['plan_ms'] for x in astats]))}
    seg = None
    # the same path from raw document text: Punkt first (one step over the whole batch, so not
    # for C4, whose 25 GB per GPU only fit as sub-batches)
    if args.segmented_line and world == 1 and args.workload != 'c4':
        torch.cuda.empty_cache()
        seg = timed_segmented(args, rank, world, ctx, dev)
        if args.punkt_params:  # the trained-model kernel on the same documents
            from lddl_amd.punkt import PunktParams
            seg['trained'] = timed_segmented(args, rank, world, ctx, dev,
                                             PunktParams.from_json(args.punkt_params))
            seg['trained']['punkt_params'] = os.path.relpath(args.punkt_params, REPO)
    exch = None
    if world > 1 and args.workload == 'c2' and args.exchange_line:
        torch.cuda.empty_cache()
        try:  # (after the timed region: a failure here must not cost the headline line)
            exch = c4_exchange(args, ctx, dev, corp, part, seeds, text, world)
        except Exception as e:  # noqa: BLE001
            exch = {'error': '{}: {}'.format(type(e).__name__, e)[:500]}
            print('c4_exchange failed on rank {}: {}'.format(rank, exch['error']), file=sys.stderr)
    mem = torch.cuda.memory_stats()
    if rank != 0:
        dist.destroy_process_group()
        return
    # Rooflines. Algorithmic bytes are SURVEY §8(d)'s compulsory bytes, never this
    # design's scratch:
    #  * tokenizer: text read (1 B/byte) + sentence offsets (8 B) + ids written (4 B/piece) +
    #    sent_len (4 B/sentence)  (~10.5 B per wordpiece);
    #  * pair stage: 9 B per output token (4 B id read + 4 B id write + positions/labels of the
    #    15 % masked + per-pair metadata), over the whole stage's time;
    #  * planner kernel alone: its compulsory inputs and outputs - sentence lengths (4 B) and
    #    document offsets (8 B) per duplicate pass, a 16-B A/B window descriptor per pair and 6 B
    #    (position + decision) per mask.
    # `roofline` is the kernel with the longer launch; `issue_roofline` sets each kernel's VALU and
    # SALU instruction counts (committed PMC pass of the same batch size) against the chip's issue
    # rates, the bounds these kernels actually sit on.
    n_bytes, n_sent = corp.text.size, corp.n_sent
    plan_bytes = (4 * 5 * st['kept_sent'] + 8 * 5 * st['kept_doc'] + 16 * n_pairs +
                  6 * st['masked'])
    plan_gbs = plan_bytes / (plan_ms * 1e-3) / 1e9 if plan_ms > 0 else 0.0
    tok_bytes = n_bytes + 8 * (n_sent + 1) + 4 * pieces + 4 * n_sent
    achieved = tok_bytes / (tok_ms * 1e-3) / 1e9
    # pair stage, compulsory bytes at this build's id width: every A/B token's id read
    # once and written once (id_bytes each), per masked token a uint16 position and an id_bytes
    # label, per pair its tok_off (8) + pos_off (8) + len_a (4) + is_random_next (1). SURVEY
    # 8d's 9 B per output token assumed 4-byte ids; it is kept as a labelled secondary figure.
    idb = ctx.id_bytes
    ab_tokens = st['tokens'] - 3 * n_pairs
    stage_bytes = 2 * idb * ab_tokens + (2 + idb) * st['masked'] + 21 * n_pairs
    stage_bytes_survey = 9 * st['tokens']
    stage_gbs = stage_bytes / (pair_ms * 1e-3) / 1e9
    # per-kernel counters per launch from the committed PMC passes (profiles/pmc_*.json, made by
    # tools/prof_counters.sh + tools/make_pmc_json.py) when taken on the same batch size
    pmc_kernels, pmc_src, pmc_meta = load_pmc((args.batch_bytes, int(n_bytes)))
    build_id = lib.lddl_build_id().decode()
    same_build = pmc_meta.get('build_id') == build_id

    def pmc_of(kernel):
        return pmc_entry(pmc_kernels, kernel)

    def traffic(kernel):
        return pmc_of(kernel).get('hbm_bytes_per_launch')
    # issue peaks per chip (profiles/r02_issue_rate_probe.txt, tools/ubench/issue_rate.hip): a
    # SIMD issues one wave64 VALU instruction per 2 cycles (32-wide SIMD, >= 2 waves) and one SALU
    # instruction per 4 cycles (the CU's scalar unit serves its 4 SIMDs in turn)
    valu_peak = 256 * 4 * 2.4e9 / 2
    salu_peak = 256 * 4 * 2.4e9 / 4

    def issue(kernel, ms):
        k = pmc_of(kernel)
        v, sc = k.get('SQ_INSTS_VALU'), k.get('SQ_INSTS_SALU')
        if not v or not ms:
            return None
        a, sa = v / (ms * 1e-3), (sc or 0) / (ms * 1e-3)
        return {'kernel': kernel, 'bound': 'salu_issue' if sa / salu_peak > a / valu_peak else 'valu_issue',
                'valu_instructions_per_launch': v, 'achieved': a, 'peak': valu_peak,
                'unit': 'wave64 VALU instr/s', 'frac': a / valu_peak,
                'salu_instructions_per_launch': sc, 'salu_achieved': sa, 'salu_peak': salu_peak,
                'salu_frac': sa / salu_peak,
                # additive model (4 cycles per SALU + 2 per VALU instruction): it fits both hot
                # kernels' times, but it describes their dependency chains, not a pipe bound -
                # the scalar and vector pipes serve different waves in the same cycles
                # (profiles/r05a_corun_salu_valu.txt: 86-97 % overlap; the planner keeps its time
                # beside a VALU filler, profiles/r05b_corun_planner_valu_filler.log). The pipe
                # bound is max(salu_frac, frac).
                'additive_chain_model_frac': (4.0 * (sc or 0) + 2.0 * v) / (256 * 4 * 2.4e9 * ms * 1e-3),
                'pipe_bound_frac': max(a / valu_peak, sa / salu_peak),
                'source': pmc_src, 'pmc_build_id': pmc_meta.get('build_id'),
                'pmc_git_head': pmc_meta.get('git_head'), 'same_build': same_build,
                'note': ('PMC pass of this build (lddl_build_id {})'.format(build_id) if same_build
                         else 'PMC pass taken on an earlier build of the same batch size')}

    plan_roof = {'kernel': 'plan_replay_kernel' if args.rng == 'replay' else
                 'plan_native_kernel x2 + mask_native_kernel + order_native_kernel (HIP events '
                 'around the native plan, host syncs included)',
                 'bound': 'hbm', 'achieved': plan_gbs,
                 'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': plan_gbs / HBM_PEAK_GBS,
                 'traffic': traffic('plan_replay_kernel') if args.rng == 'replay' else None,
                 'algorithmic_bytes_per_launch': plan_bytes, 'launch_ms': plan_ms,
                 'note': 'latency-bound (dependent scalar chains; issue_roofline pipe fractions '
                         '< 0.6), not HBM-bound (DESIGN.md 4)'}
    tok_roof = {'kernel': 'tokenize_batch_kernel', 'bound': 'hbm', 'achieved': achieved,
                'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': achieved / HBM_PEAK_GBS,
                'traffic': traffic('tokenize_batch_kernel'), 'algorithmic_bytes_per_launch': tok_bytes,
                'launch_ms': tok_ms,
                'note': 'latency-bound at 4 waves/SIMD (~50 % of wave cycles waiting; '
                        'issue_roofline pipe fractions < 0.6), not HBM-bound (DESIGN.md 4)'}
    stage_roof = {'kernel': 'pair stage (compaction, densify, plan, shuffle, resolve, layout, '
                            'gather)', 'bound': 'hbm', 'achieved': stage_gbs,
                  'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': stage_gbs / HBM_PEAK_GBS,
                  'algorithmic_bytes_per_step': stage_bytes, 'stage_ms': pair_ms,
                  'bytes_per_output_token': stage_bytes / max(1, st['tokens']),
                  'id_bytes': idb,
                  'survey_9b': {'algorithmic_bytes_per_step': stage_bytes_survey,
                                'frac': stage_bytes_survey / (pair_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                'note': 'SURVEY 8d: 9 B per output token (4-byte ids)'},
                  'note': 'compulsory bytes at this build\'s id width: 2 x id_bytes per A/B token '
                          '(read + write), (2 + id_bytes) per mask, 21 B per pair of metadata'}
    # the north star's path-level number ("% of HBM roofline on the 1-GPU WordPiece+masking
    # path"): tokenizer + pair-stage compulsory bytes over the whole step's time
    path_bytes = tok_bytes + stage_bytes

    def path_roof(ms, rng):
        gbs = path_bytes / (ms * 1e-3) / 1e9
        return {'rng': rng, 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': gbs / HBM_PEAK_GBS, 'algorithmic_bytes_per_step': path_bytes,
                'ms_per_step': ms,
                'frac_survey_9b': (tok_bytes + stage_bytes_survey) / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    res = {
        'metric': 'WordPiece+MLM tokens/sec (1/2/4/8 MI355X) and % of HBM roofline',
        'value': out_tokens / dt,
        'unit': 'output tokens/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': dt * 1e3 / args.steps,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'uint16' if ctx.id_bytes == 2 else 'int32',
        'data': 'synthetic',
        'config': {
            'workload': ('C2: synthetic English-like corpus (SURVEY 8d generator, seed {}), '
                         'seq {}, static masking, duplicate_factor 5, no binning; {} MiB of '
                         'sentence text per GPU per step, {} KiB partitions' if args.workload == 'c2'
                         else args.workload.upper() + ': synthetic English-like corpus (SURVEY 8d '
                         'generator, seed {}), seq {} phase 2, static masking, duplicate_factor 5, 64 '
                         'bins of 8 tokens + streaming load balance into ' + str(n_shards) +
                         ' shards (per sub-batch: RCCL count all-gather + all-to-all-v exchange '
                         'when N > 1); {} MiB of sentence text per GPU per step, {} KiB partitions, '
                         + str(len(subs or [0])) + ' sub-batch(es)').format(
                             args.seed, args.seq, args.batch_bytes >> 20, args.partition_bytes >> 10),
            'seq_len': args.seq, 'masking': 'static', 'duplicate_factor': 5,
            'rng': ('replay (CPython MT19937, random.seed per partition)' if args.rng == 'replay'
                    else 'native (Philox4x32-10 counter RNG per partition/unit/pair)'),
            'batch_bytes': int(n_bytes), 'sentences': int(n_sent), 'documents': int(corp.n_doc),
            'partitions': int(len(part) - 1), 'wordpieces': pieces, 'pairs': int(n_pairs),
            'vocab': os.path.basename(VOCAB), 'parallelism': 'dp{} (document shards)'.format(world),
        },
        'stages_ms': {'tokenize': tok_ms,
                      ('pairs_plan_and_gather' if args.workload == 'c2' else
                       'pairs_bin_and_balance'): pair_ms,
                      'per_step_pairs': [round(sum(e[1].elapsed_time(e[2]) for e in ev), 2)
                                         for ev in evs],
                      'per_step_plan': [round(x['plan_ms'], 2) for x in stats]},
        'roofline': None,  # the dominant kernel's, filled below
        'roofline_planner': plan_roof,
        'roofline_tokenizer': tok_roof,
        'roofline_pairs_stage': stage_roof,
        'issue_roofline': [x for x in (issue('tokenize_batch_kernel', tok_ms),
                                       issue('plan_replay_kernel', plan_ms)) if x],
    }
    res['roofline'] = plan_roof if plan_ms >= tok_ms else tok_roof
    res['roofline_path'] = [path_roof(dt * 1e3 / args.steps, args.rng)]
    if alt is not None:
        res['roofline_path'].append(path_roof(alt['ms_per_step'], alt['rng']))
    if bal_ms is not None:
        res['balance_phases_ms_untimed_step'] = bal_ms
        res['balance'] = {'num_shards': n_shards, 'moved_rows_per_step': moved_all,
                          'rows_per_step': rows_all,
                          'max_shard_spread_rows': st.get('shard_counts_spread'),
                          'exchange_ms_untimed_step': bal_ms.get('exchange'),
                          'note': 'moved_rows_per_step: rows received from other ranks in one '
                                  'step, all ranks (only the per-bin surplus over each rank\'s '
                                  'shard quota moves, balance.py)'}
    if alt is not None:
        res['alt_rng'] = alt
    if exch is not None:
        res['c4_exchange'] = exch
    if seg is not None:
        res['with_segmentation'] = seg
    if pcie_line is not None:
        res['pcie_inclusive'] = pcie_line
    if ref_part is not None:
        res['ref_partitioning'] = ref_part
    res['build_id'] = build_id  # lddl_build_id(): SHA-256 of the library's sources
    res['torch_alloc_retries'] = int(mem_head.get('num_alloc_retries', 0))  # headline line
    res['torch_alloc_retries_all_lines'] = int(mem.get('num_alloc_retries', 0))
    free_b, total_b = torch.cuda.mem_get_info()
    res['memory_gb'] = {'headline_max_reserved': round(mem_head.get('reserved_bytes.all.peak', 0) / 1e9, 1),
                        'headline_max_allocated': round(mem_head.get('allocated_bytes.all.peak', 0) / 1e9, 1),
                        'torch_max_reserved': round(torch.cuda.max_memory_reserved() / 1e9, 1),
                        'torch_max_allocated': round(torch.cuda.max_memory_allocated() / 1e9, 1),
                        'device_free_at_end': round(free_b / 1e9, 1),
                        'device_total': round(total_b / 1e9, 1)}
    if world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baseline(corp, part, seeds, args)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
