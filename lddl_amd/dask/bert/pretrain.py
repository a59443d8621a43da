"""`preprocess_bert_pretrain` — drop-in for the reference's `lddl.dask.bert.pretrain`
(lddl/dask/bert/pretrain.py:563-884): same flags, same output layout, GPU data plane.

Pipeline (reference call stack in SURVEY.md §3.1):
  read `*.txt` sources into blocks (readers.py)            -> lddl_amd.dask.readers (host; each
                                                              rank reads only its own blocks)
  random shuffle of documents over partitions (100-111)    -> seeded shuffle of the documents of
                                                              each shuffle group of partitions
                                                              (host; the reference's is global
                                                              and unseeded)
  split_id_text (readers.py:131-136)                       -> host, per line
  sent_tokenize + strip + drop empty (86-88)               -> lddl_segment_* (HIP Punkt; nltk on
                                                              the host with --sentence-splitter host)
  tokenizer.tokenize(s, max_length=512, truncation=True)   -> lddl_tokenize (HIP)
  _to_partition_pairs / create_pairs_from_document /
    create_masked_lm_predictions (386-402, 241-365, 182-238) -> lddl_pairs_plan / emit (HIP)
  _to_dataframe_binned (binning.py:63-93)                  -> lddl_bin_partitions (HIP)
  instance dict + serialize_np_array (345-358)             -> lddl_render_* (HIP)
  to_parquet / write_partition_binned + _metadata          -> pyarrow writer (host)

Random state: the reference draws from each Dask worker's unseeded global `random` (H1). Here
partition p is processed as if `random.seed(partition_seed(--seed, p))` had been called before
its `_to_partition_pairs`, which the test-suite replays bit for bit on the CPU.

Multi-GPU (`--schedule mpi`, launched with torchrun, one process per GPU): rank r owns the
partitions p with p % world_size == r (partitions are independent) and reads only
those blocks.

`--num-shards S` (lddl_amd; the reference runs `balance_dask_output` as a second job over the
files) writes the balancer's layout directly: `shard-<k>.parquet_<b>` (or `shard-<k>.parquet`
unbinned) with N or N+1 samples per bin, plus `.num_samples.json` (lddl/dask/load_balance.py:
90-92, 372-378) — what get_bert_pretrain_data_loader consumes. `--balance-plan stream` (default)
balances every GPU batch in HBM as it is produced (lddl_amd/balance.py: RCCL all-gather of the
batch's per-bin counts, per-rank shard quotas, all-to-all-v of only each bin's surplus rows over
a rank's quota), so HBM holds one batch at any corpus size and each shard file grows
by one row group per batch; `--balance-plan reference` writes the part files and runs the
drop-in balance_dask_output over them (the reference's exact shard contents).
"""
import argparse
import functools
import json
import os
import random
import sys
import time

import numpy as np

from ...utils import attach_bool_arg, expand_outdir_and_mkdir, parse_str_of_num_bytes
from .. import readers
from . import segment

ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                      'assets')


def partition_seed(seed, p):
    """random.seed() value of partition p (documented replacement of the unseeded worker RNG)."""
    return int(seed) * 1000003 + int(p)


def _resolve_vocab(vocab_file):
    if os.path.isfile(vocab_file):
        return vocab_file
    raise FileNotFoundError(
        '--vocab-file {!r} is not a file. The reference falls back to '
        'BertTokenizerFast.from_pretrained (a network download); lddl_amd runs offline and needs '
        'a vocab.txt path (e.g. {}/vocab_synth_uncased_30522.txt)'.format(vocab_file, ASSETS))


def plan_partitions(args):
    """Every partition of the corpus as an unread readers.Block, in the reference's partition
    order (wikipedia, books, common crawl; db.concat, pretrain.py:412-438)."""
    blocksize = args.block_size
    if args.num_blocks is not None:
        if blocksize is not None:
            raise ValueError('Only one of num_blocks or blocksize needs to be set!')
        blocksize = readers.estimate_block_size((args.wikipedia, args.books, args.common_crawl),
                                                args.num_blocks)
    blocks = []
    if args.wikipedia is not None:
        blocks += readers.plan_blocks(readers.wikipedia_dir(args.wikipedia, args.wikipedia_lang),
                                      blocksize, args.sample_ratio, args.seed)
    if args.books is not None:
        blocks += readers.plan_blocks(args.books, blocksize, args.sample_ratio, args.seed)
    if args.common_crawl is not None:
        blocks += readers.plan_blocks(args.common_crawl, blocksize, args.sample_ratio, args.seed)
    return blocks


def _greedy(items, size_of, cap):
    """Consecutive runs of `items` of at most `cap` total size (at least one item each)."""
    out, cur, size = [], [], 0
    for it in items:
        b = size_of(it)
        if cur and size + b > cap:
            out.append(cur)
            cur, size = [], 0
        cur.append(it)
        size += b
    if cur:
        out.append(cur)
    return out


def rank_batches(args, blocks, rank=0, world=1):
    """This rank's partitions (p % world == rank) as GPU batches: lists of shuffle groups, each a
    list of partitions. Shuffle groups are runs of ~--shuffle-group-bytes of input and do not
    depend on --gpu-batch-bytes; a batch is a run of whole groups of <= --gpu-batch-bytes."""
    mine = [p for p in range(len(blocks)) if p % world == rank]
    groups = _greedy(mine, lambda p: blocks[p].nbytes, args.shuffle_group_bytes)
    return _greedy(groups, lambda g: sum(blocks[p].nbytes for p in g), args.gpu_batch_bytes)


def iter_batches(args, rank=0, world=1, blocks=None, as_bytes=False):
    """This rank's partitions in GPU batches, read lazily: yields [(p, lines)] per batch. The
    documents of each shuffle group are shuffled over the group's partitions (each keeps its
    document count) by Random(partition_seed(seed, -1 - first partition of the group)), so the
    output does not depend on the GPU batch size. as_bytes: lines as UTF-8 bytes (the GPU
    segmenter's input) instead of str."""
    blocks = plan_partitions(args) if blocks is None else blocks
    for batch in rank_batches(args, blocks, rank, world):
        out = []
        for g in batch:
            parts = [(p, readers.read_block(blocks[p], as_bytes=as_bytes)) for p in g]
            docs = [d for _, lines in parts for d in lines]
            random.Random(partition_seed(args.seed, -1 - g[0])).shuffle(docs)
            k = 0
            for p, lines in parts:
                out.append((p, docs[k:k + len(lines)]))
                k += len(lines)
        yield out


def iter_doc_batches(args, rank=0, world=1, blocks=None):
    """The GPU-segmentation path's input: this rank's partitions as (partitions, corpus) GPU
    batches, corpus = build_doc_corpus's ('documents', text, doc_off, part_doc_off). Whole shuffle
    groups are read by the library's host reader (readers.read_groups_native: the same lines,
    sampling, per-group document shuffle and split_id_text as iter_batches + build_doc_corpus, in
    C++ threads), then cut into GPU batches of <= --gpu-batch-bytes of input (whole partitions),
    so the GPU work, the rendering and the file writes of consecutive batches overlap."""
    blocks = plan_partitions(args) if blocks is None else blocks
    for batch in rank_batches(args, blocks, rank, world):
        rd = readers.NativeRead([[blocks[p] for p in g] for g in batch],
                                [partition_seed(args.seed, -1 - g[0]) for g in batch],
                                threads=getattr(args, 'read_threads', 16))
        parts = [p for g in batch for p in g]
        pdo = np.zeros(len(parts) + 1, np.int64)
        np.cumsum(rd.block_ndocs, out=pdo[1:])
        try:
            for sub in _greedy(list(range(len(parts))), lambda i: blocks[parts[i]].nbytes,
                               args.gpu_batch_bytes):
                i0, i1 = sub[0], sub[-1] + 1
                d0, d1 = int(pdo[i0]), int(pdo[i1])
                text, doc_off = rd.fill(d0, d1)  # this GPU batch's documents only
                yield ([(parts[i], None) for i in range(i0, i1)],
                       ('documents', text, doc_off, pdo[i0:i1 + 1] - d0))
        finally:
            rd.close()


def get_partitions(args, rank=0, world=1):
    """Partitions (lists of raw document lines) owned by `rank`, after sampling and the shuffle."""
    return [pl for batch in iter_batches(args, rank, world) for pl in batch]


def _segment_docs(lines):
    out = []
    for raw in lines:
        if isinstance(raw, bytes):
            raw = raw.decode('utf-8')
        _, sents = segment.document_sentences(raw)
        out.append([s.encode('utf-8') for s in sents])
    return out


def build_corpus(partitions, workers=1):
    """Flatten partitions into the device corpus layout: text bytes, sentence byte offsets,
    document sentence offsets, partition document offsets (host segmentation)."""
    flat = [lines for _, lines in partitions]
    if workers > 1 and sum(len(x) for x in flat) > 2000:
        from multiprocessing import get_context
        with get_context('fork').Pool(workers) as pool:
            segd = pool.map(_segment_docs, flat, chunksize=1)
    else:
        segd = [_segment_docs(x) for x in flat]
    chunks, sent_len, doc_ns, part_nd = [], [], [], []
    for docs in segd:
        part_nd.append(len(docs))
        for sents in docs:
            doc_ns.append(len(sents))
            for s in sents:
                chunks.append(s)
                sent_len.append(len(s))
    text = np.frombuffer(b''.join(chunks), np.uint8) if chunks else np.zeros(0, np.uint8)
    sent_off = np.zeros(len(sent_len) + 1, np.int64)
    np.cumsum(sent_len, out=sent_off[1:])
    doc_sent_off = np.zeros(len(doc_ns) + 1, np.int64)
    np.cumsum(doc_ns, out=doc_sent_off[1:])
    part_doc_off = np.zeros(len(part_nd) + 1, np.int64)
    np.cumsum(part_nd, out=part_doc_off[1:])
    return text, sent_off, doc_sent_off, part_doc_off


def build_doc_corpus(partitions):
    """Raw document texts for the GPU segmenter: the text after each line's id
    (split_id_text, readers.py:131-136), documents back to back, plus document byte offsets and
    partition document offsets."""
    chunks, part_nd = [], []
    for _, lines in partitions:
        part_nd.append(len(lines))
        if lines and isinstance(lines[0], bytes):
            chunks += [readers.split_id_text_bytes(raw)[1] for raw in lines]
        else:
            chunks += [readers.split_id_text(raw)[1].encode('utf-8') for raw in lines]
    text = np.frombuffer(b''.join(chunks), np.uint8) if chunks else np.zeros(0, np.uint8)
    doc_off = np.zeros(len(chunks) + 1, np.int64)
    np.cumsum(np.fromiter(map(len, chunks), np.int64, len(chunks)), out=doc_off[1:])
    part_doc_off = np.zeros(len(part_nd) + 1, np.int64)
    np.cumsum(part_nd, out=part_doc_off[1:])
    return 'documents', text, doc_off, part_doc_off


def punkt_params(args):
    """--punkt-params JSON, else nltk's English model when nltk can load it locally (the
    reference's sent_tokenize), else the untrained parameters (what offline nltk runs)."""
    from ...punkt import PunktParams
    if getattr(args, 'punkt_params', None):
        return PunktParams.from_json(args.punkt_params)
    try:
        import nltk
        return PunktParams.from_nltk(nltk.data.load('tokenizers/punkt/english.pickle'))
    except Exception:  # nltk or its English model unavailable offline
        return PunktParams()


def make_batch_pairs(ctx, args, partitions, corpus, timer=None):
    """The GPU hot path over one batch of partitions -> PairBatch (pairs in partition order)."""
    import torch
    from ...pairs import make_pairs
    dev = ctx.device
    tm = timer or (lambda name: None)
    if corpus[0] == 'documents':  # GPU Punkt: sentences of every document of the batch
        from ... import punkt
        _, text, doc_off, part_doc_off = corpus
        d_text = torch.from_numpy(text).to(dev) if len(text) else torch.zeros(
            1, dtype=torch.uint8, device=dev)[:0]
        d_doc = torch.from_numpy(doc_off).to(dev)
        tm('h2d')
        bad = punkt.utf8_first_invalid(d_text)
        if bad >= 0:  # dask.bag.read_text decodes strictly: the reference raises here too
            raise UnicodeDecodeError('utf-8', bytes(text[max(bad - 8, 0):bad + 8]), 0, 1,
                                     'invalid UTF-8 in the input documents (byte {} of the '
                                     'batch text)'.format(bad))
        d_so, d_dso = punkt.segment(ctx, d_text, d_doc)
        tm('segment')
    else:
        _, text, sent_off, doc_sent_off, part_doc_off = corpus
        d_text = torch.from_numpy(text).to(dev) if len(text) else torch.zeros(
            1, dtype=torch.uint8, device=dev)[:0]
        d_so = torch.from_numpy(sent_off).to(dev)
        d_dso = torch.from_numpy(doc_sent_off).to(dev)
        tm('h2d')
    ids, sent_len = ctx.tokenize(d_text, d_so, max_pieces=512)
    tm('tokenize')
    seeds = np.asarray([partition_seed(args.seed, p) for p, _ in partitions], np.int64)
    pb = make_pairs(ctx, d_so, ids, sent_len, d_dso,
                    torch.from_numpy(part_doc_off).to(dev), torch.from_numpy(seeds).to(dev),
                    seq=args.target_seq_length, dup=args.duplicate_factor, masking=args.masking,
                    short_seq_prob=args.short_seq_prob, masked_lm_ratio=args.masked_lm_ratio,
                    rng=getattr(args, 'rng', 'replay'), native_seed=args.seed)
    tm('pairs')
    return pb


def process_batch(ctx, args, partitions, corpus, outdir, timer=None, executor=None, futures=None,
                  copier=None):
    """Run the GPU hot path over a group of partitions and write their files (concurrently on
    `executor` when given: the futures go to `futures`). With a `copier` (one host thread), the
    rendered columns are copied to the host and handed to the writers there, so this batch's
    copy and writes overlap the next batch's GPU work; the returned future yields the paths."""
    from ... import output
    tm = timer or (lambda name: None)
    index = [p for p, _ in partitions]
    _trace('gpu_start', index[0])
    pb = make_batch_pairs(ctx, args, partitions, corpus, timer)
    part_rows = pb.part_off.cpu().numpy()
    if args.bin_size is not None:
        import torch
        nbins = args.target_seq_length // args.bin_size
        perm, bin_id, counts = output.bin_partitions(ctx, None, pb.part_off, args.bin_size, nbins,
                                                     tok_off=pb.tok_off)
        drd = output.render_device(ctx, pb, perm, bin_id)
        counts = counts.cpu().numpy()
    else:
        nbins, counts = None, None
        drd = output.render_device(ctx, pb)
    del pb
    tm('render')

    _trace('render_device', index[0])

    def finish(stream=None):
        _trace('d2h_start', index[0])
        chunk = _D2H_CHUNK_BYTES
        if args.output_format == 'parquet' and chunk > 0:
            # string columns in partition groups of ~chunk bytes, each handed to the writers as
            # it lands (output.DeviceRendered.to_host_chunks)
            paths = []
            for p0, p1, rd in drd.to_host_chunks(part_rows, chunk, stream):
                paths += output.write_parquet(outdir, rd, part_rows[p0:p1 + 1], index[p0:p1],
                                              args.masking, nbins,
                                              None if counts is None else counts[p0:p1],
                                              executor=executor, futures=futures)
            _trace('d2h_end', index[0])
            return paths
        rd = drd.to_host(stream)
        _trace('d2h_end', index[0])
        if args.output_format == 'parquet':
            return output.write_parquet(outdir, rd, part_rows, index, args.masking, nbins,
                                        counts, executor=executor, futures=futures)
        return write_txt(outdir, rd, part_rows, index, args.masking, nbins, counts,
                         getattr(args, 'n_partitions', len(part_rows) - 1))
    if copier is not None and args.output_format == 'parquet':
        fut = copier.submit(finish, _copy_stream(ctx))
        fut.render_bytes = drd.nbytes  # pinned host bytes until the batch is written
        return fut
    paths = finish()
    tm('write')
    return paths


_T0 = time.perf_counter()
_TRACE = os.environ.get('LDDL_TRACE_PIPELINE')
# rendered batches leave the GPU in partition groups of about this many MiB of strings (0: the
# whole batch in one pinned allocation per column, the round-4 behaviour)
_D2H_CHUNK_BYTES = int(os.environ.get('LDDL_D2H_CHUNK_MB', '128')) << 20


def _trace(what, batch):
    """LDDL_TRACE_PIPELINE=1: host timeline of the CLI pipeline on stderr (diagnostics)."""
    if _TRACE:
        import threading
        sys.stderr.write('[pipe] %8.3f %-14s batch@%s %s\n' % (time.perf_counter(), what,
                                                               batch,
                                                               threading.current_thread().name))


def _row_order(ranges):
    """The sharded writer's (shard, bin, r0, r1) row ranges in row order (the balanced table is
    bin-major, `ranges` shard-major), the chunk bounds over them and whether they tile the rows
    contiguously (then the copy leaves the GPU in groups of them, as process_batch does). Empty
    ranges sort before the non-empty range that starts at the same row (key (r0, r1)); sorting on
    r0 alone put an empty (R, R) after (R, R + k) and the check failed for any batch in which a
    shard received no rows of a bin."""
    srt = sorted(ranges, key=lambda x: (x[2], x[3]))
    bounds = [srt[0][2]] + [x[3] for x in srt] if srt else [0]
    return srt, bounds, all(srt[i][2] == bounds[i] for i in range(len(srt)))


def _copy_stream(ctx):
    import torch
    s = getattr(ctx, '_copy_stream', None)
    if s is None:
        s = ctx._copy_stream = torch.cuda.Stream(device=ctx.device)
    return s


def _txt_line(row, masking):
    """pretrain.py:508-527 line format."""
    from ...utils import deserialize_np_array
    if masking:
        return ('is_random_next: {} - [CLS] {} [SEP] {} [SEP] - masked_lm_positions: {} - '
                'masked_lm_labels: {} - {}').format(row['is_random_next'], row['A'], row['B'],
                                                    deserialize_np_array(
                                                        row['masked_lm_positions']),
                                                    row['masked_lm_labels'], row['num_tokens'])
    return 'is_random_next: {} - [CLS] {} [SEP] {} [SEP] - {}'.format(
        row['is_random_next'], row['A'], row['B'], row['num_tokens'])


def _pad_name(n):
    """fsspec build_name_function(n - 1) (dask to_textfiles' default names): zero-padded to the
    width of the largest partition index."""
    import math
    w = int(math.ceil(math.log10(max(n - 1, 0) + 1e-8)))
    return lambda i: str(i).zfill(w)


def write_txt(outdir, rd, part_rows, index, masking, nbins, counts, n_part):
    """Debug output (`--output-format txt`, pretrain.py:501-531): dask's to_textfiles writes
    partition i to `<i>.txt` (i zero-padded to the width of n_part - 1); the binned writer
    (binning.py:439-509) names (i, b) `<i>_<b>.txt` and creates every bin's file. Lines are
    joined by '\n' without a trailing newline (last_endline=False)."""
    name = _pad_name(n_part)
    paths = []
    for p in range(len(part_rows) - 1):
        r0, r1 = int(part_rows[p]), int(part_rows[p + 1])
        spans = [(None, r0, r1)] if nbins is None else []
        if nbins is not None:
            b0 = r0
            for b in range(nbins):
                spans.append((b, b0, b0 + int(counts[p, b])))
                b0 += int(counts[p, b])
        for b, a, z in spans:
            fn = os.path.join(outdir, '{}.txt'.format(name(index[p])) if b is None else
                              '{}_{}.txt'.format(index[p], b))
            with open(fn, 'w') as f:
                f.write('\n'.join(_txt_line(rd.row(r), masking) for r in range(a, z)))
            paths.append(fn)
    return paths


def _open_file_budget(needed, headroom=256):
    """Raise this process's soft RLIMIT_NOFILE so that `needed` parquet writers can stay open
    (plus headroom for pyarrow, sockets and libraries); False if the hard limit is too low."""
    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    want = needed + headroom
    if soft == resource.RLIM_INFINITY or want <= soft:
        return True
    if hard != resource.RLIM_INFINITY and want > hard:
        return False
    try:
        resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
    except (ValueError, OSError):
        return False
    return True


class ShardWriters:
    """This rank's balanced shards, written as the batches stream through: one parquet file per
    (shard, bin) named like the load balancer's (`shard-<k>.parquet_<b>`, or `shard-<k>.parquet`
    unbinned, load_balance.py:90-92), one row group per batch in batch order. Each batch's
    writes run on the thread pool while the next batch is on the GPU; a writer is never
    appended from two threads (a batch's writes finish before the next batch's start).

    Every (shard, bin) file stays open until close() (the reference example's 4096 shards x 8
    bins are 32,768 files on one rank): the soft RLIMIT_NOFILE is raised for them. When the hard
    limit (or `max_open`) cannot hold them all, each batch's row group is written to a piece file
    and closed at once, and close() appends the pieces of each shard, in batch order, into its
    file (the same files, one more pass over the data)."""

    def __init__(self, outdir, nbins, binned, masking, pool, n_local_shards=None, max_open=None,
                 max_inflight_bytes=8 << 30):
        self.outdir, self.nbins, self.binned, self.masking, self.pool = (outdir, nbins, binned,
                                                                         masking, pool)
        self.max_inflight_bytes = max_inflight_bytes  # pinned bytes of rendered batches
        self.writers, self.pending, self.shards, self.jobs = {}, [], set(), []
        self.last_chunked = None  # the last batch left the GPU in row-range groups (tests)
        needed = (n_local_shards or 0) * nbins
        self.pieces = None  # {(shard, bin): [piece paths]} in piece mode
        if (max_open is not None and needed > max_open) or not _open_file_budget(needed):
            self.pieces = {}
            self.piece_dir = os.path.join(outdir, '.lddl_amd_pieces.{}'.format(os.getpid()))
            os.makedirs(self.piece_dir, exist_ok=True)

    def name(self, s, b):
        return os.path.join(self.outdir, 'shard-{}.parquet{}'.format(
            s, '_{}'.format(b) if self.binned else ''))

    def _append(self, key, rd, r0, r1):
        from ... import output
        self._write(key, output.table(rd, r0, r1, self.masking, self.binned))

    def _write(self, key, t):
        import pyarrow.parquet as pq
        from ... import output
        if self.pieces is not None:
            lst = self.pieces.setdefault(key, [])
            fn = os.path.join(self.piece_dir, '{}_{}.{}'.format(key[0], key[1], len(lst)))
            pq.write_table(t, fn, compression=output.DEFAULT_COMPRESSION)
            lst.append(fn)
            return
        w = self.writers.get(key)
        if w is None:
            w = self.writers[key] = pq.ParquetWriter(self.name(*key), t.schema,
                                                     compression=output.DEFAULT_COMPRESSION)
        w.write_table(t)

    def _merge(self, key):
        """Piece mode: the pieces of one (shard, bin), row group by row group, into its file."""
        import pyarrow.parquet as pq
        from ... import output
        w = None
        for fn in self.pieces.pop(key):
            pf = pq.ParquetFile(fn)
            for g in range(pf.num_row_groups):
                t = pf.read_row_group(g)
                if w is None:
                    w = pq.ParquetWriter(self.name(*key), t.schema,
                                         compression=output.DEFAULT_COMPRESSION)
                w.write_table(t)
            os.remove(fn)
        if w is not None:
            w.close()

    def add(self, ctx, bb, copier=None):
        """Render this batch's rows of the rank's shards (GPU) and queue their writes. With a
        `copier` thread, the host copy and the queueing run there (in batch order: a batch's
        appends are queued after the previous batch's have finished), overlapping the next
        batch's GPU work."""
        from ... import output
        self.shards.update(bb.shards)
        if bb.n_rows == 0:
            return
        drd = output.render_device(ctx, bb.table, bb.rows, bb.bin_ids() if self.binned else None)
        ranges = [(s, b) + tuple(bb.shard_range(m, b)) for m, s in enumerate(bb.shards)
                  for b in range(self.nbins)]

        writes = []  # this batch's write futures: its pinned copy lives until they finish
        srt, bounds, contiguous = _row_order(ranges)
        chunked = _D2H_CHUNK_BYTES > 0 and contiguous
        self.last_chunked = chunked

        def job(stream=None):
            if chunked:
                first = True
                for p0, p1, rd in drd.to_host_chunks(bounds, _D2H_CHUNK_BYTES, stream):
                    if first:  # appends stay in batch order per (shard, bin) writer
                        for f in self.pending:
                            f.result()
                        self.pending, first = [], False
                    new = [self.pool.submit(self._append, (s, b), rd, r0, r1)
                           for s, b, r0, r1 in srt[p0:p1] if r1 > r0]
                    self.pending += new
                    writes.extend(new)
                return
            rd = drd.to_host(stream)
            for f in self.pending:
                f.result()
            self.pending = [self.pool.submit(self._append, (s, b), rd, r0, r1)
                            for s, b, r0, r1 in ranges if r1 > r0]
            writes.extend(self.pending)
        if copier is None:
            job()
            return
        nb = drd.nbytes
        # a batch's bytes count until its WRITES have finished (not only its copy job), so the
        # pinned host copies held at once stay within max_inflight_bytes plus the newest batch
        while self.jobs and (len(self.jobs) >= 2 or
                             sum(b for _, b, _ in self.jobs) + nb > self.max_inflight_bytes):
            j, _, ws = self.jobs.pop(0)
            j.result()
            for f in ws:
                f.result()
        self.jobs.append((copier.submit(job, _copy_stream(ctx)), nb, writes))

    def close(self):
        """Finish the writes; shards of a bin that received no rows get an empty file (every bin
        has all shards, as the loader requires)."""
        import pyarrow.parquet as pq
        from ... import output
        for j, _, _ in self.jobs:
            j.result()
        self.jobs = []
        for f in self.pending:
            f.result()
        self.pending = []
        merged = set()
        if self.pieces is not None:  # one writer open per pool thread at a time
            merged = set(self.pieces)
            for f in [self.pool.submit(self._merge, k) for k in list(self.pieces)]:
                f.result()
            os.rmdir(self.piece_dir)
        paths, done = [], []
        empty = output.schema(self.masking, self.binned).empty_table()
        for s in sorted(self.shards):
            for b in range(self.nbins):
                w = self.writers.pop((s, b), None)
                if w is not None:  # footers written on the pool (one writer per task)
                    done.append(self.pool.submit(w.close))
                elif (s, b) not in merged:  # (merged: written from its pieces above)
                    done.append(self.pool.submit(pq.write_table, empty, self.name(s, b),
                                                 compression=output.DEFAULT_COMPRESSION))
                paths.append(self.name(s, b))
        for f in done:
            f.result()
        return paths


def num_samples_of_shards(shard_counts, binned):
    """`.num_samples.json` content of the balanced layout (load_balance.py:372-378) from the
    int64[S, B] shard counts."""
    out = {}
    S, B = shard_counts.shape
    for b in range(B):
        for s in range(S):
            out['shard-{}.parquet{}'.format(s, '_{}'.format(b) if binned else '')] = int(
                shard_counts[s, b])
    return out


def _default_inflight_bytes():
    """1/8 of the host's memory, clamped to 2-16 GiB."""
    try:
        total = os.sysconf('SC_PAGE_SIZE') * os.sysconf('SC_PHYS_PAGES')
    except (ValueError, OSError):
        total = 64 << 30
    return int(max(2 << 30, min(16 << 30, total // 8)))


def _any_rank(flag, device):
    """True when `flag` holds on any rank (all-reduce MAX: RCCL on a device tensor, gloo on the
    host)."""
    import torch
    import torch.distributed as dist
    dev = device if dist.get_backend() == 'nccl' else 'cpu'
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item())


def _warm_gpu_path(ctx, args):
    """One tiny batch of made-up documents through segment -> tokenize -> pairs -> render, output
    discarded: the first launch of each kernel (code object loading) and the first allocations
    happen here, while the host reader is still reading, instead of in the first real batch."""
    import torch
    from ... import output
    doc = ('The first sentence is here. A second one follows it! Then a third, with more words '
           'in it? The fourth ends the document.')
    lines = [('{} {}'.format(k, doc)).encode('utf-8') for k in range(8)]
    corpus = build_doc_corpus([(0, lines[:4]), (1, lines[4:])])
    pb = make_batch_pairs(ctx, args, [(0, None), (1, None)], corpus)
    if args.bin_size is not None:
        nbins = args.target_seq_length // args.bin_size
        perm, bin_id, _ = output.bin_partitions(ctx, None, pb.part_off, args.bin_size, nbins,
                                                tok_off=pb.tok_off)
        output.render_device(ctx, pb, perm, bin_id)
    else:
        output.render_device(ctx, pb)
    torch.cuda.synchronize(ctx.device)


def _empty_pairs(ctx, masking):
    """A PairBatch without rows (a rank with fewer batches still takes part in the collectives)."""
    import torch
    from ...pairs import PairBatch
    dev = ctx.device
    e64 = torch.zeros(1, dtype=torch.int64, device=dev)
    pb = PairBatch(torch.zeros(0, dtype=ctx.id_dtype, device=dev), e64,
                   torch.zeros(0, dtype=torch.int32, device=dev),
                   torch.zeros(0, dtype=torch.uint8, device=dev))
    if masking:
        pb.pos = torch.zeros(0, dtype=torch.int16, device=dev)
        pb.labels = torch.zeros(0, dtype=ctx.id_dtype, device=dev)
        pb.pos_off = e64.clone()
    return pb


def _prefetch(gen, depth=1):
    """Iterate `gen` in a background thread, `depth` items ahead (the host read / decode of batch
    k+1 overlaps the GPU work and the file writes of batch k). Exceptions are re-raised here."""
    import queue
    import threading
    q = queue.Queue(maxsize=depth)
    done = object()

    def run():
        try:
            for item in gen:
                q.put(item)
        except BaseException as e:  # noqa: B902 - handed to the consumer
            q.put(e)
            return
        q.put(done)
    threading.Thread(target=run, daemon=True).start()
    while True:
        item = q.get()
        if item is done:
            return
        if isinstance(item, BaseException):
            raise item
        yield item


class _StageTimer:
    """Cumulative wall time per stage (device-synchronised), printed at the end of main."""

    def __init__(self, enabled):
        self.enabled, self.t, self.acc = enabled, None, {}

    def __call__(self, name):
        if not self.enabled:
            return
        import torch
        torch.cuda.current_stream().synchronize()  # (not the copy stream: it overlaps)
        now = time.perf_counter()
        if self.t is not None:
            self.acc[name] = self.acc.get(name, 0.0) + now - self.t
        self.t = now

    def mark(self):
        if self.enabled:
            self.t = time.perf_counter()


def _run_gpu_workers(args, n_workers, vocab, ctx0, batch_it, outdir, pool, copier, inflight,
                     timer=None):
    """The non-balanced batch loop over `n_workers` GPU worker threads (main's --gpu-workers).
    Worker 0 uses the main Context; the others create their own (a Context holds per-call state:
    the segmenter's count / fill pair). Returns the number of files written; `inflight` is left
    empty."""
    import threading
    import torch
    from ...context import Context
    lock = threading.Lock()
    errors = []
    n_files = [0]

    def drain(limit_batches, limit_bytes):
        # wait for the oldest batches' writes while more than `limit_batches` are in flight or
        # their pinned bytes exceed `limit_bytes` (the newest batch always proceeds)
        while True:
            with lock:
                if not (len(inflight) > limit_batches or (len(inflight) > 1 and sum(
                        getattr(j, 'render_bytes', 0) for j, _ in inflight) > limit_bytes)):
                    return
                j, fs = inflight.pop(0)
            if not isinstance(j, list):
                n = len(j.result())
                with lock:
                    n_files[0] += n
            for f in fs:
                f.result()

    def worker(k):
        try:
            wctx = ctx0
            if k > 0:
                wctx = Context(vocab, do_lower_case=True, device=ctx0.device.index)
                if args.sentence_splitter == 'gpu':
                    from ... import punkt
                    punkt.set_params(wctx, getattr(ctx0, '_punkt_params', None))
            st = torch.cuda.Stream(device=wctx.device)
            wt = _StageTimer(args.profile_stages)  # this worker's stages (its own stream)
            timers.append(wt)
            with torch.cuda.device(wctx.device), torch.cuda.stream(st):
                while not errors:
                    with lock:
                        item = next(batch_it, None)
                    if item is None:
                        return
                    batch, corpus = item
                    _trace('batch_ready', batch[0][0] if batch else -1)
                    futs = []
                    wt.mark()
                    job = process_batch(wctx, args, batch, corpus, outdir, wt, pool, futs, copier)
                    with lock:
                        if isinstance(job, list):
                            n_files[0] += len(job)
                        inflight.append((job, futs))
                    drain(n_workers + 1, args.max_inflight_render_bytes)
                st.synchronize()
        except BaseException as e:  # noqa: B902 - re-raised by the caller
            errors.append(e)

    timers = []
    threads = [threading.Thread(target=worker, args=(k,), name='gpu-worker-{}'.format(k))
               for k in range(n_workers)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    drain(0, 0)
    if timer is not None and timer.enabled:  # per-stage seconds summed over the workers
        for wt in timers:
            for k, v in wt.acc.items():
                timer.acc[k] = timer.acc.get(k, 0.0) + v
        timer.acc['gpu_workers'] = n_workers
    return n_files[0]


def _warm_parquet_writer(outdir):
    import pyarrow as pa
    import pyarrow.parquet as pq
    fn = os.path.join(outdir, '.lddl_amd_warmup.{}.parquet'.format(os.getpid()))
    try:
        pq.write_table(pa.table({'A': pa.array(['x'])}), fn)
    finally:
        if os.path.exists(fn):
            os.remove(fn)


def main(args):
    if args.bin_size is not None:
        if args.bin_size > args.target_seq_length:
            raise ValueError('Please provide a bin size that is <= target-seq-length')
        if args.target_seq_length % args.bin_size != 0:
            raise ValueError('Please provide a bin size that can divide the target '
                             'sequence length.')
    if args.output_format not in ('parquet', 'txt'):
        raise ValueError('Format {} not supported!'.format(args.output_format))
    if args.num_shards is not None and args.output_format != 'parquet':
        raise ValueError('--num-shards writes balanced parquet shards only')
    if args.num_shards is not None and args.num_shards < 1:
        raise ValueError('--num-shards must be >= 1')
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    vocab = _resolve_vocab(args.vocab_file)
    tic = time.perf_counter()
    _trace('main', -1)
    outdir = expand_outdir_and_mkdir(args.sink)
    blocks = plan_partitions(args)
    args.n_partitions = len(blocks)
    _trace('planned', -1)
    if args.sentence_splitter == 'host':
        # host segmentation first: its process pool forks before this process touches the GPU
        batches = [(b, ('sentences',) + build_corpus(b, args.local_n_workers))
                   for b in iter_batches(args, rank, world, blocks)]
    else:
        # the host reader starts now, in its own thread, overlapping the device setup below
        batches = _prefetch(iter_doc_batches(args, rank, world, blocks))
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=max(1, args.write_threads))
    # pyarrow's parquet writer initialises lazily on its first file (~0.3-0.8 s, measured on the
    # box): one tiny write on a writer thread now overlaps that with the setup and the first batch
    pool.submit(_warm_parquet_writer, outdir)
    _trace('setup_start', -1)
    import torch
    import torch.distributed as dist
    if world > 1:
        if os.environ.get('LDDL_SHARE_DEVICE') == '1':
            # every rank on device 0, gloo collectives staged through host memory: a rehearsal
            # of the multi-rank path on a one-GPU machine (never how a node is run)
            torch.cuda.set_device(0)
            if not dist.is_initialized():
                dist.init_process_group('gloo')
        else:
            torch.cuda.set_device(local)
            if not dist.is_initialized():
                dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    from ...context import Context
    ctx = Context(vocab, do_lower_case=True)  # BertTokenizerFast default, SURVEY H5
    if args.sentence_splitter == 'gpu':
        from ... import punkt
        punkt.set_params(ctx, punkt_params(args))
    # (only when the read outlasts the setup: with less than one GPU batch of input per rank the
    # warm-up would sit on the critical path; 1 GB seq 128: segment 0.06-0.09 -> 0.035 s, the run
    # 1.36-1.47 -> 1.26-1.39 s on one box, profiles/r05s_*)
    warm = os.environ.get('LDDL_CLI_WARMUP', '1') != '0' and \
        sum(b.nbytes for b in blocks) >= world * args.gpu_batch_bytes
    if args.sentence_splitter == 'gpu' and warm:
        _warm_gpu_path(ctx, args)
    timer = _StageTimer(args.profile_stages)
    _trace('setup_end', -1)
    timer.mark()
    n_files = 0
    pending = []  # writes of the previous batch (at most two batches of rendered rows in memory)
    stream = writers = None
    if args.num_shards is not None and args.balance_plan == 'stream':
        from ...balance import StreamBalancer
        binned = args.bin_size is not None
        bin_size = args.bin_size if binned else args.target_seq_length
        nbins = args.target_seq_length // bin_size
        stream = StreamBalancer(ctx, bin_size, nbins, num_shards=args.num_shards)
        from ...balance import shard_owner
        writers = ShardWriters(outdir, nbins, binned, args.masking, pool,
                               n_local_shards=int((shard_owner(args.num_shards, world) == rank).sum()),
                               max_open=args.max_open_files,
                               max_inflight_bytes=args.max_inflight_render_bytes)
    copier = ThreadPoolExecutor(max_workers=1)  # device -> host copies of rendered batches
    inflight = []  # (copy future, write futures) of the batches not yet written
    batch_it = iter(batches)
    gpu_workers = max(1, int(getattr(args, 'gpu_workers', 1) or 1))
    if stream is None and gpu_workers > 1:
        # Several GPU batches in flight: a batch's replay planner is one sequential chain per
        # partition (~0.1 s for a 1 MiB partition whatever the batch size), so one batch of a few
        # hundred partitions leaves the GPU mostly idle while it runs. Each worker thread owns a
        # Context and a stream, takes the next batch from the reader and runs it through the
        # whole GPU path; batches are independent (files are named by partition), so they may
        # finish in any order.
        n_files += _run_gpu_workers(args, gpu_workers, vocab, ctx, batch_it, outdir, pool, copier,
                                    inflight, timer)
        timer.mark()
        batch_it = iter(())
    while True:
        item = next(batch_it, None)
        if stream is not None and world > 1:
            # every rank steps the balancer until no rank has a batch left: the loop ends on the
            # iterators themselves (one tiny all-reduce per step), never on a separate count
            if not _any_rank(item is not None, ctx.device):
                break
            if item is None:  # this rank is out of batches: it still takes part in the exchange
                writers.add(ctx, stream.step(_empty_pairs(ctx, args.masking)), copier)
                continue
        elif item is None:
            break
        batch, corpus = item
        timer('read')
        _trace('batch_ready', batch[0][0] if batch else -1)
        if stream is None:
            futs = []
            job = process_batch(ctx, args, batch, corpus, outdir, timer, pool, futs, copier)
            if isinstance(job, list):
                n_files += len(job)
            inflight.append((job, futs))
            # at most two rendered batches in host memory besides this one, and no more pinned
            # bytes than --max-inflight-render-bytes (the newest batch always proceeds)
            while len(inflight) > 2 or (len(inflight) > 1 and sum(
                    getattr(j, 'render_bytes', 0) for j, _ in inflight) > args.max_inflight_render_bytes):
                j, fs = inflight.pop(0)
                if not isinstance(j, list):
                    n_files += len(j.result())
                for f in fs:
                    f.result()
            timer('write_wait')
        else:
            bb = stream.step(make_batch_pairs(ctx, args, batch, corpus, timer))
            timer('balance')
            writers.add(ctx, bb, copier)
            del bb
            timer('render')
        timer.mark()
    for f in pending:
        f.result()
    for j, fs in inflight:
        if not isinstance(j, list):
            n_files += len(j.result())
        for f in fs:
            f.result()
    timer('write_wait')
    if stream is not None:
        n_files += len(writers.close())
        timer('write_wait')
        if rank == 0:
            with open(os.path.join(outdir, '.num_samples.json'), 'w') as f:
                json.dump(num_samples_of_shards(stream.all_shard_counts, binned), f)
    copier.shutdown()
    pool.shutdown()
    if world > 1:
        dist.barrier()
    if rank == 0 and stream is None and args.output_format == 'parquet':
        from ... import output
        output.write_dataset_metadata(outdir, len(blocks),
                                      None if args.bin_size is None else
                                      args.target_seq_length // args.bin_size)
    if args.num_shards is not None and args.balance_plan == 'reference':
        # the reference's second job over the part files: balance_dask_output in place
        # (load_balance.py:381-418), its exact shard layout, originals deleted
        from .. import load_balance as LB
        if world > 1:
            dist.barrier()
        LB.main(LB.attach_args().parse_args(['--indir', outdir, '--num-shards',
                                             str(args.num_shards)]))
    if rank == 0:
        print('Running the dask pipeline took {} s'.format(time.perf_counter() - tic))
        if args.profile_stages:
            print('stage seconds (rank 0{}): '.format(
                ', summed over {} GPU workers'.format(timer.acc['gpu_workers'])
                if 'gpu_workers' in timer.acc else '') + json.dumps(
                {k: round(v, 3) for k, v in timer.acc.items() if k != 'gpu_workers'}))
            hs = torch.cuda.host_memory_stats()  # torch's pinned host allocator
            print('pinned host memory peak (rank 0): {:.2f} GB'.format(max(
                [v for k, v in hs.items() if 'bytes' in k and k.endswith('peak')] or [0]) / 1e9))
    if world > 1:
        dist.barrier()
    return n_files


def attach_args(parser=None):
    parser = parser or argparse.ArgumentParser(
        'LDDL preprocessor for the BERT pretraining task (MI355X data plane): text shards under '
        "'source' directories -> parquet shards under --sink, input to the load balancer.")
    parser.add_argument('--schedule', type=str, default='mpi', choices=['mpi', 'local'],
                        help='mpi: one process per GPU under torchrun (partitions striped over '
                        'ranks); local: this process only. Default: mpi')
    parser.add_argument('--local-n-workers', type=int, default=min(os.cpu_count() or 1, 16),
                        help='host processes for sentence segmentation. Default: min(cpus, 16)')
    parser.add_argument('--local-threads-per-worker', type=int, default=1,
                        help='accepted for compatibility. Default: 1')
    parser.add_argument('--wikipedia', type=str, default=None,
                        help="path to the 'source' subdirectory of the Wikipedia corpus")
    parser.add_argument('--books', type=str, default=None,
                        help="path to the 'source' subdirectory of the books corpus")
    parser.add_argument('--common-crawl', type=str, default=None,
                        help="path to the 'source' subdirectory of the Common Crawl corpus")
    parser.add_argument('--sink', type=str, default=None, required=True,
                        help='output directory (parquet or txt files)')
    parser.add_argument('--output-format', type=str, default='parquet',
                        choices=['parquet', 'txt'], help='Default: parquet')
    parser.add_argument('--wikipedia-lang', type=str, default='en', choices=['en', 'zh'],
                        help='Default: en')
    parser.add_argument('--target-seq-length', type=int, default=128,
                        help='maximum tokens of [CLS] A [SEP] B [SEP]. Default: 128')
    parser.add_argument('--short-seq-prob', type=float, default=0.1,
                        help='probability of a shorter random target length. Default: 0.1')
    parser.add_argument('--block-size', type=functools.partial(parse_str_of_num_bytes,
                                                               return_str=False),
                        default=None, metavar='n[KMG]',
                        help='bytes per input block (= partition = output shard)')
    parser.add_argument('--num-blocks', type=int, default=None,
                        help='number of input blocks (alternative to --block-size)')
    parser.add_argument('--bin-size', type=int, default=None,
                        help='enable sequence binning with this stride of num_tokens')
    parser.add_argument('--sample-ratio', type=float, default=0.9,
                        help='fraction of documents kept. Default: 0.9')
    parser.add_argument('--seed', type=int, default=12345, help='Default: 12345')
    parser.add_argument('--duplicate-factor', type=int, default=5, help='Default: 5')
    parser.add_argument('--vocab-file', type=str, default='bert-large-uncased',
                        help='path to a BERT vocab.txt (offline: no model-name download)')
    attach_bool_arg(parser, 'masking', default=False,
                    help_str='static masking in the preprocessor (default: off = dynamic '
                    'masking in the data loader)')
    parser.add_argument('--masked-lm-ratio', type=float, default=0.15, help='Default: 0.15')
    parser.add_argument('--gpu-batch-bytes', type=int, default=512 << 20,
                        help='lddl_amd: input text bytes per GPU batch of partitions (bounds HBM '
                             'use; consecutive batches overlap their GPU work, rendering and file '
                             'writes; does not change the part.* output). Default: 512 MiB '
                             '(1 GB end to end: 570 MB/s at 256 MiB, 618 at 512 MiB, 468 at 1 GiB)')
    parser.add_argument('--read-threads', type=int, default=min(os.cpu_count() or 1, 16),
                        help='lddl_amd: host threads of the input reader (GPU segmentation path). '
                             'Default: min(cpus, 16)')
    parser.add_argument('--shuffle-group-bytes', type=int, default=1 << 30,
                        help='lddl_amd: documents are shuffled across the partitions of runs of '
                             'this many input bytes (the reference shuffles globally, '
                             'pretrain.py:100-111; INTEGRATION.md)')
    parser.add_argument('--sentence-splitter', choices=['gpu', 'host'], default='gpu',
                        help='gpu: Punkt on the GPU (exact nltk PunktSentenceTokenizer); host: '
                             "nltk's sent_tokenize in host processes (requires nltk)")
    parser.add_argument('--punkt-params', type=str, default=None,
                        help='JSON PunktParameters (abbrev_types, collocations, sent_starters, '
                             'ortho_context); default: nltk English model if loadable, else '
                             'untrained')
    parser.add_argument('--rng', choices=['replay', 'native'], default='replay',
                        help="lddl_amd: 'replay' reproduces CPython random per partition "
                             "(random.seed(partition seed)), bit-exact with the reference; "
                             "'native' draws the same distributions from Philox counter streams "
                             "keyed by --seed (documents and pairs in parallel)")
    parser.add_argument('--num-shards', type=int, default=None,
                        help="lddl_amd: write the load balancer's layout (shard-<k>.parquet[_<b>] "
                             'with N or N+1 samples per bin + .num_samples.json) instead of '
                             'part.* files (see --balance-plan)')
    parser.add_argument('--balance-plan', choices=['stream', 'reference'], default='stream',
                        help="lddl_amd, with --num-shards: 'stream' balances each GPU batch in "
                             "HBM as it is produced (per-rank shard quotas from the all-gathered "
                             "bin counts: only each bin's surplus over a rank's quota crosses "
                             "ranks, and every shard ends each batch with N or N+1 rows per bin; "
                             "one batch resident); 'reference' writes "
                             "the part files and runs balance_dask_output over them, the "
                             "reference's exact shard layout")
    parser.add_argument('--max-inflight-render-bytes', type=int, default=_default_inflight_bytes(),
                        help='pinned host bytes of rendered batches waiting for their parquet '
                             'writes (default: 1/8 of host memory, 2-16 GiB); the GPU waits for '
                             'the writes beyond it; the newest batch always proceeds, so the peak is this '
                             'bound plus one rendered batch')
    parser.add_argument('--max-open-files', type=int, default=None,
                        help='--num-shards: most shard files kept open at once (default: as many '
                             'as RLIMIT_NOFILE allows, raised to its hard limit); above it, each '
                             'batch is written as a piece and the pieces are merged at the end')
    parser.add_argument('--gpu-workers', type=int, default=1,
                        help='lddl_amd: GPU batches processed concurrently, each by a host thread '
                             'with its own stream (without --num-shards; the balanced path keeps '
                             'batch order). Default: 1')
    parser.add_argument('--write-threads', type=int, default=min(os.cpu_count() or 1, 16),
                        help='lddl_amd: parquet files written concurrently (threads). Default: '
                             'min(cpus, 16)')
    attach_bool_arg(parser, 'profile-stages', default=False,
                    help_str='lddl_amd: print device-synchronised seconds per stage (read, h2d, '
                    'segment, tokenize, pairs, render, write, balance)')
    return parser


def console_script():
    main(attach_args().parse_args())


if __name__ == '__main__':
    sys.exit(0 if console_script() is None else 0)
