"""`preprocess_bert_pretrain` — drop-in for the reference's `lddl.dask.bert.pretrain`
(lddl/dask/bert/pretrain.py:563-884): same flags, same output layout, GPU data plane.

Pipeline (reference call stack in SURVEY.md §3.1):
  read `*.txt` sources into blocks (readers.py)            -> lddl_amd.dask.readers (host)
  random shuffle of documents over partitions (100-111)    -> seeded permutation (host; the
                                                              reference's is unseeded)
  split_id_text (readers.py:131-136)                       -> host, per line
  sent_tokenize + strip + drop empty (86-88)               -> lddl_segment_* (HIP Punkt; host
                                                              segment.py with --sentence-splitter host)
  tokenizer.tokenize(s, max_length=512, truncation=True)   -> lddl_tokenize (HIP)
  _to_partition_pairs / create_pairs_from_document /
    create_masked_lm_predictions (386-402, 241-365, 182-238) -> lddl_pairs_plan / emit (HIP)
  _to_dataframe_binned (binning.py:63-93)                  -> lddl_bin_partitions (HIP)
  instance dict + serialize_np_array (345-358)             -> lddl_render_* (HIP)
  to_parquet / write_partition_binned                      -> pyarrow writer (host)

Random state: the reference draws from each Dask worker's unseeded global `random` (H1). Here
partition p is processed as if `random.seed(partition_seed(--seed, p))` had been called before
its `_to_partition_pairs`, which the test-suite replays bit for bit on the CPU.

Multi-GPU (`--schedule mpi`, launched with torchrun): rank r owns partitions p with
p % world_size == r (partitions are independent); there is no data-path collective.
"""
import argparse
import functools
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


def get_partitions(args, rank=0, world=1):
    """Partitions (lists of raw document lines) owned by `rank`, after sampling and the shuffle."""
    blocksize = args.block_size
    if args.num_blocks is not None:
        if blocksize is not None:
            raise ValueError('Only one of num_blocks or blocksize needs to be set!')
        blocksize = readers.estimate_block_size((args.wikipedia, args.books, args.common_crawl),
                                                args.num_blocks)
    parts = []
    if args.wikipedia is not None:
        parts += readers.read_wikipedia(args.wikipedia, args.wikipedia_lang, blocksize,
                                        args.sample_ratio, args.seed)
    if args.books is not None:
        parts += readers.read_books(args.books, blocksize, args.sample_ratio, args.seed)
    if args.common_crawl is not None:
        parts += readers.read_common_crawl(args.common_crawl, blocksize, args.sample_ratio,
                                           args.seed)
    mine = [p for p in range(len(parts)) if p % world == rank]
    # shuffle documents over this rank's partitions, keeping each partition's document count
    docs = [d for p in mine for d in parts[p]]
    random.Random(partition_seed(args.seed, -1 - rank)).shuffle(docs)
    out, k = [], 0
    for p in mine:
        n = len(parts[p])
        out.append((p, docs[k:k + n]))
        k += n
    return out


def _segment_docs(lines):
    out = []
    for raw in lines:
        _, sents = segment.document_sentences(raw)
        out.append([s.encode('utf-8') for s in sents])
    return out


def build_corpus(partitions, workers=1):
    """Flatten partitions into the device corpus layout: text bytes, sentence byte offsets,
    document sentence offsets, partition document offsets."""
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
        for raw in lines:
            chunks.append(readers.split_id_text(raw)[1].encode('utf-8'))
    text = np.frombuffer(b''.join(chunks), np.uint8) if chunks else np.zeros(0, np.uint8)
    doc_off = np.zeros(len(chunks) + 1, np.int64)
    np.cumsum([len(c) for c in chunks], out=doc_off[1:])
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


def process_batch(ctx, args, partitions, corpus, outdir):
    """Run the GPU hot path over a group of partitions and write their files."""
    import torch
    from ...pairs import make_pairs
    from ... import output
    dev = ctx.device
    if corpus[0] == 'documents':  # GPU Punkt: sentences of every document of the batch
        from ... import punkt
        _, text, doc_off, part_doc_off = corpus
        d_text = torch.from_numpy(text).to(dev) if len(text) else torch.zeros(
            1, dtype=torch.uint8, device=dev)[:0]
        d_so, d_dso = punkt.segment(ctx, d_text, torch.from_numpy(doc_off).to(dev))
    else:
        _, text, sent_off, doc_sent_off, part_doc_off = corpus
        d_text = torch.from_numpy(text).to(dev) if len(text) else torch.zeros(
            1, dtype=torch.uint8, device=dev)[:0]
        d_so = torch.from_numpy(sent_off).to(dev)
        d_dso = torch.from_numpy(doc_sent_off).to(dev)
    ids, sent_len = ctx.tokenize(d_text, d_so, max_pieces=512)
    seeds = np.asarray([partition_seed(args.seed, p) for p, _ in partitions], np.int64)
    pb = make_pairs(ctx, d_so, ids, sent_len, d_dso,
                    torch.from_numpy(part_doc_off).to(dev), torch.from_numpy(seeds).to(dev),
                    seq=args.target_seq_length, dup=args.duplicate_factor, masking=args.masking,
                    short_seq_prob=args.short_seq_prob, masked_lm_ratio=args.masked_lm_ratio,
                    rng=getattr(args, 'rng', 'replay'), native_seed=args.seed)
    part_rows = pb.part_off.cpu().numpy()
    index = [p for p, _ in partitions]
    if args.bin_size is not None:
        nbins = args.target_seq_length // args.bin_size
        nt = ((pb.tok_off[1:] - pb.tok_off[:-1]) + 3).to(torch.int32)
        perm, bin_id, counts = output.bin_partitions(ctx, nt, pb.part_off, args.bin_size, nbins)
        rd = output.render(ctx, pb, perm, bin_id)
        counts = counts.cpu().numpy()
    else:
        nbins, counts = None, None
        rd = output.render(ctx, pb)
    if args.output_format == 'parquet':
        return output.write_parquet(outdir, rd, part_rows, index, args.masking, nbins, counts)
    return write_txt(outdir, rd, part_rows, index, args.masking, nbins, counts)


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


def write_txt(outdir, rd, part_rows, index, masking, nbins, counts):
    """Debug output (`--output-format txt`): dask's to_textfiles names partition i `<i>.txt`;
    the binned writer (binning.py:439-509) adds `_<bin>`."""
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
            fn = os.path.join(outdir, '{}.txt'.format(index[p]) if b is None else
                              '{}.txt_{}'.format(index[p], b))
            with open(fn, 'w') as f:
                for r in range(a, z):
                    f.write(_txt_line(rd.row(r), masking) + '\n')
            paths.append(fn)
    return paths


def _batches(partitions, max_bytes):
    cur, size = [], 0
    for p, lines in partitions:
        b = sum(len(x) for x in lines)
        if cur and size + b > max_bytes:
            yield cur
            cur, size = [], 0
        cur.append((p, lines))
        size += b
    if cur:
        yield cur


def main(args):
    if args.bin_size is not None:
        if args.bin_size > args.target_seq_length:
            raise ValueError('Please provide a bin size that is <= target-seq-length')
        if args.target_seq_length % args.bin_size != 0:
            raise ValueError('Please provide a bin size that can divide the target '
                             'sequence length.')
    if args.output_format not in ('parquet', 'txt'):
        raise ValueError('Format {} not supported!'.format(args.output_format))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    vocab = _resolve_vocab(args.vocab_file)
    tic = time.perf_counter()
    outdir = expand_outdir_and_mkdir(args.sink)
    partitions = get_partitions(args, rank, world)
    if args.sentence_splitter == 'gpu':
        batches = [(b, build_doc_corpus(b)) for b in _batches(partitions, args.gpu_batch_bytes)]
    else:  # host segmentation first: its process pool forks before this process touches the GPU
        batches = [(b, ('sentences',) + build_corpus(b, args.local_n_workers))
                   for b in _batches(partitions, args.gpu_batch_bytes)]
    import torch
    if world > 1:
        torch.cuda.set_device(local)
    from ...context import Context
    ctx = Context(vocab, do_lower_case=True)  # BertTokenizerFast default, SURVEY H5
    if args.sentence_splitter == 'gpu':
        from ... import punkt
        punkt.set_params(ctx, punkt_params(args))
    n_files = 0
    for batch, corpus in batches:
        n_files += len(process_batch(ctx, args, batch, corpus, outdir))
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group('gloo')
        dist.barrier()
    if rank == 0:
        print('Running the dask pipeline took {} s'.format(time.perf_counter() - tic))
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
    parser.add_argument('--gpu-batch-bytes', type=int, default=1 << 30,
                        help='lddl_amd: input text bytes per GPU batch of partitions')
    parser.add_argument('--sentence-splitter', choices=['gpu', 'host'], default='gpu',
                        help='gpu: Punkt on the GPU (exact nltk PunktSentenceTokenizer); host: '
                             'lddl_amd.dask.bert.segment (nltk if importable, else rules)')
    parser.add_argument('--punkt-params', type=str, default=None,
                        help='JSON PunktParameters (abbrev_types, collocations, sent_starters, '
                             'ortho_context); default: nltk English model if loadable, else '
                             'untrained')
    parser.add_argument('--rng', choices=['replay', 'native'], default='replay',
                        help="lddl_amd: 'replay' reproduces CPython random per partition "
                             "(random.seed(partition seed)), bit-exact with the reference; "
                             "'native' draws the same distributions from Philox counter streams "
                             "keyed by --seed (documents and pairs in parallel)")
    return parser


def console_script():
    main(attach_args().parse_args())


if __name__ == '__main__':
    sys.exit(0 if console_script() is None else 0)
