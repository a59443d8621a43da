"""Output stage on the GPU: per-partition binning (vs the reference's _to_dataframe_binned
goldens and the oracle), string/npy rendering (vs Python ' '.join / np.save) and the
`preprocess_bert_pretrain` CLI end to end (parquet files vs the oracle replay)."""
import io
import json
import os

import numpy as np
import pyarrow.parquet as pq
import pytest

from conftest import GOLDEN, VOCAB_UNCASED

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def ctx():
    from lddl_amd.context import Context
    return Context(VOCAB_UNCASED, True)


def test_bin_golden(ctx):
    import torch
    from lddl_amd.output import bin_partitions
    with open(os.path.join(GOLDEN, 'binning.json')) as f:
        cases = json.load(f)
    for c in cases:
        nt = np.asarray(c['num_tokens'], np.int32)
        nbins = c['seq'] // c['bin_size']
        d_nt = torch.from_numpy(nt).cuda()
        off = torch.tensor([0, len(nt)], dtype=torch.int64).cuda()
        perm, bin_id, counts = bin_partitions(ctx, d_nt, off, c['bin_size'], nbins)
        assert perm.cpu().tolist() == c['uid_order']
        assert bin_id.cpu().tolist() == c['bin_id']
        assert counts.cpu().numpy().sum() == len(nt)


def test_bin_many_partitions_vs_oracle(ctx):
    import torch
    from oracle import oracle as O
    from lddl_amd.output import bin_partitions
    rng = np.random.default_rng(3)
    sizes = rng.integers(0, 3000, 40)
    sizes[5] = 0
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    for seq, bs in ((512, 8), (128, 32), (512, 1)):
        nb = seq // bs
        nt = rng.integers(5, seq + 1, off[-1]).astype(np.int32)
        perm, bin_id, counts = bin_partitions(ctx, torch.from_numpy(nt).cuda(),
                                              torch.from_numpy(off).cuda(), bs, nb)
        perm, bin_id, counts = perm.cpu().numpy(), bin_id.cpu().numpy(), counts.cpu().numpy()
        # the same rows given as a pair table's token offsets (num_tokens = len(A)+len(B)+3)
        tok_off = np.concatenate([[0], np.cumsum(nt.astype(np.int64) - 3)]).astype(np.int64)
        p2, b2, c2 = bin_partitions(ctx, None, torch.from_numpy(off).cuda(), bs, nb,
                                    tok_off=torch.from_numpy(tok_off).cuda())
        np.testing.assert_array_equal(p2.cpu().numpy(), perm)
        np.testing.assert_array_equal(b2.cpu().numpy(), bin_id)
        np.testing.assert_array_equal(c2.cpu().numpy(), counts)
        for p in range(len(sizes)):
            a, z = off[p], off[p + 1]
            eb, eo, ec = O.bin_samples(nt[a:z], bs, nb)
            np.testing.assert_array_equal(perm[a:z] - a, eo)
            np.testing.assert_array_equal(bin_id[a:z], eb[eo])
            np.testing.assert_array_equal(counts[p], ec)


def _py_rows(pairs, vocab, order=None):
    """The reference's instance dicts (pretrain.py:345-358) from oracle/GPU pair arrays."""
    rows = []
    n = len(pairs['len_a'])
    for q in (range(n) if order is None else order):
        t = pairs['tokens'][pairs['tok_off'][q]:pairs['tok_off'][q + 1]]
        na = pairs['len_a'][q]
        d = {'A': ' '.join(vocab[i] for i in t[:na]), 'B': ' '.join(vocab[i] for i in t[na:]),
             'is_random_next': bool(pairs['is_random_next'][q]),
             'num_tokens': int(len(t) + 3)}
        if 'pos' in pairs:
            p0, p1 = pairs['pos_off'][q], pairs['pos_off'][q + 1]
            buf = io.BytesIO()
            np.save(buf, np.asarray(pairs['pos'][p0:p1], np.uint16))
            d['masked_lm_positions'] = buf.getvalue()
            d['masked_lm_labels'] = ' '.join(vocab[i] for i in pairs['labels'][p0:p1])
        rows.append(d)
    return rows


def test_render_matches_python(ctx):
    import torch
    from lddl_amd import synth
    from lddl_amd.pairs import make_pairs
    from lddl_amd.output import render
    corp = synth.generate(seed=5, n_bytes=200_000, nonascii_frac=0.05)
    text = torch.from_numpy(corp.text).cuda()
    so = torch.from_numpy(corp.sent_off).cuda()
    ids, sl = ctx.tokenize(text, so)
    part = torch.tensor([0, corp.n_doc], dtype=torch.int64).cuda()
    for masking in (True, False):
        pb = make_pairs(ctx, so, ids, sl, torch.from_numpy(corp.doc_sent_off).cuda(), part,
                        torch.tensor([9], dtype=torch.int64).cuda(), seq=128, dup=2,
                        masking=masking)
        h = pb.to_host()
        order = np.random.default_rng(1).permutation(pb.n_pairs)
        rd = render(ctx, pb, torch.from_numpy(order).cuda())
        exp = _py_rows(h, ctx.tokens, order)
        for r in range(0, pb.n_pairs, 7):
            assert rd.row(r) == exp[r]


def _write_source(root, n_docs=300, seed=11):
    from lddl_amd import synth
    corp = synth.generate(seed=seed, n_bytes=n_docs * 3000, nonascii_frac=0.02)
    docs = corp.documents()
    os.makedirs(os.path.join(root, 'en'))
    lines = ['wiki-{} {}'.format(i, ' '.join(d)) for i, d in enumerate(docs)]
    half = len(lines) // 2
    for k, chunk in enumerate((lines[:half], lines[half:])):
        with open(os.path.join(root, 'en', 'wiki_{}.txt'.format(k)), 'w') as f:
            f.write('\n'.join(chunk) + '\n\n')


@pytest.mark.parametrize('binned,params,workers,chunk', [(False, False, 1, None),
                                                          (True, False, 2, 1),
                                                          (False, True, 2, 0),
                                                          (True, False, 3, None),
                                                          (False, False, 1, 1)])
def test_pretrain_cli_vs_oracle(tmp_path, monkeypatch, binned, params, workers, chunk):
    """CLI output == the oracle's rows per partition. workers = 3: one partition per GPU batch
    (--gpu-batch-bytes 1) over three concurrent GPU worker threads (--gpu-workers). chunk: the
    rendered batch's device-to-host copy in partition groups of that many bytes (1: one
    partition per group; 0: the whole batch at once; None: the default 128 MiB)."""
    from lddl_amd import synth
    from lddl_amd.dask.bert import pretrain as P
    if chunk is not None:
        monkeypatch.setattr(P, '_D2H_CHUNK_BYTES', chunk)
    from oracle import oracle as O
    src = tmp_path / 'source'
    _write_source(str(src))
    sink = tmp_path / 'out'
    argv = ['--schedule', 'local', '--wikipedia', str(src), '--sink', str(sink), '--masking',
            '--target-seq-length', '128', '--num-blocks', '4', '--seed', '7',
            '--vocab-file', VOCAB_UNCASED, '--local-n-workers', '1', '--duplicate-factor', '2',
            '--gpu-workers', str(workers)]
    if workers > 2:
        argv += ['--gpu-batch-bytes', '1', '--shuffle-group-bytes', '1']
    if binned:
        argv += ['--bin-size', '32']
    prm = None
    if params:  # trained Punkt parameters through --punkt-params
        prm_path = os.path.join(GOLDEN, 'punkt_params.json')
        argv += ['--punkt-params', prm_path]
        with open(prm_path) as f:
            prm = json.load(f)
    args = P.attach_args().parse_args(argv)
    P.main(args)
    # CPU replay: the same host partitions, the oracle tokenizer + pair/mask replay
    args = P.attach_args().parse_args(argv)
    parts = P.get_partitions(args)
    tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
    vocab = [l.rstrip('\n') for l in open(VOCAB_UNCASED, encoding='utf-8')]
    cls, sep, msk = (tok.token_id(t) for t in ('[CLS]', '[SEP]', '[MASK]'))
    punkt = O.Punkt(prm)  # the CLI segments on the GPU: nltk's Punkt (untrained or params)
    for p, lines in parts:
        _, dtext, doc_off, _ = P.build_doc_corpus([(p, lines)])
        st, en, cnt = punkt.spans(dtext, doc_off)
        docs, k = [], 0
        for d in range(len(doc_off) - 1):
            ss = [bytes(dtext[doc_off[d] + st[j]:doc_off[d] + en[j]]).decode().strip()
                  for j in range(k, k + cnt[d])]
            docs.append([x for x in ss if x])
            k += cnt[d]
        corp = synth.from_documents(docs)
        text, so, dso = corp.text, corp.sent_off, corp.doc_sent_off
        ids, off = tok.tokenize(text, so)
        lens = np.diff(off)
        keep = lens > 0
        kpos = np.concatenate([[0], np.cumsum(keep)])
        kd = kpos[dso]
        kd = np.concatenate([kd[:1], kd[1:][np.diff(kd) > 0]])
        k_off = np.concatenate([[0], np.cumsum(lens[keep])])
        out = O.partition_pairs(kd, k_off, ids, P.partition_seed(7, p), 2, 128, True,
                                tok.vocab_size, cls, sep, msk)
        rows = _py_rows(out, vocab)
        if not binned:
            t = pq.read_table(sink / 'part.{}.parquet'.format(p)).to_pylist()
            assert t == rows
        else:
            nt = np.asarray([r['num_tokens'] for r in rows])
            bins = np.minimum((nt - 1) // 32, 3)
            for b in range(4):
                t = pq.read_table(sink / 'part.{}.parquet_{}'.format(p, b)).to_pylist()
                exp = [dict(r, bin_id=b) for r, bb in zip(rows, bins) if bb == b]
                assert t == exp


def test_bin_stable_single_segment_vs_oracle(ctx):
    import torch
    from oracle import oracle as O
    from lddl_amd.output import bin_stable
    rng = np.random.default_rng(9)
    for n, seq, bs in ((0, 512, 8), (1, 128, 32), (5000, 128, 32), (300_001, 512, 8),
                       (70_000, 512, 1)):
        nb = seq // bs
        nt = rng.integers(5, seq + 1, n).astype(np.int32)
        perm, bin_id, counts = bin_stable(ctx, torch.from_numpy(nt).cuda(), bs, nb)
        eb, eo, ec = O.bin_samples(nt, bs, nb)
        np.testing.assert_array_equal(perm.cpu().numpy(), eo)
        np.testing.assert_array_equal(bin_id.cpu().numpy(), eb[eo])
        np.testing.assert_array_equal(counts.cpu().numpy(), ec)


def test_pretrain_cli_native_rng(tmp_path):
    """--rng native: same layout and schema; every row is a valid masked NSP sample."""
    from lddl_amd.dask.bert import pretrain as P
    src = tmp_path / 'source'
    _write_source(str(src))
    sink = tmp_path / 'out'
    argv = ['--schedule', 'local', '--wikipedia', str(src), '--sink', str(sink), '--masking',
            '--target-seq-length', '128', '--num-blocks', '4', '--seed', '7', '--rng', 'native',
            '--vocab-file', VOCAB_UNCASED, '--local-n-workers', '1', '--duplicate-factor', '2',
            '--bin-size', '32']
    P.main(P.attach_args().parse_args(argv))
    n = 0
    for p in range(4):
        for b in range(4):
            t = pq.read_table(sink / 'part.{}.parquet_{}'.format(p, b)).to_pylist()
            for r in t:
                na, nb = len(r['A'].split()), len(r['B'].split())
                assert r['num_tokens'] == na + nb + 3 <= 128 and na >= 1 and nb >= 1
                assert r['bin_id'] == b == min((r['num_tokens'] - 1) // 32, 3)
                pos = np.frombuffer(r['masked_lm_positions'][-2 * len(r['masked_lm_labels'].split()):],
                                    np.uint16)
                assert len(pos) == max(1, int(np.round(r['num_tokens'] * 0.15)))
                assert np.all(np.diff(pos.astype(int)) > 0)
                n += 1
    assert n > 50


def _cli(tmp_path, sink, extra, seq=128, dup=2, masking=True):
    from lddl_amd.dask.bert import pretrain as P
    src = tmp_path / 'source'
    if not src.exists():
        _write_source(str(src))
    argv = ['--schedule', 'local', '--wikipedia', str(src), '--sink', str(sink),
            '--target-seq-length', str(seq), '--num-blocks', '4', '--seed', '7',
            '--vocab-file', VOCAB_UNCASED, '--local-n-workers', '1', '--duplicate-factor',
            str(dup)] + (['--masking'] if masking else []) + extra
    args = P.attach_args().parse_args(argv)
    P.main(args)
    return P.attach_args().parse_args(argv)


@pytest.mark.parametrize('binned', [False, True])
def test_pretrain_cli_dask_metadata(tmp_path, binned):
    """_common_metadata + _metadata as dask's ArrowDatasetEngine.write_metadata leaves them
    (binning.py:325-339, pretrain.py:473-478): row groups of every partition in order, file
    paths part.<i>.parquet (binned: the last bin file's row groups)."""
    from lddl_amd.dask.bert import pretrain as P
    sink = tmp_path / 'out'
    args = _cli(tmp_path, sink, ['--bin-size', '32'] if binned else [])
    n_part = len(P.plan_partitions(args))
    md = pq.read_metadata(sink / '_metadata')
    names = [md.row_group(i).column(0).file_path for i in range(md.num_row_groups)]
    assert names == ['part.{}.parquet'.format(p) for p in range(n_part)]
    suffix = '_3' if binned else ''
    assert md.num_rows == sum(pq.read_metadata(sink / 'part.{}.parquet{}'.format(p, suffix)).num_rows
                              for p in range(n_part))
    assert pq.read_schema(sink / '_common_metadata').equals(
        pq.read_schema(sink / 'part.0.parquet{}'.format(suffix)))


@pytest.mark.parametrize('binned', [False, True])
def test_pretrain_cli_txt_output(tmp_path, binned):
    """--output-format txt (pretrain.py:501-531, binning.py:439-509): the parquet rows of the
    same run as the reference's text lines, dask's file names, no trailing newline."""
    from lddl_amd.dask.bert import pretrain as P
    extra = ['--bin-size', '32'] if binned else []
    args = _cli(tmp_path, tmp_path / 'pq', extra)
    _cli(tmp_path, tmp_path / 'txt', extra + ['--output-format', 'txt'])
    for p in range(len(P.plan_partitions(args))):
        if binned:
            for b in range(4):
                rows = pq.read_table(tmp_path / 'pq' / 'part.{}.parquet_{}'.format(p, b)).to_pylist()
                got = (tmp_path / 'txt' / '{}_{}.txt'.format(p, b)).read_text()
                assert got == '\n'.join(P._txt_line(r, True) for r in rows)
        else:
            rows = pq.read_table(tmp_path / 'pq' / 'part.{}.parquet'.format(p)).to_pylist()
            got = (tmp_path / 'txt' / '{}.txt'.format(p)).read_text()
            assert got == '\n'.join(P._txt_line(r, True) for r in rows)
            if not rows:
                assert got == ''
                continue
            r = rows[0]  # (numpy's array str may wrap a long positions list onto new lines)
            assert got.startswith('is_random_next: {} - [CLS] {} [SEP] {} [SEP] - '
                                  'masked_lm_positions: ['.format(r['is_random_next'], r['A'],
                                                                  r['B']))
            assert '] - masked_lm_labels: {} - {}'.format(r['masked_lm_labels'],
                                                         r['num_tokens']) in got


@pytest.mark.parametrize('binned,masking,chunk', [(True, True, None), (False, False, None),
                                                   (True, True, 1)])
def test_pretrain_cli_num_shards_balanced(tmp_path, monkeypatch, binned, masking, chunk):
    """--num-shards (stream plan, world size 1): per GPU batch, bin b's rows (the part.* rows of
    the batch's partitions, in order) are cut into consecutive runs, shard s taking
    batch_shard_counts' share (N or N+1 per shard after every batch), with .num_samples.json;
    checked for one batch and for one batch per partition (`--gpu-batch-bytes 1`); then
    get_bert_pretrain_data_loader consumes them. chunk = 1: the rendered rows leave the GPU one
    (shard, bin) range at a time."""
    from lddl_amd.balance import batch_shard_counts
    from lddl_amd.dask.bert import pretrain as P0
    seen = []  # whether each sharded batch's ranges tiled its rows (the chunked copy ran)
    real_order = P0._row_order

    def row_order(ranges):
        out = real_order(ranges)
        seen.append(out[2])
        return out
    monkeypatch.setattr(P0, '_row_order', row_order)
    if chunk is not None:
        monkeypatch.setattr(P0, '_D2H_CHUNK_BYTES', chunk)

    def dealt(batches, S):  # batches: bin b's rows per GPU batch -> rows per shard
        out, prior = [[] for _ in range(S)], 0
        for rows in batches:
            n = batch_shard_counts([prior], [len(rows)], S)[:, 0]
            o = 0
            for k in range(S):
                out[k] += rows[o:o + n[k]]
                o += n[k]
            prior += len(rows)
        return out
    import logging
    from lddl_amd.torch import get_bert_pretrain_data_loader
    from lddl_amd.dask.bert import pretrain as P
    extra = (['--bin-size', '32'] if binned else []) + ['--shuffle-group-bytes', '1']
    args = _cli(tmp_path, tmp_path / 'parts', extra, masking=masking)
    _cli(tmp_path, tmp_path / 'shards', extra + ['--num-shards', '4'], masking=masking)
    _cli(tmp_path, tmp_path / 'shards_b', extra + ['--num-shards', '4', '--gpu-batch-bytes', '1'],
         masking=masking)
    nb = 4 if binned else 1
    n_part = len(P.plan_partitions(args))
    assert len(P.rank_batches(P.attach_args().parse_args(
        ['--sink', 'x', '--gpu-batch-bytes', '1', '--shuffle-group-bytes', '1']),
        P.plan_partitions(args))) == n_part  # one batch per partition in shards_b
    assert seen and all(seen)  # every batch took the chunked copy
    ns = json.loads((tmp_path / 'shards' / '.num_samples.json').read_text())
    ns_b = json.loads((tmp_path / 'shards_b' / '.num_samples.json').read_text())
    assert ns == ns_b  # the same counts per shard (N / N+1 after every batch)
    assert len(ns) == 4 * nb
    for b in range(nb):
        sfx = '_{}'.format(b) if binned else ''
        per_part = [pq.read_table(tmp_path / 'parts' / 'part.{}.parquet{}'.format(p, sfx)).to_pylist()
                    for p in range(n_part)]
        one = dealt([[r for rows in per_part for r in rows]], 4)
        each = dealt(per_part, 4)
        counts = []
        for s in range(4):
            fn = 'shard-{}.parquet{}'.format(s, sfx)
            t = pq.read_table(tmp_path / 'shards' / fn)
            assert ns[fn] == t.num_rows
            assert t.to_pylist() == one[s]
            tb = pq.read_table(tmp_path / 'shards_b' / fn)
            assert tb.to_pylist() == each[s]
            assert ns_b[fn] == tb.num_rows
            counts.append(t.num_rows)
        assert max(counts) - min(counts) <= 1
    dl = get_bert_pretrain_data_loader(
        str(tmp_path / 'shards'), vocab_file=VOCAB_UNCASED,
        data_loader_kwargs={'batch_size': 16, 'num_workers': 2}, log_level=logging.WARNING)
    n = sum(batch['input_ids'].size(0) for batch in dl)
    # the loader evens out files to the smallest count per bin (lost-samples rule)
    assert sum(ns.values()) - 4 * nb <= n <= sum(ns.values())


def test_pretrain_cli_num_shards_reference_plan(tmp_path):
    """--balance-plan reference: the part files balanced by balance_dask_output in place — the
    reference's shard layout (its plans are pinned by tests/golden/balance.json)."""
    import shutil
    from lddl_amd.dask import load_balance as LB
    extra = ['--bin-size', '32']
    _cli(tmp_path, tmp_path / 'parts', extra)
    ref = tmp_path / 'ref'
    shutil.copytree(tmp_path / 'parts', ref)
    LB.main(LB.attach_args().parse_args(['--indir', str(ref), '--num-shards', '3']))
    got = tmp_path / 'got'
    _cli(tmp_path, got, extra + ['--num-shards', '3', '--balance-plan', 'reference'])
    names = sorted(os.listdir(ref))
    assert names == sorted(os.listdir(got))
    assert not any(n.startswith('part.') for n in names)
    for n in names:
        if '.parquet' in n:
            assert pq.read_table(got / n).to_pylist() == pq.read_table(ref / n).to_pylist()
    assert (got / '.num_samples.json').read_text() == (ref / '.num_samples.json').read_text()


def test_pretrain_cli_num_shards_piece_mode(tmp_path):
    """--max-open-files below the (shard, bin) file count: each batch is written as a piece and
    the pieces are merged at close — the same files as with every writer open (the
    reference example's 4096 shards x 8 bins exceed the usual 1024-descriptor soft limit)."""
    extra = ['--bin-size', '32', '--shuffle-group-bytes', '1', '--gpu-batch-bytes', '1',
             '--num-shards', '4']
    _cli(tmp_path, tmp_path / 'open', extra)
    _cli(tmp_path, tmp_path / 'pieces', extra + ['--max-open-files', '3'])
    names = sorted(x for x in os.listdir(tmp_path / 'open') if x.startswith('shard-'))
    assert len(names) == 16
    assert sorted(x for x in os.listdir(tmp_path / 'pieces') if not x.startswith('.')) == \
        sorted(x for x in os.listdir(tmp_path / 'open') if not x.startswith('.'))
    for fn in names:
        a = pq.read_table(tmp_path / 'open' / fn)
        b = pq.read_table(tmp_path / 'pieces' / fn)
        assert a.equals(b), fn
        assert pq.ParquetFile(tmp_path / 'pieces' / fn).num_row_groups == \
            pq.ParquetFile(tmp_path / 'open' / fn).num_row_groups


def _cli_world2(tmp_path, sink, extra, env_extra=None):
    import socket
    import subprocess
    import sys
    src = tmp_path / 'source'
    if not src.exists():
        _write_source(str(src))
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    env = dict(os.environ, LDDL_SHARE_DEVICE='1', **(env_extra or {}))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env['PYTHONPATH'] = repo + os.pathsep + env.get('PYTHONPATH', '')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(port), '-m',
           'lddl_amd.dask.bert.pretrain', '--schedule', 'local', '--wikipedia', str(src),
           '--sink', str(sink), '--target-seq-length', '128', '--num-blocks', '2', '--seed', '7',
           '--vocab-file', VOCAB_UNCASED, '--local-n-workers', '1', '--duplicate-factor', '2',
           '--masking'] + extra
    r = subprocess.run(cmd, env=env, cwd=repo, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_pretrain_cli_num_shards_world2_unequal_batches(tmp_path):
    """Two ranks (sharing the one GPU, gloo collectives staged through host memory) with
    different numbers of GPU batches (3 partitions, one batch each: 2 and 1): the collective loop
    ends on the batch iterators themselves, the rank that runs out keeps taking part with empty
    batches, and the shards hold exactly the rows of the same run's part files, N or N+1 per
    shard and bin (termination no longer depends on a second count of the batches)."""
    extra = ['--bin-size', '32', '--shuffle-group-bytes', '1', '--gpu-batch-bytes', '1']
    _cli_world2(tmp_path, tmp_path / 'parts', extra)
    _cli_world2(tmp_path, tmp_path / 'shards', extra + ['--num-shards', '3'])
    n_part = len([x for x in os.listdir(tmp_path / 'parts') if x.endswith('.parquet_0')])
    assert n_part == 3
    ns = json.loads((tmp_path / 'shards' / '.num_samples.json').read_text())
    for b in range(4):
        parts = sorted(str(r) for p in range(n_part) for r in pq.read_table(
            tmp_path / 'parts' / 'part.{}.parquet_{}'.format(p, b)).to_pylist())
        shards, counts = [], []
        for s in range(3):
            t = pq.read_table(tmp_path / 'shards' / 'shard-{}.parquet_{}'.format(s, b))
            assert ns['shard-{}.parquet_{}'.format(s, b)] == t.num_rows
            shards += [str(r) for r in t.to_pylist()]
            counts.append(t.num_rows)
        assert sorted(shards) == parts
        assert max(counts) - min(counts) <= 1
