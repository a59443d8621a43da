"""Host-side pieces that need no GPU: readers, layout utils, sentence segmentation fallback,
CLI flag parity."""
import os
import random

import numpy as np
import pytest

from lddl_amd import utils as U
from lddl_amd.dask import readers as R


def test_parse_str_of_num_bytes():
    assert U.parse_str_of_num_bytes('1k') == 1024
    assert U.parse_str_of_num_bytes('1.5M') == int(1.5 * 1024 ** 2)
    assert U.parse_str_of_num_bytes('2g') == 2 * 1024 ** 3
    assert U.parse_str_of_num_bytes('1024') == 102  # reference quirk kept
    assert U.parse_str_of_num_bytes('8K', return_str=True) == '8K'
    with pytest.raises(ValueError):
        U.parse_str_of_num_bytes('xk')


def test_bin_ids_and_paths():
    paths = ['/a/part.0.parquet_0', '/a/part.0.parquet_1', '/a/part.1.parquet_1']
    assert U.get_all_bin_ids(paths) == [0, 1]
    assert U.get_file_paths_for_bin_id(paths, 1) == paths[1:]
    with pytest.raises(ValueError):
        U.get_all_bin_ids(['/a/part.0.parquet_1'])
    assert U.get_all_bin_ids(['/a/part.0.parquet']) == []


def test_serialize_np_array_roundtrip():
    a = np.asarray([3, 1, 4, 159], np.uint16)
    b = U.serialize_np_array(a)
    assert len(b) == 128 + 8
    np.testing.assert_array_equal(U.deserialize_np_array(b), a)


def test_split_id_text():
    assert R.split_id_text('wiki-1 hello world') == ('wiki-1', 'hello world')
    assert R.split_id_text('wiki-2\tx') == ('wiki-2', 'x')
    assert R.split_id_text('alone') == ('alone', '')


def test_blocks_follow_dask_read_block(tmp_path):
    data = b''.join(b'line%03d xx\n' % i for i in range(50))
    f = tmp_path / 'a.txt'
    f.write_bytes(data)
    for bs in (7, 12, 13, 64, 1000):
        blocks = R.read_blocks([str(f)], bs)
        lines = [l for b in blocks for l in b if l]
        assert lines == data.split(b'\n')[:-1]
        # dask: block k (k > 0) starts after the first newline at or after offset k*bs - 1
        starts = R._block_starts(data, bs)
        for k, s in enumerate(starts[1:-1], 1):
            j = data.find(b'\n', k * bs - 1)
            assert s == j + 1


def test_random_sample_is_dask_semantics(tmp_path):
    d = tmp_path / 'src'
    d.mkdir()
    (d / 'x.txt').write_text(''.join('doc{} text\n'.format(i) for i in range(200)))
    a = R.read_bag_of_text(str(d), None, 0.5, 42)
    b = R.read_bag_of_text(str(d), None, 0.5, 42)
    assert a == b and 60 < len(a[0]) < 140
    # partition 0 state: 624 words of randint(0, 2**32) from Random(42), then random() < p
    r0 = random.Random(42)
    st = (3, tuple(r0.randint(0, 1 << 32) for _ in range(624)) + (624,), None)
    r = random.Random()
    r.setstate(st)
    assert a[0] == ['doc{} text'.format(i) for i in range(200) if r.random() < 0.5]


def test_host_splitter_refuses_without_nltk(monkeypatch):
    """--sentence-splitter host runs nltk's sent_tokenize or nothing (no approximation)."""
    import sys
    from lddl_amd.dask.bert import segment as S
    monkeypatch.setattr(S, '_splitter', None)
    monkeypatch.setitem(sys.modules, 'nltk', None)
    with pytest.raises(RuntimeError, match='needs nltk'):
        S.sent_tokenize('One. Two.')


def test_file_block_starts_match_in_memory_blocks(tmp_path):
    rng = np.random.default_rng(4)
    lines = [b'x' * int(n) for n in rng.integers(0, 300, 400)]
    data = b'\n'.join(lines) + b'\n'
    f = tmp_path / 'a.txt'
    f.write_bytes(data)
    for bs in (1, 7, 100, 4096, 70_000, 10 ** 7):
        assert R._file_block_starts(str(f), bs) == R._block_starts(data, bs)
    # plan + read == the in-memory blocks, filtered
    for bs in (None, 50, 1000):
        got = [R.read_block(b) for b in R.plan_blocks(str(tmp_path), bs)]
        exp = [R._filter(b) for b in R.read_blocks([str(f)], bs)]
        assert got == exp


def test_ranks_read_only_their_blocks(tmp_path, monkeypatch):
    from lddl_amd.dask.bert import pretrain as P
    src = tmp_path / 'src' / 'en'
    src.mkdir(parents=True)
    (src / 'w.txt').write_text(''.join('wiki-{} text {}\n'.format(i, i) for i in range(400)))
    args = P.attach_args().parse_args(['--sink', str(tmp_path / 'o'), '--wikipedia',
                                       str(tmp_path / 'src'), '--num-blocks', '8',
                                       '--sample-ratio', '1.0', '--gpu-batch-bytes', '3000'])
    seen = []
    orig = R.read_block
    monkeypatch.setattr(R, 'read_block', lambda b, **kw: seen.append(b.start) or orig(b, **kw))
    parts = {}
    for rank in range(3):
        seen.clear()
        mine = P.get_partitions(args, rank, 3)
        blocks = P.plan_partitions(args)
        assert sorted(seen) == sorted(blocks[p].start for p in range(len(blocks)) if p % 3 == rank)
        for p, lines in mine:
            assert p % 3 == rank
            parts[p] = lines
    # every document exactly once over all ranks (shuffled inside each rank's batches)
    docs = sorted(d for lines in parts.values() for d in lines)
    assert docs == sorted('wiki-{} text {}'.format(i, i) for i in range(400))


def test_pretrain_flags_match_reference_surface():
    from lddl_amd.dask.bert import pretrain as P
    ap = P.attach_args()
    flags = {a for act in ap._actions for a in act.option_strings}
    want = {'--schedule', '--local-n-workers', '--local-threads-per-worker', '--wikipedia',
            '--books', '--common-crawl', '--sink', '--output-format', '--wikipedia-lang',
            '--target-seq-length', '--short-seq-prob', '--block-size', '--num-blocks',
            '--bin-size', '--sample-ratio', '--seed', '--duplicate-factor', '--vocab-file',
            '--masking', '--no-masking', '--masked-lm-ratio'}
    assert want <= flags
    a = ap.parse_args(['--sink', '/tmp/x'])
    assert (a.target_seq_length, a.short_seq_prob, a.sample_ratio, a.seed, a.duplicate_factor,
            a.masking, a.masked_lm_ratio, a.output_format) == (128, 0.1, 0.9, 12345, 5, False,
                                                               0.15, 'parquet')
    with pytest.raises(ValueError):
        P.main(ap.parse_args(['--sink', '/tmp/x', '--bin-size', '48']))


def test_load_balance_flags():
    from lddl_amd.dask import load_balance as LB
    a = LB.attach_args().parse_args(['--indir', 'x', '--num-shards', '4', '--bin-ids', '0', '2'])
    assert (a.indir, a.outdir, a.num_shards, a.bin_ids, a.keep_orig) == ('x', None, 4, [0, 2],
                                                                          False)


def test_pack_token_counts_match_str_split():
    """The loader's host pack (lddl_amd/torch/bert.py _canon/_ntok) gives the GPU splitter bytes
    whose ASCII-whitespace tokens are the reference's str.split() tokens (bert.py:80-81)."""
    import random
    from lddl_amd.torch.bert import _canon, _ntok
    ws = [' ', '  ', '\t', '\n', '\x0b', '\x0c', '\r', '\x1c', '\x1f', '\x85', '\xa0', ' ',
          ' ', ' ', ' ', ' ', ' ', ' ', '　']
    words = ['the', '##ing', 'café', '–', '’s', '中文', '…', 'x​y', 'a⁠b', '[MASK]']
    rng = random.Random(5)
    cases = ['', ' ', 'a', ' a', 'a ', 'a  b', 'a　b', '\xa0', 'a–b c']
    for _ in range(2000):
        n = rng.randint(0, 8)
        s = ''.join(rng.choice(words) + (rng.choice(ws) if rng.random() < 0.3 else ' ')
                    for _ in range(n))
        if rng.random() < 0.2:
            s = rng.choice(ws) + s
        cases.append(s)
    for s in cases:
        b = _canon(s)
        assert b.split() == [t.encode('utf-8') for t in s.split()], repr(s)
        assert _ntok(b) == len(s.split()), repr(s)


def test_sampled_out_malformed_line_still_raises(tmp_path):
    """dask.bag.read_text decodes the whole block strictly, so a malformed line raises even when
    random_sample would drop it: the GPU path's bytes reader decodes the lines it
    samples out on the host (the kept ones go to lddl_utf8_check)."""
    f = tmp_path / 'a.txt'
    lines = [b'wiki-%d good text %d' % (i, i) for i in range(200)]
    bad = 57
    lines[bad] = b'wiki-57 bad \xff\xfe text'
    f.write_bytes(b'\n'.join(lines) + b'\n')
    for seed in range(100):  # a seed whose sample drops the malformed line
        blocks = R.plan_blocks(str(tmp_path), None, sample_ratio=0.5, sample_seed=seed)
        r = __import__('random').Random()
        r.setstate(blocks[0].state)
        if [r.random() < 0.5 for _ in lines][bad] is False:
            break
    with pytest.raises(UnicodeDecodeError):
        R.read_block(blocks[0], as_bytes=False)
    with pytest.raises(UnicodeDecodeError):
        R.read_block(blocks[0], as_bytes=True)


def test_txt_output_matches_reference_writer(tmp_path):
    """--output-format txt: the CLI's writer (pretrain.write_txt / _txt_line) against the files the
    REFERENCE's own `_save_txt` wrote (pretrain.py:501-531; to_textfiles / to_textfiles_binned,
    binning.py:439-509) for the same rows (tests/golden/make_txt_golden.py): names and bytes."""
    import base64
    import json
    from conftest import GOLDEN
    from lddl_amd.dask.bert import pretrain as P

    class Rows:  # the Rendered.row() interface write_txt reads
        def __init__(self, rows):
            self.rows = rows

        def row(self, r):
            return self.rows[r]
    with open(os.path.join(GOLDEN, 'txt_output.json')) as f:
        cases = json.load(f)
    for c in cases:
        nbins = c['seq'] // c['bin_size'] if c['bin_size'] else None
        rows, part_rows, counts = [], [0], []
        for prows in c['partitions']:
            prows = [dict(r, masked_lm_positions=base64.b64decode(r['masked_lm_positions']))
                     if 'masked_lm_positions' in r else r for r in prows]
            if nbins:  # the GPU path hands write_txt each partition's rows bin after bin (stable)
                b = np.minimum((np.asarray([r['num_tokens'] for r in prows], np.int64) - 1) //
                               c['bin_size'], nbins - 1)
                prows = [prows[i] for i in np.argsort(b, kind='stable')]
                counts.append(np.bincount(b, minlength=nbins))
            rows += prows
            part_rows.append(len(rows))
        out = tmp_path / c['name']
        out.mkdir()
        n_part = len(c['partitions'])
        P.write_txt(str(out), Rows(rows), np.asarray(part_rows), list(range(n_part)), c['masking'],
                    nbins, np.asarray(counts) if nbins else None, n_part)
        got = {fn: (out / fn).read_text() for fn in sorted(os.listdir(out))}
        assert got == c['files'], c['name']


def _ws_corpus(d, n_files=3, n_lines=300, seed=5):
    import random
    rng = random.Random(seed)
    ws = ['\t', ' ', '\x1c', ' ', '　', ' ', '\x85', ' \r', '\x0b']
    words = ['abc', 'déjà', 'x', '中文', '[CLS]', 'q r', '', '\U0001f600']
    for f in range(n_files):
        lines = []
        for i in range(n_lines):
            parts = [rng.choice(words) for _ in range(rng.randint(0, 6))]
            line = (rng.choice(ws) * rng.randint(0, 2) + 'id{}'.format(i) + rng.choice(ws) +
                    ' '.join(parts) + rng.choice(ws) * rng.randint(0, 2))
            lines.append('' if rng.random() < 0.1 else line)
        with open(os.path.join(d, 'f{}.txt'.format(f)), 'w', encoding='utf-8') as fh:
            fh.write('\n'.join(lines) + '\n')


@pytest.mark.parametrize('ratio,bs', [(1.0, None), (1.0, 2500), (0.7, None), (0.6, 1700)])
def test_native_reader_matches_python(tmp_path, ratio, bs):
    """lddl_read_groups (C++ threads) == the per-line Python path: read_block(as_bytes=True)
    lines (strip with str.isspace at both ends, empty dropped, random_sample), the per-group
    Random(seed).shuffle of pretrain.iter_batches and split_id_text_bytes."""
    import random
    _ws_corpus(str(tmp_path))
    blocks = R.plan_blocks(str(tmp_path), bs, ratio, 99)
    groups = [blocks[i:i + 3] for i in range(0, len(blocks), 3)]
    seeds = [12345 * 1000003 - 1 - 3 * i for i in range(len(groups))] + [-7]
    if len(groups) > 1:
        seeds[1] = -(1 << 40) - 3  # negative and two-limb seeds
    seeds = seeds[:len(groups)]
    text, doc_off, nd = R.read_groups_native(groups, seeds, threads=4)
    exp, nde = [], []
    for g, sd in zip(groups, seeds):
        parts = [R.read_block(b, as_bytes=True) for b in g]
        docs = [x for lines in parts for x in lines]
        random.Random(sd).shuffle(docs)
        k = 0
        for lines in parts:
            nde.append(len(lines))
            exp += [R.split_id_text_bytes(x)[1] for x in docs[k:k + len(lines)]]
            k += len(lines)
    got = [bytes(text[doc_off[i]:doc_off[i + 1]]) for i in range(len(doc_off) - 1)]
    assert got == exp
    assert list(nd) == nde


def test_native_reader_rejects_malformed_utf8(tmp_path):
    """A malformed line raises even when random_sample would drop it (dask decodes whole
    blocks strictly); overlong / surrogate / > U+10FFFF sequences are malformed as in Python."""
    for bad in (b'\xc0\xaf', b'\xed\xa0\x80', b'\xf4\x90\x80\x80', b'\xe2\x82', b'\x80'):
        p = tmp_path / 'x{}'.format(bad.hex())
        p.mkdir()
        with pytest.raises(UnicodeDecodeError):
            bad.decode('utf-8')
        (p / 'a.txt').write_bytes(b'id0 good line\nid1 bad ' + bad + b' here\nid2 ok\n')
        blocks = R.plan_blocks(str(p), None, 0.01, 3)
        with pytest.raises(UnicodeDecodeError):
            R.read_groups_native([blocks], [1])


def test_shard_writers_piece_mode_same_files(tmp_path):
    """ShardWriters with fewer open files allowed than (shard, bin) files: per-batch pieces
    merged at close give the same files, row group for row group, as open writers; empty
    (shard, bin) pairs still get their empty file."""
    from concurrent.futures import ThreadPoolExecutor
    import pyarrow as pa
    import pyarrow.parquet as pq
    from lddl_amd.dask.bert.pretrain import ShardWriters
    out = {}
    for mode, max_open in (('open', None), ('pieces', 2)):
        d = tmp_path / mode
        d.mkdir()
        with ThreadPoolExecutor(4) as pool:
            w = ShardWriters(str(d), 2, True, True, pool, n_local_shards=3, max_open=max_open)
            assert (w.pieces is not None) == (mode == 'pieces')
            w.shards.update([0, 1, 2])
            for t in range(3):  # batches
                for s in range(3):
                    for b in range(2):
                        if (s, b) == (2, 1):
                            continue  # never receives rows
                        n = 1 + (t + s + b) % 3
                        w._write((s, b), pa.table({
                            'A': pa.array(['a{}{}{}{}'.format(t, s, b, i) for i in range(n)]),
                            'num_tokens': pa.array(np.arange(n, dtype=np.uint16))}))
            assert len(w.close()) == 6
        out[mode] = {fn: pq.read_table(d / fn) for fn in os.listdir(d)}
        assert not any(x.startswith('.lddl_amd_pieces') for x in os.listdir(d))
    assert set(out['open']) == set(out['pieces']) and len(out['open']) == 6
    for fn in out['open']:
        assert out['open'][fn].equals(out['pieces'][fn]), fn
        assert pq.ParquetFile(tmp_path / 'open' / fn).num_row_groups == \
            pq.ParquetFile(tmp_path / 'pieces' / fn).num_row_groups
