"""Native counter-RNG pair mode (rng='native', LDDL_RNG_NATIVE): no bit-exact oracle exists (the
reference draws from an unseeded MT19937), so these tests check what the reference
guarantees: every pair is a valid NSP pair of its partition (A and B are windows of the
partition's documents, lengths within target_seq_length - 3), the masked count per pair is
the reference's max(1, round(ratio * num_tokens)) capped by the candidates, positions are sorted
non-special indices, the 80/10/10 decision rates hold within 0.1 percentage point, the pair
statistics agree with the replay mode on the same corpus, and a partition's output does not
depend on batching or on repeated runs."""
import numpy as np
import pytest
import torch

from conftest import VOCAB_UNCASED

pytestmark = pytest.mark.gpu

LEN_MASK = (1 << 30) - 1


def partition_docs(corp, partition_bytes):
    doc_bytes = corp.sent_off[corp.doc_sent_off]
    cuts = np.searchsorted(doc_bytes, np.arange(0, doc_bytes[-1], partition_bytes), 'left')
    cuts = np.unique(np.concatenate([[0], cuts, [corp.n_doc]]))
    return cuts.astype(np.int64)


@pytest.fixture(scope='module')
def ctx():
    from lddl_amd.context import Context
    return Context(VOCAB_UNCASED, True)


def batch(ctx, n_bytes, part_bytes, seed=77, specials_every=0):
    """specials_every > 0: every that many bytes, a run of 5 lowercase letters in the text is
    overwritten with a literal [CLS] or [SEP] (sentence boundaries unchanged)."""
    from lddl_amd import synth
    corp = synth.generate(seed=seed, n_bytes=n_bytes, nonascii_frac=0.01, threads=16)
    if specials_every:
        t = np.array(corp.text, copy=True)
        low = (t >= ord('a')) & (t <= ord('z'))
        for k, at in enumerate(range(0, len(t) - 5, specials_every)):
            while at < len(t) - 5 and not low[at:at + 5].all():
                at += 1
            if at < len(t) - 5:
                t[at:at + 5] = np.frombuffer(b'[CLS]' if k % 2 else b'[SEP]', np.uint8)
        corp.text = t
    part = partition_docs(corp, part_bytes)
    seeds = np.arange(len(part) - 1, dtype=np.int64) * 7919 + 12345
    dev = ctx.device
    text = torch.from_numpy(corp.text).to(dev)
    sent_off = torch.from_numpy(corp.sent_off).to(dev)
    ids, sent_len = ctx.tokenize(text, sent_off)
    return dict(corp=corp, part=part, seeds=seeds, sent_off=sent_off, ids=ids, sent_len=sent_len,
                doc_off=torch.from_numpy(corp.doc_sent_off).to(dev))


def run(ctx, b, rng='native', parts=None, seq=128, masking=True, native_seed=4242):
    from lddl_amd.pairs import make_pairs
    part, seeds = b['part'], b['seeds']
    if parts is not None:
        part, seeds = part[parts[0]:parts[1] + 1], seeds[parts[0]:parts[1]]
    return make_pairs(ctx, b['sent_off'], b['ids'], b['sent_len'], b['doc_off'],
                      torch.from_numpy(part).to(ctx.device), torch.from_numpy(seeds).to(ctx.device),
                      seq=seq, dup=5, masking=masking, rng=rng, native_seed=native_seed).to_host()


def doc_tokens(b):
    """Kept tokens of every document (concatenated sentences) as int32 arrays."""
    ids = b['ids'].cpu().numpy()
    lens = b['sent_len'].cpu().numpy() & LEN_MASK
    so = b['corp'].sent_off
    dso = b['corp'].doc_sent_off
    docs = []
    for d in range(len(dso) - 1):
        parts = [ids[so[s]:so[s] + lens[s]] for s in range(dso[d], dso[d + 1]) if lens[s]]
        docs.append(np.concatenate(parts).astype(np.int32) if parts else np.zeros(0, np.int32))
    return docs


def aligned_find(hay, needle):
    i = hay.find(needle)
    while i >= 0 and i % 4:
        i = hay.find(needle, i + 1)
    return i


@pytest.mark.parametrize('seq', [128, 512])
def test_native_pairs_valid(ctx, seq):
    b = batch(ctx, 3 << 20, 64 << 10)
    out = run(ctx, b, seq=seq)
    cls_id, sep_id, mask_id = (ctx.vocab[t] for t in ('[CLS]', '[SEP]', '[MASK]'))
    docs = doc_tokens(b)
    docs_b = [d.tobytes() for d in docs]
    part, po = b['part'], out['part_off']
    tok_off, len_a, pos_off = out['tok_off'], out['len_a'], out['pos_off']
    assert len(po) == len(part)
    n_checked = 0
    for p in range(len(part) - 1):
        pdocs = [i for i in range(part[p], part[p + 1]) if len(docs[i])]
        for q in range(po[p], min(po[p + 1], po[p] + 40)):
            toks = out['tokens'][tok_off[q]:tok_off[q + 1]].astype(np.int32)
            na = int(len_a[q])
            nb = len(toks) - na
            assert na >= 1 and nb >= 1 and na + nb <= seq - 3
            pos = out['pos'][pos_off[q]:pos_off[q + 1]].astype(np.int64)
            lab = out['labels'][pos_off[q]:pos_off[q + 1]]
            assert np.all(np.diff(pos) > 0)
            assert np.all(((pos >= 1) & (pos <= na)) | ((pos >= na + 2) & (pos <= na + nb + 1)))
            idx = np.where(pos <= na, pos - 1, pos - 2)
            toks[idx] = lab
            nc = int(np.sum((toks != cls_id) & (toks != sep_id)))
            want = min(max(1, int(np.round((na + nb + 3) * 0.15))), nc)
            assert len(pos) == want
            A, B = toks[:na].tobytes(), toks[na:].tobytes()
            da = [d for d in pdocs if aligned_find(docs_b[d], A) >= 0]
            assert da, 'A is not a window of a document of its partition'
            db = [d for d in pdocs if aligned_find(docs_b[d], B) >= 0]
            assert db, 'B is not a window of a document of its partition'
            if not out['is_random_next'][q]:
                assert set(da) & set(db), 'actual-next B must come from the document of A'
            n_checked += 1
    assert n_checked > 500


def test_native_rates_and_stats(ctx):
    b = batch(ctx, 80 << 20, 1 << 20, seed=91)
    nat = run(ctx, b)
    rep = run(ctx, b, rng='replay')
    mask_id = ctx.vocab['[MASK]']
    pos, lab, po, to, la = nat['pos'], nat['labels'], nat['pos_off'], nat['tok_off'], nat['len_a']
    pair_of = np.repeat(np.arange(len(la)), np.diff(po))
    p = pos.astype(np.int64)
    idx = to[pair_of] + np.where(p <= la[pair_of], p - 1, p - 2)
    got = nat['tokens'][idx]
    n = len(got)
    assert n > 8_000_000
    f_mask = np.mean(got == mask_id)
    f_keep = np.mean(got == lab)
    f_rand = 1.0 - f_mask - f_keep
    print('native masks={} [MASK]={:.5f} keep={:.5f} random={:.5f}'.format(n, f_mask, f_keep, f_rand))
    assert abs(f_mask - 0.8) < 1e-3 and abs(f_keep - 0.1) < 1e-3 and abs(f_rand - 0.1) < 1e-3
    rnd = got[(got != mask_id) & (got != lab)]
    assert abs(rnd.mean() / ctx.vocab_size - 0.5) < 0.01  # uniform replacement ids
    # masked fraction per pair follows the reference's rounding rule exactly
    num = np.diff(to) + 3
    want = np.maximum(1, np.round(num * 0.15)).astype(np.int64)
    assert np.mean(np.diff(po) == want) > 0.999  # (only literal [CLS]/[SEP] text lowers it)
    # pair statistics agree with the replay (reference-RNG) mode on the same corpus
    assert abs(len(nat['len_a']) / len(rep['len_a']) - 1) < 0.01
    assert abs(nat['is_random_next'].mean() - rep['is_random_next'].mean()) < 0.01
    assert abs(nat['num_tokens'].mean() / rep['num_tokens'].mean() - 1) < 0.01
    assert abs(np.diff(po).mean() / np.diff(rep['pos_off']).mean() - 1) < 0.01


def test_native_batching_invariant_and_deterministic(ctx):
    b = batch(ctx, 2 << 20, 64 << 10, seed=5)
    full = run(ctx, b)
    again = run(ctx, b)
    for k in ('tokens', 'tok_off', 'len_a', 'is_random_next', 'pos', 'labels', 'pos_off'):
        np.testing.assert_array_equal(full[k], again[k])
    n_part = len(b['part']) - 1
    h = n_part // 2
    tail = run(ctx, b, parts=(h, n_part))
    po = full['part_off']
    q0, q1 = po[h], po[-1]
    np.testing.assert_array_equal(tail['len_a'], full['len_a'][q0:q1])
    np.testing.assert_array_equal(tail['is_random_next'], full['is_random_next'][q0:q1])
    t0 = full['tok_off'][q0]
    np.testing.assert_array_equal(tail['tokens'], full['tokens'][t0:full['tok_off'][q1]])
    m0 = full['pos_off'][q0]
    np.testing.assert_array_equal(tail['pos'], full['pos'][m0:full['pos_off'][q1]])
    np.testing.assert_array_equal(tail['labels'], full['labels'][m0:full['pos_off'][q1]])
    other = run(ctx, b, native_seed=4243)
    assert not np.array_equal(other['tokens'], full['tokens'])


def test_native_masking_stream_is_separate(ctx):
    """Masking draws come from their own stream: without masking the same pairs come out in the
    same order."""
    b = batch(ctx, 1 << 20, 64 << 10, seed=6)
    m = run(ctx, b)
    u = run(ctx, b, masking=False)
    np.testing.assert_array_equal(m['len_a'], u['len_a'])
    np.testing.assert_array_equal(m['tok_off'], u['tok_off'])
    assert u.get('pos') is None


def _oracle_inputs(b):
    """The GPU tokenizer's output as the oracle's per-sentence token runs (tokenization parity is
    tested in test_tokenize_gpu.py)."""
    ids = b['ids'].cpu().numpy()
    lens = (b['sent_len'].cpu().numpy() & LEN_MASK).astype(np.int64)
    so = b['corp'].sent_off
    tok_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    flat = np.concatenate([ids[so[s]:so[s] + lens[s]] for s in range(len(lens))]
                          or [np.zeros(0, np.int32)]).astype(np.int32)
    return tok_off, flat


@pytest.mark.parametrize('seq,masking,lds_words', [(128, True, None), (512, True, None),
                                                   (1024, True, None), (128, False, None),
                                                   (128, True, '64')])
def test_native_bit_exact_vs_oracle(ctx, seq, masking, lds_words, monkeypatch):
    """rng='native' against the C restatement of the same algorithm and streams
    (oracle/native_oracle.c): pair windows, truncation, random-next choice, masked positions and
    decisions and the partition order, bit for bit, partition by partition — with literal
    [CLS] / [SEP] in the text (the candidate walk), at seq 1024 (the gather's one-pair-per-
    half-wave instantiation) and, with LDDL_NATIVE_LDS_WORDS=64, every
    partition through the planner's global-prefix path instead of the LDS tables."""
    from oracle import oracle as O
    if lds_words:
        monkeypatch.setenv('LDDL_NATIVE_LDS_WORDS', lds_words)
    b = batch(ctx, 1_500_000, 200_000, seed=33, specials_every=3000)
    tok_off, flat = _oracle_inputs(b)
    assert ((b['sent_len'].cpu().numpy() & (1 << 30)) != 0).sum() > 50  # literal specials kept
    out = run(ctx, b, seq=seq, masking=masking, native_seed=987654321)
    part, seeds = b['part'], b['seeds']
    po = out['part_off']
    cls_id, sep_id, mask_id = (ctx.vocab[t] for t in ('[CLS]', '[SEP]', '[MASK]'))
    for p in range(len(part) - 1):
        ds = b['corp'].doc_sent_off[part[p]:part[p + 1] + 1]
        exp = O.partition_pairs_native(ds, tok_off, flat, 987654321, int(seeds[p]), 5, seq, masking,
                                       len(ctx), cls_id, sep_id, mask_id)
        q0, q1 = po[p], po[p + 1]
        assert q1 - q0 == len(exp['len_a']), p
        t0, t1 = out['tok_off'][q0], out['tok_off'][q1]
        np.testing.assert_array_equal(out['tokens'][t0:t1], exp['tokens'], err_msg=str(p))
        np.testing.assert_array_equal(np.diff(out['tok_off'][q0:q1 + 1]), np.diff(exp['tok_off']))
        np.testing.assert_array_equal(out['len_a'][q0:q1], exp['len_a'])
        np.testing.assert_array_equal(out['is_random_next'][q0:q1], exp['is_random_next'])
        if masking:
            m0, m1 = out['pos_off'][q0], out['pos_off'][q1]
            np.testing.assert_array_equal(out['pos'][m0:m1], exp['pos'])
            np.testing.assert_array_equal(out['labels'][m0:m1], exp['labels'])
            np.testing.assert_array_equal(np.diff(out['pos_off'][q0:q1 + 1]), np.diff(exp['pos_off']))
