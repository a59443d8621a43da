"""GPU pair construction + static masking (replay RNG) vs the reference goldens, starting from
the raw Punkt sentences: tokenize -> drop empty sentences/docs -> plan -> gather."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, VOCAB_UNCASED

pytestmark = pytest.mark.gpu

PAIR_CASES = ['s128_mask', 's128_nomask', 's512_mask', 's512_nomask_short', 's64_mask_ratio']


def load(name):
    with np.load(os.path.join(GOLDEN, name)) as z:
        return dict(z)


@pytest.fixture(scope='module')
def ctx():
    from lddl_amd.context import Context
    return Context(VOCAB_UNCASED, True)


@pytest.fixture(scope='module')
def docs_dev(ctx):
    g = load('documents_uncased.npz')
    text = torch.from_numpy(g['text'].copy()).cuda()
    sent_off = torch.from_numpy(g['sent_off']).cuda()
    ids, sent_len = ctx.tokenize(text, sent_off)
    line_off = g['line_sent_off']
    # original line index of every kept document (a line whose sentences all normalise away is
    # dropped by the reference before partitioning)
    lens = (sent_len.cpu().numpy() & ((1 << 30) - 1))
    kept_lines = [i for i in range(len(line_off) - 1) if lens[line_off[i]:line_off[i + 1]].sum() > 0]
    return dict(sent_off=sent_off, ids=ids, sent_len=sent_len,
                doc_sent_off=torch.from_numpy(line_off).cuda(), kept_lines=kept_lines,
                n_lines=len(line_off) - 1)


def part_doc_off_for(sizes, kept_lines, n_lines):
    bounds = np.concatenate([[0], np.cumsum(sizes)])
    return np.asarray([kept_lines[b] if b < len(kept_lines) else n_lines for b in bounds], np.int64)


@pytest.mark.parametrize('name', PAIR_CASES)
def test_pairs_golden_gpu(name, ctx, docs_dev):
    from lddl_amd.pairs import make_pairs
    g = load('pairs_{}.npz'.format(name))
    dup, seq, masking = g['params'].tolist()
    pdo = part_doc_off_for(g['part_doc_sizes'], docs_dev['kept_lines'], docs_dev['n_lines'])
    if pdo[-1] < docs_dev['n_lines']:  # docs after the last golden partition are not used
        pass
    out = make_pairs(ctx, docs_dev['sent_off'], docs_dev['ids'], docs_dev['sent_len'],
                     docs_dev['doc_sent_off'], torch.from_numpy(pdo).cuda(),
                     torch.from_numpy(g['seeds'].astype(np.int64)).cuda(), seq=seq, dup=dup,
                     masking=bool(masking), short_seq_prob=float(g['short_seq_prob']),
                     masked_lm_ratio=float(g['ratio'])).to_host()
    n = len(g['num_tokens'])
    assert len(out['len_a']) == n
    np.testing.assert_array_equal(out['is_random_next'], g['is_random_next'])
    np.testing.assert_array_equal(out['num_tokens'], g['num_tokens'])
    np.testing.assert_array_equal(np.diff(g['a_off']), out['len_a'])
    exp_tok = np.concatenate([np.concatenate([g['a'][g['a_off'][q]:g['a_off'][q + 1]],
                                              g['b'][g['b_off'][q]:g['b_off'][q + 1]]])
                              for q in range(n)])
    np.testing.assert_array_equal(out['tokens'], exp_tok)
    if masking:
        np.testing.assert_array_equal(out['pos_off'], g['pos_off'])
        np.testing.assert_array_equal(out['pos'], g['pos'])
        np.testing.assert_array_equal(out['labels'], g['labels'])


def test_mask_pool_overflow_replans(ctx, docs_dev, monkeypatch):
    """A mask pool that is too small makes the planner re-plan with the exact size: same output."""
    name = 's128_mask'
    monkeypatch.setenv('LDDL_AMD_MASK_POOL', '100')
    test_pairs_golden_gpu(name, ctx, docs_dev)


@pytest.mark.parametrize('env', [{'LDDL_FY_MODE': '0'}, {'LDDL_FY_MODE': '1'},
                                 {'LDDL_FY_LW': '32'}, {'LDDL_FY_RA': '0'}, {'LDDL_FY_RA': '2'},
                                 {'LDDL_FY_RA': '3'}, {'LDDL_FY_PF': '2'}, {'LDDL_FY_PF': '8'}])
def test_fy_resolve_variants_golden(ctx, docs_dev, monkeypatch, env):
    """Every mask-replay variant against the reference goldens: the guarded and the branch-free
    steps at every sequence length (the defaults use one kind per length), and 32 pairs per wave
    at seq 512, 0 / 2 / 3 entries read ahead in its move-only groups (default 1; the
    branch-free steps rely on the planner's padded draw regions) and 2 / 8 draw vectors in flight
    (default 4)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for name in ('s128_mask', 's512_mask', 's64_mask_ratio'):
        test_pairs_golden_gpu(name, ctx, docs_dev)


@pytest.mark.parametrize('env', [{'LDDL_FY_RA': '5'}, {'LDDL_FY_PF': '3'}, {'LDDL_FY_LW': '8'},
                                 {'LDDL_FY_PF': '8', 'LDDL_FY_RA': '2'},
                                 {'LDDL_FY_MODE': '0', 'LDDL_FY_RA': '2'}])
def test_fy_resolve_rejects_unsupported_knobs(docs_dev, monkeypatch, env):
    """Unsupported LDDL_FY_* values and combinations raise instead of falling through to another
    variant. A fresh Context: the failed call is not allowed to touch the shared one."""
    from lddl_amd.context import Context
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    with pytest.raises(Exception, match='LDDL_FY'):
        test_pairs_golden_gpu('s512_mask', Context(VOCAB_UNCASED, True), docs_dev)


def test_partition_shuffle_global_path(ctx, docs_dev, monkeypatch):
    """The partition shuffle's path for partitions beyond the LDS budget (swaps in global
    memory, inverse permutation by cycles) gives the reference's pair order."""
    monkeypatch.setenv('LDDL_SHUFFLE_GLOBAL', '1')
    for name in ('s128_mask', PAIR_CASES[0]):
        test_pairs_golden_gpu(name, ctx, docs_dev)


def test_pairs_large_partition_vs_oracle(ctx):
    """A partition with more documents than the planner's LDS document table (> 511): the
    planner instantiation that reads document offsets from global memory, next to a small
    partition, checked token for token against the oracle (seq 128, static masking)."""
    from lddl_amd import synth
    from lddl_amd.pairs import make_pairs
    from oracle import oracle as O
    vocab = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         'lddl_amd', 'assets', 'vocab_synth_uncased_30522.txt')
    corp = synth.generate(seed=77, n_bytes=3_500_000, nonascii_frac=0.02, threads=4)
    n_doc = corp.n_doc
    assert n_doc > 600, n_doc
    part = np.asarray([0, n_doc - 40, n_doc], np.int64)  # 40 documents, then the rest
    seeds = np.asarray([5, 6], np.int64)
    so = torch.from_numpy(corp.sent_off).cuda()
    ids, sl = ctx.tokenize(torch.from_numpy(corp.text).cuda(), so)
    pb = make_pairs(ctx, so, ids, sl, torch.from_numpy(corp.doc_sent_off).cuda(),
                    torch.from_numpy(part).cuda(), torch.from_numpy(seeds).cuda(), seq=128, dup=2,
                    masking=True).to_host()
    tok = O.Tokenizer(vocab)
    e_ids, e_off = tok.tokenize(corp.text, corp.sent_off)
    exp = {'tokens': [], 'num_tokens': [], 'len_a': [], 'pos': [], 'labels': []}
    for p in range(2):
        ds = corp.doc_sent_off[part[p]:part[p + 1] + 1]
        out = O.partition_pairs(ds, e_off, e_ids, int(seeds[p]), 2, 128, True, tok.vocab_size,
                                *(tok.token_id(t) for t in ('[CLS]', '[SEP]', '[MASK]')))
        for k in exp:
            exp[k].append(out[k])
    for k in exp:
        assert np.array_equal(pb[k], np.concatenate(exp[k])), k


@pytest.mark.parametrize('seq,extra', [(128, 40000), (512, 40000), (256, 0), (200, 0)])
def test_pairs_wide_vs_oracle(tmp_path, seq, extra):
    """Against the oracle: a vocab of more than 65,536 entries (4-byte token ids and labels in
    the pair tables and the gather, random-token mask decisions above 65,535; the extra vocab
    lines are bracketed, so no word of the text can produce them and the tokenization is
    unchanged), and seq 200 / 256 with the BERT-sized vocab (the 1-byte-draw mask replay at 16
    pairs per wave, which the reference goldens at 64 / 128 / 512 do not reach). (The gather's
    seq > 600 instantiation runs in test_native_gpu.py: the replay planner stops at seq 512.)"""
    from lddl_amd import synth
    from lddl_amd.context import Context
    from lddl_amd.pairs import make_pairs
    from oracle import oracle as O
    vocab = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         'lddl_amd', 'assets', 'vocab_synth_uncased_30522.txt')
    if extra:
        big = tmp_path / 'vocab_big.txt'
        with open(vocab) as f:
            lines = f.read().splitlines()
        big.write_text('\n'.join(lines + ['[extra{}]'.format(i) for i in range(extra)]) + '\n')
        vocab = str(big)
    ctx = Context(vocab)
    assert ctx.id_bytes == (4 if extra else 2)
    corp = synth.generate(seed=91 + seq, n_bytes=600_000, threads=4)
    part = np.linspace(0, corp.n_doc, 4).astype(np.int64)
    seeds = np.asarray([11, 12, 13], np.int64)
    so = torch.from_numpy(corp.sent_off).cuda()
    ids, sl = ctx.tokenize(torch.from_numpy(corp.text).cuda(), so)
    pb = make_pairs(ctx, so, ids, sl, torch.from_numpy(corp.doc_sent_off).cuda(),
                    torch.from_numpy(part).cuda(), torch.from_numpy(seeds).cuda(), seq=seq, dup=2,
                    masking=True).to_host()
    tok = O.Tokenizer(vocab)
    assert tok.vocab_size == 30522 + extra
    e_ids, e_off = tok.tokenize(corp.text, corp.sent_off)
    exp = {'tokens': [], 'num_tokens': [], 'len_a': [], 'pos': [], 'labels': []}
    for p in range(3):
        ds = corp.doc_sent_off[part[p]:part[p + 1] + 1]
        out = O.partition_pairs(ds, e_off, e_ids, int(seeds[p]), 2, seq, True, tok.vocab_size,
                                *(tok.token_id(t) for t in ('[CLS]', '[SEP]', '[MASK]')))
        for k in exp:
            exp[k].append(out[k])
    for k in exp:
        assert np.array_equal(np.asarray(pb[k]).astype(np.int64),
                              np.concatenate(exp[k]).astype(np.int64)), k
    if extra:
        assert np.concatenate(exp['tokens']).max() > 65535  # random-token decisions reach them


def test_pairs_empty_and_dropped_inputs(ctx):
    """Edge inputs of the compaction and layout: no partitions; partitions whose documents hold
    only sentences that tokenize to nothing (dropped, pretrain.py:89-97); and such documents
    between real ones (kept-sentence and token offsets across the gaps), the last against the
    oracle."""
    from lddl_amd.pairs import make_pairs
    from oracle import oracle as O
    vocab = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         'lddl_amd', 'assets', 'vocab_synth_uncased_30522.txt')
    real = ['the quick brown fox jumps over the lazy dog .', 'a second sentence of the document .',
            'and one more line here .', 'short .', 'the end of the first real document .']
    other = ['another document begins here with words .', 'it also has a second sentence .',
             'and a third sentence to pair .', 'final words .']
    docs = [['   ', ' '], real, ['  ', '   ', ''], other, ['  ']]
    sents = [s for d in docs for s in d]
    text = ''.join(sents).encode()
    sent_off = np.concatenate([[0], np.cumsum([len(s.encode()) for s in sents])]).astype(np.int64)
    doc_sent_off = np.concatenate([[0], np.cumsum([len(d) for d in docs])]).astype(np.int64)
    so = torch.from_numpy(sent_off).cuda()
    ids, sl = ctx.tokenize(torch.from_numpy(np.frombuffer(text, np.uint8).copy()).cuda(), so)
    dso = torch.from_numpy(doc_sent_off).cuda()

    def run(part, seeds):
        return make_pairs(ctx, so, ids, sl, dso, torch.from_numpy(np.asarray(part, np.int64)).cuda(),
                          torch.from_numpy(np.asarray(seeds, np.int64)).cuda(), seq=64, dup=3,
                          masking=True).to_host()

    out = run([0], [])  # no partitions
    assert len(out['len_a']) == 0 and len(out['tokens']) == 0
    out = run([0, 1], [7])  # one partition of dropped sentences only
    assert len(out['len_a']) == 0 and len(out['tokens']) == 0
    out = run([0, 5], [7])  # dropped documents around real ones
    tok = O.Tokenizer(vocab)
    e_ids, e_off = tok.tokenize(np.frombuffer(text, np.uint8), sent_off)
    # the reference drops empty sentences and then empty documents before pairing
    lens = np.diff(e_off)
    kept_docs = [[s for s in range(doc_sent_off[d], doc_sent_off[d + 1]) if lens[s] > 0]
                 for d in range(len(docs))]
    kept_docs = [d for d in kept_docs if d]
    ks = [s for d in kept_docs for s in d]
    k_off = np.concatenate([[0], np.cumsum([lens[s] for s in ks])]).astype(np.int64)
    k_ids = np.concatenate([e_ids[e_off[s]:e_off[s + 1]] for s in ks]).astype(np.int32)
    k_doc = np.concatenate([[0], np.cumsum([len(d) for d in kept_docs])]).astype(np.int64)
    exp = O.partition_pairs(k_doc, k_off, k_ids, 7, 3, 64, True, tok.vocab_size,
                            *(tok.token_id(t) for t in ('[CLS]', '[SEP]', '[MASK]')))
    assert len(exp['len_a']) > 0
    for k in ('tokens', 'num_tokens', 'len_a', 'pos', 'labels'):
        assert np.array_equal(np.asarray(out[k]).astype(np.int64), np.asarray(exp[k]).astype(np.int64)), k


@pytest.mark.parametrize('seq,ratio,env', [(20, 0.9, {}), (20, 0.9, {'LDDL_FY_MODE': '1'}),
                                           (131, 0.7, {}), (200, 0.02, {}),
                                           (300, 0.9, {}), (300, 0.9, {'LDDL_FY_RA': '3'}),
                                           (512, 0.5, {'LDDL_FY_LW': '32'})])
def test_mask_replay_extremes_vs_oracle(monkeypatch, seq, ratio, env):
    """The mask replay (`fy_resolve`) against the oracle where its step kinds meet their edges:
    seq 20 (a handful of candidates, most of each 16-entry draw region padding), masked_lm_ratio
    0.9 (nearly every group finalises slots) and 0.02 (one mask per pair: move-only groups
    throughout), seq 131 (the last register-draw length), 200 / 300 / 512 (1- and 2-byte draws,
    16 and 32 pairs per wave, read-ahead 1 and 3)."""
    from lddl_amd import synth
    from lddl_amd.context import Context
    from lddl_amd.pairs import make_pairs
    from oracle import oracle as O
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    vocab = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                         'lddl_amd', 'assets', 'vocab_synth_uncased_30522.txt')
    ctx = Context(vocab)
    corp = synth.generate(seed=700 + seq, n_bytes=300_000, threads=4)
    part = np.linspace(0, corp.n_doc, 3).astype(np.int64)
    seeds = np.asarray([21, 22], np.int64)
    so = torch.from_numpy(corp.sent_off).cuda()
    ids, sl = ctx.tokenize(torch.from_numpy(corp.text).cuda(), so)
    pb = make_pairs(ctx, so, ids, sl, torch.from_numpy(corp.doc_sent_off).cuda(),
                    torch.from_numpy(part).cuda(), torch.from_numpy(seeds).cuda(), seq=seq, dup=2,
                    masking=True, masked_lm_ratio=ratio).to_host()
    tok = O.Tokenizer(vocab)
    e_ids, e_off = tok.tokenize(corp.text, corp.sent_off)
    exp = {'tokens': [], 'num_tokens': [], 'len_a': [], 'pos': [], 'labels': []}
    for p in range(2):
        ds = corp.doc_sent_off[part[p]:part[p + 1] + 1]
        out = O.partition_pairs(ds, e_off, e_ids, int(seeds[p]), 2, seq, True, tok.vocab_size,
                                *(tok.token_id(t) for t in ('[CLS]', '[SEP]', '[MASK]')),
                                masked_lm_ratio=ratio)
        for k in exp:
            exp[k].append(out[k])
    assert len(pb['num_tokens']) > 0
    for k in exp:
        assert np.array_equal(np.asarray(pb[k]).astype(np.int64),
                              np.concatenate(exp[k]).astype(np.int64)), k
