"""GPU collate (_to_encoded_inputs) and dynamic masking (_mask_tokens) vs reference goldens."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, VOCAB_CASED, VOCAB_UNCASED

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g():
    with np.load(os.path.join(GOLDEN, 'collate.npz')) as z:
        return dict(z)


@pytest.fixture(scope='module')
def ctx_c():
    from lddl_amd.context import Context
    return Context(VOCAB_CASED, False)


@pytest.fixture(scope='module')
def ctx_u():
    from lddl_amd.context import Context
    return Context(VOCAB_UNCASED, True)


def _strings(ctx, flat, off):
    return [' '.join(ctx.tokens[i] for i in flat[off[k]:off[k + 1]]) for k in range(len(off) - 1)]


def batch_dyn(g, ctx):
    A = _strings(ctx, g['dyn_a'], g['dyn_a_off'])
    B = _strings(ctx, g['dyn_b'], g['dyn_b_off'])
    return [(a, b, bool(r)) for a, b, r in zip(A, B, g['dyn_is_random_next'])]


def batch_static(g, ctx):
    from io import BytesIO
    A = _strings(ctx, g['static_a'], g['static_a_off'])
    B = _strings(ctx, g['static_b'], g['static_b_off'])
    out = []
    for k in range(len(A)):
        pos = g['static_pos'][g['static_pos_off'][k]:g['static_pos_off'][k + 1]].astype(np.uint16)
        bio = BytesIO()
        np.save(bio, pos)
        lab = ' '.join(ctx.tokens[i] for i in g['static_lab'][g['static_lab_off'][k]:
                                                              g['static_lab_off'][k + 1]])
        out.append((A[k], B[k], bool(g['static_is_random_next'][k]), bio.getvalue(), lab))
    return out


@pytest.mark.parametrize('align', [8, 1, 64])
def test_encode_dynamic(g, ctx_c, align):
    from lddl_amd.torch.bert import _to_encoded_inputs
    enc = _to_encoded_inputs(batch_dyn(g, ctx_c), ctx_c, sequence_length_alignment=align)
    for k in ('input_ids', 'token_type_ids', 'attention_mask', 'special_tokens_mask',
              'next_sentence_labels'):
        np.testing.assert_array_equal(enc[k].cpu().numpy(), g['dyn{}_{}'.format(align, k)], err_msg=k)


def test_encode_static(g, ctx_u):
    from lddl_amd.torch.bert import _to_encoded_inputs
    enc = _to_encoded_inputs(batch_static(g, ctx_u), ctx_u)
    for k in ('input_ids', 'token_type_ids', 'attention_mask', 'labels', 'next_sentence_labels'):
        np.testing.assert_array_equal(enc[k].cpu().numpy(), g['static_' + k], err_msg=k)


@pytest.mark.parametrize('seed', [0, 1234])
def test_mask_replay_bit_exact(g, ctx_c, seed):
    from lddl_amd.torch.bert import _mask_tokens
    ids = torch.from_numpy(g['dyn8_input_ids']).cuda()
    stm = torch.from_numpy(g['dyn8_special_tokens_mask']).cuda()
    rep = {k: torch.from_numpy(g['mask{}_{}'.format(seed, k)]) for k in
           ('masked', 'replaced', 'random', 'words')}
    out, labels = _mask_tokens(ids.clone(), stm, ctx_c, 0.15, -1, replay=rep)
    np.testing.assert_array_equal(out.cpu().numpy(), g['mask{}_input_ids'.format(seed)])
    np.testing.assert_array_equal(labels.cpu().numpy(), g['mask{}_labels'.format(seed)])


def test_mask_native_rates(ctx_c):
    """north_star: 15% / 80-10-10 each within 0.1% (absolute) under the native counter RNG.
    >= 2e7 masked slots, so 1e-3 is > 10 sigma for every rate. Input ids are out-of-vocab
    sentinels (>= len(tokenizer)), so a random replacement (drawn from [0, len)) can never equal
    the original: keep / random / [MASK] are told apart exactly (a random draw of the [MASK] id
    itself, probability 0.1 / V = 3.4e-6, is the only confusion left)."""
    from lddl_amd.torch.bert import _mask_tokens
    V = len(ctx_c)
    mid = ctx_c.special_ids['[MASK]']
    B, L = 8192, 2048
    g = torch.Generator(device='cuda').manual_seed(3)
    ids = torch.randint(V + 10, V + 5000, (B, L), device='cuda', generator=g)
    stm = torch.zeros(B, L, dtype=torch.long, device='cuda')
    stm[:, 0] = 1
    stm[:, 1800:] = 1
    n_ok = int((stm == 0).sum())
    tot = dict(masked=0, repl=0, rand=0, keep=0)
    calls = 0
    while tot['masked'] < 2e7:
        out, lab = _mask_tokens(ids.clone(), stm, ctx_c, 0.15, -1, seed=99, counter=calls)
        m = lab != -1
        assert not bool((m & (stm == 1)).any())
        assert bool((lab[m] == ids[m]).all())
        tot['masked'] += int(m.sum())
        tot['repl'] += int((m & (out == mid)).sum())
        tot['keep'] += int((m & (out == ids)).sum())
        tot['rand'] += int((m & (out < V) & (out != mid)).sum())
        assert bool(((out == ids) | m).all())  # unmasked slots untouched
        calls += 1
    n = calls * n_ok
    assert tot['repl'] + tot['keep'] + tot['rand'] == tot['masked']
    assert abs(tot['masked'] / n - 0.15) < 1e-3
    assert abs(tot['repl'] / tot['masked'] - 0.8) < 1e-3
    assert abs(tot['rand'] / tot['masked'] - 0.1) < 1e-3
    assert abs(tot['keep'] / tot['masked'] - 0.1) < 1e-3


def test_mask_special_tokens_mask_none(ctx_c):
    """special_tokens_mask=None: special slots are the ids of all_special_ids (the reference's
    get_special_tokens_mask(ids, already_has_special_tokens=True), bert.py:167-172)."""
    from lddl_amd.torch.bert import _mask_tokens
    V = len(ctx_c)
    sp = ctx_c.all_special_ids
    ids = torch.randint(0, V, (64, 256), device='cuda')
    ids[:, ::7] = sp[0]
    ids[:, 3::11] = sp[3]
    ids[:, 0] = ctx_c.special_ids['[CLS]']
    exp = torch.tensor([ctx_c.get_special_tokens_mask(r, already_has_special_tokens=True)
                        for r in ids.cpu().tolist()], device='cuda')
    a = _mask_tokens(ids.clone(), None, ctx_c, seed=7, counter=1)
    b = _mask_tokens(ids.clone(), exp, ctx_c, seed=7, counter=1)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert not bool(((a[1] != -1) & (exp == 1)).any())


def test_tokenizer_duck_type(ctx_u):
    """tokenize(s, max_length, truncation), mask_token, convert_tokens_to_ids(str),
    get_special_tokens_mask against the oracle tokenizer."""
    from oracle import oracle as O
    tok = O.Tokenizer(VOCAB_UNCASED, lowercase=True)
    s = 'Hello, World! Tokenization of naïve café-style text [MASK] works.'
    b = np.frombuffer(s.encode(), np.uint8)
    ids, off = tok.tokenize(b, np.asarray([0, len(b)], np.int64))
    exp = [ctx_u.tokens[i] for i in ids[off[0]:off[1]]]
    assert ctx_u.tokenize(s) == exp
    assert ctx_u.tokenize(s, max_length=5, truncation=True) == exp[:5]
    w = next(t for t in ctx_u.tokens[1000:] if t.isalpha() and t.islower() and len(t) > 2)
    long_s = ' '.join([w] * 700)
    assert len(ctx_u.tokenize(long_s, max_length=512, truncation=True)) == 512
    assert len(ctx_u.tokenize(long_s)) == 700
    assert ctx_u.tokenize('') == []
    assert ctx_u.convert_tokens_to_ids(ctx_u.mask_token) == ctx_u.special_ids['[MASK]']
    assert ctx_u.convert_tokens_to_ids(['[CLS]', 'zzzznotaword']) == [
        ctx_u.special_ids['[CLS]'], ctx_u.special_ids['[UNK]']]
    assert ctx_u.get_special_tokens_mask([5, 6], [7]) == [1, 0, 0, 1, 0, 1]
    cls = ctx_u.special_ids['[CLS]']
    assert ctx_u.get_special_tokens_mask([cls, 999, 5], already_has_special_tokens=True) == [
        1, 0, 0]


def test_encode_rejects_position_beyond_length(g, ctx_u):
    from lddl_amd.torch.bert import _to_encoded_inputs
    batch = batch_static(g, ctx_u)[:2]
    bad = list(batch[0])
    from io import BytesIO
    bio = BytesIO()
    np.save(bio, np.asarray([1, 600], np.uint16))
    bad[3] = bio.getvalue()
    bad[4] = 'a b'
    with pytest.raises(IndexError):
        _to_encoded_inputs([tuple(bad), batch[1]], ctx_u)


def test_encode_unicode_whitespace_split(ctx_u):
    """Python's str.split() whitespace (\x1c-\x1f, U+00A0, U+3000 ...) separates tokens exactly
    as in the reference's _to_encoded_inputs."""
    from lddl_amd.torch.bert import _to_encoded_inputs
    a = 'the\x1cquick\u00a0brown fox'
    b = 'jumps\u3000over  the\tlazy'
    enc = _to_encoded_inputs([(a, b, False)], ctx_u)
    want = ([ctx_u.special_ids['[CLS]']] + ctx_u.convert_tokens_to_ids(a.split()) +
            [ctx_u.special_ids['[SEP]']] + ctx_u.convert_tokens_to_ids(b.split()) +
            [ctx_u.special_ids['[SEP]']])
    got = enc['input_ids'][0].cpu().tolist()
    assert got[:len(want)] == want and all(x == 0 for x in got[len(want):])


def test_mask_native_deterministic(ctx_c):
    from lddl_amd.torch.bert import _mask_tokens
    ids = torch.randint(5, len(ctx_c), (8, 64), device='cuda')
    stm = torch.zeros_like(ids)
    a = _mask_tokens(ids.clone(), stm, ctx_c, seed=5, counter=3)
    b = _mask_tokens(ids.clone(), stm, ctx_c, seed=5, counter=3)
    c = _mask_tokens(ids.clone(), stm, ctx_c, seed=5, counter=4)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert not torch.equal(a[1], c[1])


@pytest.mark.parametrize('align', [8, 1])
def test_fused_collate_mask_equals_two_pass(g, ctx_c, align):
    """lddl_collate_encode_masked == lddl_collate_encode + lddl_mask_dynamic (same Philox
    stream), i.e. the loader's one-kernel collate is the reference's _to_encoded_inputs followed
    by _mask_tokens."""
    from lddl_amd.torch.bert import PackedBatch, encode_packed, _mask_tokens
    pk = PackedBatch(batch_dyn(g, ctx_c))
    two = encode_packed(pk, ctx_c, align)
    ids, lab = _mask_tokens(two['input_ids'], two.pop('special_tokens_mask'), ctx_c, 0.15, -1,
                            seed=1234567, counter=(3 << 32) + 5)
    one = encode_packed(pk, ctx_c, align, mask=(0.15, 1234567, (3 << 32) + 5))
    assert set(one) == {'input_ids', 'token_type_ids', 'attention_mask', 'labels',
                        'next_sentence_labels'}
    assert torch.equal(one['input_ids'], ids) and torch.equal(one['labels'], lab)
    for k in ('token_type_ids', 'attention_mask', 'next_sentence_labels'):
        assert torch.equal(one[k], two[k])
    assert int((lab != -1).sum()) > 0


@pytest.mark.gpu
def test_host_stager_round_trip_and_reuse():
    """HostStager: one H2D copy per batch through a reused pinned ring; every dtype and shape
    (empty arrays included) arrives intact, and no pinned memory is allocated once the ring's
    slots have grown."""
    import torch
    from lddl_amd.torch.bert import HostStager
    st = HostStager(depth=3)
    rng = np.random.default_rng(5)
    dev = torch.device('cuda', 0)
    for it in range(40):
        n = 1000 + (it % 7) * 300
        arrs = [rng.integers(0, 255, n * 3, dtype=np.uint8), rng.integers(-2**40, 2**40, n + 1),
                rng.integers(-2**30, 2**30, 2 * n, dtype=np.int32), np.zeros(0, np.uint8),
                rng.integers(0, 2**15, 17, dtype=np.int16)]
        got = st.stage(arrs, dev)
        for a, g in zip(arrs, got):
            assert g.is_cuda and g.numel() == a.size
            np.testing.assert_array_equal(g.cpu().numpy().view(a.dtype), a)
    assert st.allocations <= 3 * 2
