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
    """15% / 80-10-10 within 0.1% (absolute) under the native counter RNG."""
    from lddl_amd.torch.bert import _mask_tokens
    B, L = 256, 512
    ids = torch.randint(5, len(ctx_c), (B, L), device='cuda')
    stm = torch.zeros(B, L, dtype=torch.long, device='cuda')
    stm[:, 0] = 1
    stm[:, 300:] = 1
    n_ok = int((stm == 0).sum())
    tot_masked = tot_repl = tot_rand = tot_keep = 0
    for counter in range(40):
        x = ids.clone()
        out, lab = _mask_tokens(x, stm, ctx_c, 0.15, -1, seed=99, counter=counter)
        m = lab != -1
        assert not bool((m & (stm == 1)).any())
        tot_masked += int(m.sum())
        tot_repl += int((m & (out == ctx_c.special_ids['[MASK]'])).sum())
        same = m & (out == ids)
        tot_keep += int(same.sum())
        tot_rand += int((m & (out != ids) & (out != ctx_c.special_ids['[MASK]'])).sum())
    n = 40 * n_ok
    assert abs(tot_masked / n - 0.15) < 0.001
    assert abs(tot_repl / tot_masked - 0.8) < 0.001 * 10  # 80% of the masked
    # random words equal to the original (1/V) are counted as keeps; both ~10%
    assert abs((tot_rand + tot_keep) / tot_masked - 0.2) < 0.01


def test_mask_native_deterministic(ctx_c):
    from lddl_amd.torch.bert import _mask_tokens
    ids = torch.randint(5, len(ctx_c), (8, 64), device='cuda')
    stm = torch.zeros_like(ids)
    a = _mask_tokens(ids.clone(), stm, ctx_c, seed=5, counter=3)
    b = _mask_tokens(ids.clone(), stm, ctx_c, seed=5, counter=3)
    c = _mask_tokens(ids.clone(), stm, ctx_c, seed=5, counter=4)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert not torch.equal(a[1], c[1])
