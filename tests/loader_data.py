"""Deterministic small datasets in the balanced-shard layout, shared by the loader tests and the
golden generator (tests/golden/make_loader_golden.py)."""
import io
import json
import os
import random

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq


def _npy(a):
    b = io.BytesIO()
    np.save(b, np.asarray(a, np.uint16))
    return b.getvalue()


def make_loader_dataset(root, vocab_file, binned=True, n_shards=4, static=True, seed=3):
    """Balanced shards: per bin, shard k holds base or base+1 samples. A/B are space-joined
    vocab tokens; with static masking, positions/labels follow the reference's columns."""
    with open(vocab_file, encoding='utf-8') as f:
        vocab = [l.rstrip('\n') for l in f]
    words = [w for w in vocab[1000:6000] if not w.startswith('[')]
    rng = random.Random(seed)
    os.makedirs(root, exist_ok=True)
    bins = [(0, 13), (1, 10)] if binned else [(None, 17)]
    counts = {}
    for b, base in bins:
        for k in range(n_shards):
            n = base + (1 if k < 2 else 0)
            rows = {'A': [], 'B': [], 'is_random_next': [], 'num_tokens': []}
            if static:
                rows['masked_lm_positions'] = []
                rows['masked_lm_labels'] = []
            for r in range(n):
                la = rng.randint(1, 12 if b != 1 else 40)
                lb = rng.randint(1, 12 if b != 1 else 40)
                A = [rng.choice(words) for _ in range(la)]
                B = [rng.choice(words) for _ in range(lb)]
                rows['A'].append(' '.join(A))
                rows['B'].append(' '.join(B))
                rows['is_random_next'].append(rng.random() < 0.5)
                rows['num_tokens'].append(la + lb + 3)
                if static:
                    cand = [i for i in range(1, la + lb + 3) if i != la + 1 and i != la + lb + 2]
                    pos = sorted(rng.sample(cand, max(1, (la + lb) // 7)))
                    seq = ['[CLS]'] + A + ['[SEP]'] + B + ['[SEP]']
                    rows['masked_lm_positions'].append(_npy(pos))
                    rows['masked_lm_labels'].append(' '.join(seq[p] for p in pos))
            name = 'shard-{}.parquet'.format(k) + ('' if b is None else '_{}'.format(b))
            fields = [('A', pa.string()), ('B', pa.string()), ('is_random_next', pa.bool_()),
                      ('num_tokens', pa.uint16())]
            if static:
                fields += [('masked_lm_positions', pa.binary()), ('masked_lm_labels', pa.string())]
            pq.write_table(pa.table({k2: rows[k2] for k2, _ in fields},
                                    schema=pa.schema(fields)), os.path.join(root, name))
            counts[name] = n
    with open(os.path.join(root, '.num_samples.json'), 'w') as f:
        json.dump(counts, f)
    return counts
