"""bench.py cpu_baseline worker: the oracle (CPU restatement of the reference) over one run of
partitions, in a spawned process that imports only numpy and the oracle.

TEST INFRASTRUCTURE ONLY (the CPU baseline leg of bench.py)."""
import time

import numpy as np

_CPU_TOK = None


def cpu_worker(job):
    """One CPU process of the baseline: tokenize + pairs + static masking of its partitions with
    the oracle (C restatement of the reference, one thread). job = (text bytes, sentence offsets,
    document sentence offsets, partition document offsets, seeds, seq), all rebased to 0."""
    text, sent_off, doc_sent, part, seeds, seq, vocab = job
    from oracle import oracle as O
    global _CPU_TOK
    if _CPU_TOK is None:  # vocab loaded once per worker process, before the timed map
        _CPU_TOK = O.Tokenizer(vocab, lowercase=True)
    tok = _CPU_TOK
    cls_id, sep_id, mask_id = (tok.token_id(t) for t in ('[CLS]', '[SEP]', '[MASK]'))
    t0 = time.perf_counter()
    ids, off = tok.tokenize(text, sent_off)
    lens = np.diff(off)
    keep = lens > 0  # drop empty sentences, then empty documents (pretrain.py:89-97)
    k_off = np.concatenate([[0], np.cumsum(lens[keep])])  # ids is already compact
    kept_pos = np.concatenate([[0], np.cumsum(keep)])
    n_out = 0
    for p in range(len(part) - 1):
        kd = kept_pos[doc_sent[part[p]:part[p + 1] + 1]]
        kd = np.concatenate([kd[:1], kd[1:][np.diff(kd) > 0]])
        out = O.partition_pairs(kd, k_off, ids, int(seeds[p]), 5, seq, True,
                                tok.vocab_size, cls_id, sep_id, mask_id)
        n_out += int(out['num_tokens'].sum())
    return n_out, time.perf_counter() - t0
