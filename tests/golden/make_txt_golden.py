"""Golden fixture for the debug txt output (tests/golden/txt_output.json), made by the REFERENCE's
own writer in the dev container (/root/reference does not exist on the GPU box):

  `_save_txt` (lddl/dask/bert/pretrain.py:501-531) -> dask.bag.to_textfiles (unbinned) or
  `to_textfiles_binned` (lddl/dask/bert/binning.py:439-509, bin parsed from the line's last field)

over reference-generated pair dicts (`create_pairs_from_document` on the uncased golden documents,
seeded per partition as in make_goldens.py), for three configurations. Recorded per case: the
input rows of each dask partition and the exact bytes of every file the reference wrote.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_txt_golden.py

Import recipe: make_goldens.import_reference. Only data is written.
"""
import base64
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_goldens as G  # noqa: E402


def main():
    ref = G.import_reference()
    import dask
    import dask.bag as db
    tok = G.Tok416(G.VOCAB_UNCASED, lower=True)
    lines = G.make_doc_lines(60_000, 777, 0.03)
    docs = ref.pretrain._get_documents(G.ListBag(lines), tok).items  # pretrain.py:77-97
    vocab_words = G.id_ordered_vocab(tok.vocab)
    cases = []
    for name, masking, bin_size, seq in (('mask', True, None, 128), ('mask_binned', True, 32, 128),
                                         ('nomask_binned', False, 64, 256)):
        parts = []
        for p, (a, z) in enumerate(((0, 6), (6, 9), (9, 9))):  # the last partition is empty
            parts.append(G.partition_pairs(ref, docs[a:z], 300 + p, 2, seq, 0.1, masking, 0.15,
                                           vocab_words) if z > a else [])
        bag = db.Bag({('pairs', i): rows for i, rows in enumerate(parts)}, 'pairs', len(parts))
        with tempfile.TemporaryDirectory() as d, dask.config.set(scheduler='synchronous'):
            ref.pretrain._save_txt(bag, d, bin_size=bin_size, target_seq_length=seq,
                                   masking=masking)
            files = {}
            for fn in sorted(os.listdir(d)):
                with open(os.path.join(d, fn), 'rb') as f:
                    files[fn] = f.read().decode('utf-8')

        def enc(r):
            r = dict(r)
            if 'masked_lm_positions' in r:
                r['masked_lm_positions'] = base64.b64encode(r['masked_lm_positions']).decode()
            return r
        cases.append(dict(name=name, masking=masking, bin_size=bin_size, seq=seq,
                          partitions=[[enc(r) for r in rows] for rows in parts], files=files))
        print('{}: {} rows, {} files'.format(name, sum(map(len, parts)), len(files)))
    with open(os.path.join(HERE, 'txt_output.json'), 'w') as f:
        json.dump(cases, f)


if __name__ == '__main__':
    main()
