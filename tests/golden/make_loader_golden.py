"""Golden batches of the REFERENCE loader (lddl.torch.get_bert_pretrain_data_loader) over the
deterministic datasets of tests/loader_data.py. Run in the dev container only:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_loader_golden.py

* raw (unbinned, return_raw_samples=True): the sample order of ParquetDataset + ShuffleBuffer;
* binned static masking (return_raw_samples=False): the collated tensors of every step of two
  epochs (bin choice of Binned, shuffle buffer order, _to_encoded_inputs).
Both use num_workers=2 DataLoader workers, as the reference requires persistent workers.
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from make_goldens import import_reference, VOCAB_UNCASED  # noqa: E402
from loader_data import make_loader_dataset  # noqa: E402


def main():
    ref = import_reference()
    import transformers
    out = {}
    with tempfile.TemporaryDirectory() as d:
        raw_dir = os.path.join(d, 'raw')
        make_loader_dataset(raw_dir, VOCAB_UNCASED, binned=False, static=False)
        dl = ref.torch_bert.get_bert_pretrain_data_loader(
            raw_dir, local_rank=0, shuffle_buffer_size=8, shuffle_buffer_warmup_factor=2,
            tokenizer_class=transformers.BertTokenizerFast, vocab_file=VOCAB_UNCASED,
            data_loader_kwargs={'batch_size': 3, 'num_workers': 2}, return_raw_samples=True,
            base_seed=777, start_epoch=1)
        seq = []
        for epoch in range(2):
            for batch in dl:
                seq += ['{}|{}|{}'.format(a, b, int(c)) for a, b, c in zip(*batch[:3])]
                seq.append('--batch--')
        out['raw_order'] = np.asarray(seq)
        out['raw_len'] = np.asarray(len(dl))
        bin_dir = os.path.join(d, 'bin')
        make_loader_dataset(bin_dir, VOCAB_UNCASED, binned=True, static=True)
        dl = ref.torch_bert.get_bert_pretrain_data_loader(
            bin_dir, local_rank=0, shuffle_buffer_size=8, shuffle_buffer_warmup_factor=2,
            tokenizer_class=transformers.BertTokenizerFast, vocab_file=VOCAB_UNCASED,
            data_loader_kwargs={'batch_size': 3, 'num_workers': 2}, base_seed=4242)
        k = 0
        for epoch in range(2):
            for batch in dl:
                for name in ('input_ids', 'token_type_ids', 'attention_mask', 'labels',
                             'next_sentence_labels'):
                    out['bin{}_{}'.format(k, name)] = batch[name].numpy()
                k += 1
        out['bin_steps'] = np.asarray(k)
        out['bin_len'] = np.asarray(len(dl))
    np.savez_compressed(os.path.join(HERE, 'loader.npz'), **out)
    print('loader goldens: raw {} entries, binned {} steps'.format(len(out['raw_order']), k))


if __name__ == '__main__':
    main()
