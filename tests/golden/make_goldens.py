"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself (run in the dev
container only; /root/reference does not exist on the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py

Import recipe: the reference is pure Python; its deps dask 2021.10 / nltk 3.6.5
live in /opt/conda/lib/python3.9/site-packages; `dask.dataframe` does not import under NumPy 2,
so the six modules lddl/dask/bert/binning.py:35-41 imports are stubbed (only
`_to_dataframe_binned` is called, which uses none of them); mpi4py is a single-rank fake;
`np.NAN` (lddl/dask/load_balance.py:262) is shimmed.

Tokenizer: the reference pins transformers==4.16.2 (setup.py:55) whose
`tokenize(s, max_length=512, truncation=True)` (lddl/dask/bert/pretrain.py:79-80) truncates to
512 pieces; the installed 5.15 ignores those kwargs, so `Tok416` restores the 4.16.2 semantics
through the backend (`enable_truncation` + `encode(add_special_tokens=False).tokens`).
Sentence splitting: nltk's English punkt model is not available offline, so
`nltk.tokenize.sent_tokenize` is the untrained `PunktSentenceTokenizer().tokenize`.
vocab_words (pretrain.py:384) iterates a Rust HashMap whose order changes per process;
fixtures pass the id-ordered tuple, which is what lddl_amd uses.

Everything written is data (inputs + expected outputs); nothing from the reference is copied.
"""
import io
import json
import os
import random
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
ASSETS = os.path.join(REPO, 'lddl_amd', 'assets')
VOCAB_UNCASED = os.path.join(ASSETS, 'vocab_synth_uncased_30522.txt')
VOCAB_CASED = os.path.join(ASSETS, 'vocab_synth_cased_28996.txt')


def import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, '/root/reference')
    sys.path.append('/opt/conda/lib/python3.9/site-packages')
    np.NAN = np.nan
    import dask  # noqa: F401  (real dask 2021.10, pure python)
    for name in ('dask.dataframe', 'dask.dataframe.core', 'dask.dataframe.io',
                 'dask.dataframe.io.parquet', 'dask.dataframe.io.parquet.core',
                 'dask.dataframe.io.parquet.arrow'):
        sys.modules[name] = types.ModuleType(name)
    sys.modules['dask.dataframe.core'].Scalar = object
    sys.modules['dask.dataframe.io.parquet.core'].get_engine = None
    sys.modules['dask.dataframe.io.parquet.arrow']._index_in_schema = None

    class _Comm:
        def Get_size(self):
            return 1

        def Get_rank(self):
            return 0

        def barrier(self):
            return None

        def Allreduce(self, a, b, op=None):
            return None

    mpi = types.ModuleType('mpi4py')
    mpi.MPI = types.SimpleNamespace(COMM_WORLD=_Comm(), SUM='sum', MAX='max', IN_PLACE='in_place')
    sys.modules['mpi4py'] = mpi
    import nltk
    from nltk.tokenize.punkt import PunktSentenceTokenizer
    _punkt = PunktSentenceTokenizer()
    nltk.tokenize.sent_tokenize = lambda text, language='english': _punkt.tokenize(text)
    from lddl.dask.bert import pretrain, binning
    from lddl.dask import load_balance
    from lddl.torch import bert as torch_bert
    return types.SimpleNamespace(pretrain=pretrain, binning=binning, load_balance=load_balance,
                                 torch_bert=torch_bert)


class Tok416:
    """transformers 4.16.2 `tokenize(s, max_length, truncation)` semantics on the 5.15 backend."""

    def __init__(self, vocab_file, lower=True):
        import transformers
        self.hf = transformers.BertTokenizerFast(vocab_file, do_lower_case=lower)
        self.bt = self.hf.backend_tokenizer
        self.vocab = self.hf.vocab

    def tokenize(self, s, max_length=None, truncation=False):
        if truncation and max_length is not None:
            self.bt.enable_truncation(max_length)
        else:
            self.bt.no_truncation()
        return self.bt.encode(s, add_special_tokens=False).tokens


def id_ordered_vocab(vocab):
    return tuple(w for w, _ in sorted(vocab.items(), key=lambda kv: kv[1]))


class ListBag:
    """Minimal stand-in for a dask bag partition: `_get_documents` only maps and filters."""

    def __init__(self, items):
        self.items = list(items)

    def map(self, f):
        return ListBag(map(f, self.items))

    def filter(self, f):
        return ListBag(filter(f, self.items))


def ragged(list_of_lists, dtype=np.int32):
    off = np.zeros(len(list_of_lists) + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in list_of_lists])
    flat = np.fromiter((v for x in list_of_lists for v in x), dtype=dtype, count=int(off[-1]))
    return flat, off


# ------------------------------------------------------------------------------------------------
# F1: MT19937 / CPython `random` stream (pins the replay RNG)
# ------------------------------------------------------------------------------------------------
def gen_mt():
    out = []
    for seed in (0, 1, 42, 12345, 2**32 - 1, 2**32, 2**40 + 3, 123456789012345678901234567890):
        random.seed(seed)
        st = random.getstate()[1]
        rec = {'seed': str(seed), 'state_head': list(st[:8]), 'state_pos': st[624]}
        rec['u32'] = [random.getrandbits(32) for _ in range(64)]
        rec['random_hex'] = [random.random().hex() for _ in range(32)]
        rec['randint'] = [[a, b, random.randint(a, b)] for a, b in
                          [(0, 0), (0, 1), (2, 125), (1, 7), (0, 30521), (0, 2**31 - 1), (5, 5)] * 4]
        x = list(range(50))
        random.shuffle(x)
        rec['shuffle50'] = x
        rec['randrange'] = [random.randrange(n) for n in (1, 2, 3, 1000, 16384)]
        rec['sample'] = random.sample(list(range(100)), 100)
        rec['choices'] = random.choices(list(range(8)), weights=[5, 0, 3, 9, 1, 1, 0, 2], k=40)
        rec['tail_u32'] = [random.getrandbits(32) for _ in range(4)]
        out.append(rec)
    with open(os.path.join(HERE, 'mt19937.json'), 'w') as f:
        json.dump(out, f)


# ------------------------------------------------------------------------------------------------
# F2: sentence -> wordpiece ids (pretrain.py:79-80 through the pinned tokenizer semantics)
# ------------------------------------------------------------------------------------------------
EDGE_SENTENCES = [
    'Hello World.', 'The quick brown fox, jumped over the lazy dog!', '',
    'a[MASK]b [CLS] x[SEP]y [PAD][UNK] [mask] [ MASK ] [MASK', '[[MASK]]', 'café naïve résumé Ångström',
    '中文字符 and 日本語 mixed中text', 'tab\there\nnewline\rcr\u000bvt\u000cff',
    'ctrl\u0000\u0001\u0007\u007f\u0085­soft​zw‍j�rep﻿bom',
    'spaces nbsp em　ideo ls ps', 'İstanbul ΣΟΦΙΑ ẞ ß ﬁ Ω K',
    'x' * 99, 'y' * 100, 'z' * 101, 'w' * 250 + ' tail', 'é' * 120, 'ab' + '́' * 200,
    ' '.join(['plut'] * 700), ' '.join(['strommeth'] * 300), '!' * 600,
    'don\'t stop-believing (ok) "quoted" 3.14159 1,000,000 $5 #tag @me 50% a&b c/d e\\f',
    '\U0001F600 emoji \U0001F44D\U0001F3FD and ❤️', 'ＡＢＣ fullwidth １２',
    'नमस्ते สวัสดี 각가 שלום',
    'ᴖ5\U0001D165\U0001D16E combininģ́⃝', 'end.', '...', '-', 'A', '­', '\u0000',
]


def random_unicode_strings(rng, n):
    pools = [
        (0x20, 0x7F), (0x20, 0x7F), (0x20, 0x7F), (0xA0, 0x250), (0x300, 0x370), (0x370, 0x530),
        (0x4E00, 0x9FFF), (0x3000, 0x3100), (0xAC00, 0xD7A4), (0x2000, 0x2070), (0xF900, 0xFB00),
        (0xFE00, 0xFF70), (0x1F300, 0x1F700), (0x0, 0x20), (0x10000, 0x30000), (0xE000, 0xE100),
        (0x600, 0x700), (0x900, 0xA00), (0x1E00, 0x2000),
    ]
    out = []
    for _ in range(n):
        L = rng.randint(1, 60)
        chars = []
        for _ in range(L):
            lo, hi = pools[rng.randrange(len(pools))]
            cp = rng.randrange(lo, hi)
            if 0xD800 <= cp < 0xE000:
                cp = 0x41
            chars.append(chr(cp))
        out.append(''.join(chars))
    return out


def gen_tokenize(tok_u, tok_c):
    from lddl_amd import synth
    rng = random.Random(99)
    corp = synth.generate(seed=4242, n_bytes=300_000, nonascii_frac=0.08, threads=4)
    sents = list(EDGE_SENTENCES) + random_unicode_strings(rng, 400)
    sents += [corp.sentence(i) for i in range(0, corp.n_sent, 3)]
    ids_u = [tok_u.hf.convert_tokens_to_ids(tok_u.tokenize(s, max_length=512, truncation=True))
             for s in sents]
    ids_c = [tok_c.hf.convert_tokens_to_ids(tok_c.tokenize(s, max_length=512, truncation=True))
             for s in sents]
    text = [s.encode('utf-8') for s in sents]
    sent_off = np.zeros(len(text) + 1, np.int64)
    sent_off[1:] = np.cumsum([len(b) for b in text])
    fu, ou = ragged(ids_u)
    fc, oc = ragged(ids_c)
    np.savez_compressed(os.path.join(HERE, 'tokenize.npz'),
                        text=np.frombuffer(b''.join(text), np.uint8), sent_off=sent_off,
                        ids_uncased=fu, off_uncased=ou, ids_cased=fc, off_cased=oc)
    print('tokenize: {} sentences, {} / {} pieces'.format(len(sents), len(fu), len(fc)))


# ------------------------------------------------------------------------------------------------
# F3: documents — raw `<id> <text>` lines -> reference _get_documents (pretrain.py:77-97)
# ------------------------------------------------------------------------------------------------
def make_doc_lines(n_bytes, seed, nonascii):
    from lddl_amd import synth
    corp = synth.generate(seed=seed, n_bytes=n_bytes, nonascii_frac=nonascii, threads=4)
    lines = ['wiki-{} {}'.format(d, ' '.join(doc)) for d, doc in enumerate(corp.documents())]
    # edge documents: literal special tokens, a doc whose sentences all normalise away, a
    # one-sentence doc, tab-separated id, a doc with a >512-piece sentence
    lines.insert(3, 'edge-0 Look at [MASK] here. And [SEP] there [CLS]. Fine.')
    lines.insert(5, 'edge-1 \u0000\u0001\u0002 \u00ad\u200b')
    lines.insert(6, 'edge-1b Real sentence. \u0000\u0001 \u00ad. Another real one.')
    lines.insert(7, 'edge-2 Only one sentence here')
    lines.insert(9, 'edge-3\tTab separated id. Second one!')
    lines.insert(11, 'edge-4 ' + ' '.join(['plut'] * 600) + '. Short after.')
    return lines


def gen_documents(ref, tok, lines, tag):
    docs = ref.pretrain._get_documents(ListBag(lines), tok).items
    # The hot-path input: the stripped, non-empty Punkt sentences of every line.
    from lddl.dask.readers import split_id_text
    import nltk
    sent_strs, line_sent = [], [0]
    for line in lines:
        _, text = split_id_text(line)
        ss = [s.strip() for s in nltk.tokenize.sent_tokenize(text)]
        sent_strs += [s for s in ss if s]
        line_sent.append(len(sent_strs))
    vocab = tok.vocab
    doc_ids = [d._id for d in docs]
    sent_ids = [[vocab[t] for t in s._tokens] for d in docs for s in d._sentences]
    doc_nsent = [len(d._sentences) for d in docs]
    text = [s.encode('utf-8') for s in sent_strs]
    sent_off = np.zeros(len(text) + 1, np.int64)
    sent_off[1:] = np.cumsum([len(b) for b in text])
    flat, off = ragged(sent_ids)
    np.savez_compressed(os.path.join(HERE, 'documents_{}.npz'.format(tag)),
                        text=np.frombuffer(b''.join(text), np.uint8), sent_off=sent_off,
                        line_sent_off=np.asarray(line_sent, np.int64),
                        line_ids=np.asarray([split_id_text(l)[0] for l in lines]),
                        doc_ids=np.asarray(doc_ids), doc_nsent=np.asarray(doc_nsent, np.int64),
                        ids=flat, ids_off=off)
    print('documents_{}: {} lines -> {} docs, {} sentences'.format(tag, len(lines), len(docs),
                                                                   len(sent_ids)))
    return docs


# ------------------------------------------------------------------------------------------------
# F4: pairs + static masking — _to_partition_pairs (pretrain.py:386-402) per seeded partition
# ------------------------------------------------------------------------------------------------
def partition_pairs(ref, docs, seed, dup, seq, short_seq_prob, masking, ratio, vocab_words):
    random.seed(seed)
    docs = tuple(docs)
    pairs = []
    for _ in range(dup):
        for di in range(len(docs)):
            pairs.extend(ref.pretrain.create_pairs_from_document(
                docs, di, max_seq_length=seq, short_seq_prob=short_seq_prob, masking=masking,
                masked_lm_ratio=ratio, vocab_words=vocab_words))
    random.shuffle(pairs)
    return pairs


def gen_pairs(ref, tok, docs, cases):
    vocab = tok.vocab
    vocab_words = id_ordered_vocab(vocab)
    for c in cases:
        parts = []
        lo = 0
        for size in c['partition_sizes']:
            parts.append(docs[lo:lo + size])
            lo += size
        A, B, rn, nt, pos, lab, pair_off, npy = [], [], [], [], [], [], [0], []
        for p, part in enumerate(parts):
            pairs = partition_pairs(ref, part, c['seeds'][p], c['dup'], c['seq'], c['short'],
                                    c['masking'], c['ratio'], vocab_words)
            for q in pairs:
                A.append([vocab[t] for t in q['A'].split(' ')])
                B.append([vocab[t] for t in q['B'].split(' ')])
                rn.append(q['is_random_next'])
                nt.append(q['num_tokens'])
                if c['masking']:
                    npy.append(q['masked_lm_positions'])
                    pos.append(np.load(io.BytesIO(q['masked_lm_positions'])).tolist())
                    lab.append([vocab[t] for t in q['masked_lm_labels'].split(' ')])
            pair_off.append(len(A))
        fa, oa = ragged(A)
        fb, ob = ragged(B)
        extra = {}
        if c['masking']:
            fp, op = ragged(pos, np.uint16)
            fl, ol = ragged(lab)
            extra = dict(pos=fp, pos_off=op, labels=fl, labels_off=ol,
                         npy_first=np.frombuffer(npy[0], np.uint8),
                         npy_lens=np.asarray([len(x) for x in npy], np.int64))
        np.savez_compressed(os.path.join(HERE, 'pairs_{}.npz'.format(c['name'])),
                            part_doc_sizes=np.asarray(c['partition_sizes'], np.int64),
                            part_doc_begin=np.asarray(c.get('doc_begin', 0)),
                            seeds=np.asarray(c['seeds'], np.int64),
                            params=np.asarray([c['dup'], c['seq'], int(c['masking'])], np.int64),
                            short_seq_prob=np.asarray(c['short']), ratio=np.asarray(c['ratio']),
                            a=fa, a_off=oa, b=fb, b_off=ob, is_random_next=np.asarray(rn, bool),
                            num_tokens=np.asarray(nt, np.int64),
                            part_pair_off=np.asarray(pair_off, np.int64), **extra)
        print('pairs_{}: {} pairs'.format(c['name'], len(A)))


# ------------------------------------------------------------------------------------------------
# F5: binning — _to_dataframe_binned (binning.py:63-93)
# ------------------------------------------------------------------------------------------------
def gen_binning(ref):
    rng = random.Random(5)
    cases = []
    for seq, bin_size, n in ((128, 32, 200), (512, 8, 1000), (512, 64, 300), (128, 128, 50),
                             (512, 8, 0), (512, 8, 1), (128, 16, 64)):
        nbins = seq // bin_size
        nts = [rng.randint(5, seq) for _ in range(n)]
        if n > 3:
            nts[:3] = [seq, 1 + bin_size, bin_size]
        seqs = [{'uid': i, 'num_tokens': v} for i, v in enumerate(nts)]
        if n == 0:
            cases.append({'seq': seq, 'bin_size': bin_size, 'num_tokens': [], 'uid_order': [],
                          'bin_id': []})
            continue
        df = ref.binning._to_dataframe_binned(seqs, ['uid', 'num_tokens'],
                                               {'uid': np.int64, 'num_tokens': np.uint16},
                                               bin_size, nbins)
        cases.append({'seq': seq, 'bin_size': bin_size, 'num_tokens': nts,
                      'uid_order': df['uid'].tolist(), 'bin_id': df['bin_id'].tolist()})
    with open(os.path.join(HERE, 'binning.json'), 'w') as f:
        json.dump(cases, f)


# ------------------------------------------------------------------------------------------------
# F6: load balance plans — load_balance._balance (load_balance.py:321-369), single rank
# ------------------------------------------------------------------------------------------------
def gen_balance(ref):
    import pyarrow as pa
    import pyarrow.parquet as pq
    lb = ref.load_balance
    rng = random.Random(11)
    specs = [([5, 9, 2, 7], 2), ([10, 3, 3, 3, 1, 0, 8], 3), ([1, 2, 3, 4, 5, 6, 7, 8], 4),
             ([100, 1, 1, 1, 1, 1], 3), ([4, 4, 4, 5], 2), ([0, 0, 7], 2), ([13], 1),
             ([rng.randint(0, 40) for _ in range(16)], 5), ([rng.randint(20, 30) for _ in range(12)], 4),
             ([3, 8], 5), ([6, 6, 6], 2), ([2, 2, 2, 2], 2), ([9, 1], 2)]
    cases = []
    for counts, S in specs:
        with tempfile.TemporaryDirectory() as d:
            indir, outdir = os.path.join(d, 'in'), os.path.join(d, 'out')
            os.makedirs(indir)
            os.makedirs(outdir)
            paths, uid = [], 0
            for i, c in enumerate(counts):
                p = os.path.join(indir, 'part.{}.parquet_0'.format(i))
                pq.write_table(pa.table({'uid': pa.array(range(uid, uid + c), pa.int64())}), p)
                uid += c
                paths.append(p)
            rec = {'counts': counts, 'num_shards': S}
            calls = {'n': 0}
            orig_barrier = lb.barrier

            def capped_barrier():
                calls['n'] += 1
                if calls['n'] > 200:
                    raise RuntimeError('nonterminating')

            lb.barrier = capped_barrier
            try:
                shards = lb._balance(sorted(paths), S, outdir, keep_orig=True, postfix='_0')
                out = {}
                for s in shards:
                    t = pq.read_table(s._output_file.path)
                    out[os.path.basename(s._output_file.path)] = t.column('uid').to_pylist()
                rec['shards'] = out
                rec['status'] = 'ok'
            except RuntimeError as e:
                rec['status'] = str(e)
            except Exception as e:  # H7 and friends
                rec['status'] = 'error: {}'.format(type(e).__name__)
            finally:
                lb.barrier = orig_barrier
            cases.append(rec)
    with open(os.path.join(HERE, 'balance.json'), 'w') as f:
        json.dump(cases, f)
    print('balance:', [c['status'] for c in cases])


# ------------------------------------------------------------------------------------------------
# F7: collate — _to_encoded_inputs / _mask_tokens (lddl/torch/bert.py:69-196)
# ------------------------------------------------------------------------------------------------
def gen_collate(ref, tok_c, tok_u, docs_c, docs_u):
    import torch
    tb = ref.torch_bert
    out = {}
    vw_c = id_ordered_vocab(tok_c.vocab)
    vw_u = id_ordered_vocab(tok_u.vocab)
    dyn = partition_pairs(ref, docs_c[:30], 777, 2, 512, 0.1, False, 0.15, vw_c)[:48]
    sta = partition_pairs(ref, docs_u[:30], 778, 2, 128, 0.1, True, 0.15, vw_u)[:40]
    batch_dyn = [(q['A'], q['B'], q['is_random_next']) for q in dyn]
    batch_sta = [(q['A'], q['B'], q['is_random_next'], q['masked_lm_positions'],
                  q['masked_lm_labels']) for q in sta]
    enc_s = tb._to_encoded_inputs(batch_sta, tok_u.hf, sequence_length_alignment=8, ignore_index=-1)
    for k, v in enc_s.items():
        out['static_' + k] = v.numpy()
    for align in (8, 1, 64):
        enc = tb._to_encoded_inputs(batch_dyn, tok_c.hf, sequence_length_alignment=align,
                                    ignore_index=-1)
        for k, v in enc.items():
            out['dyn{}_{}'.format(align, k)] = v.numpy()
    enc = tb._to_encoded_inputs(batch_dyn, tok_c.hf, sequence_length_alignment=8, ignore_index=-1)
    stm = enc['special_tokens_mask']
    ids = enc['input_ids']
    for seed in (0, 1234):
        torch.manual_seed(seed)
        new_ids, labels = tb._mask_tokens(ids.clone(), special_tokens_mask=stm, tokenizer=tok_c.hf,
                                          mlm_probability=0.15, ignore_index=-1)
        # capture the same RNG draws in the same order (bert.py:166-191)
        torch.manual_seed(seed)
        prob = torch.full(ids.shape, 0.15)
        prob.masked_fill_(stm.bool(), value=0.0)
        masked = torch.bernoulli(prob).bool()
        repl = torch.bernoulli(torch.full(ids.shape, 0.8)).bool() & masked
        rnd = torch.bernoulli(torch.full(ids.shape, 0.5)).bool() & masked & ~repl
        words = torch.randint(len(tok_c.hf), ids.shape, dtype=torch.long)
        out['mask{}_input_ids'.format(seed)] = new_ids.numpy()
        out['mask{}_labels'.format(seed)] = labels.numpy()
        out['mask{}_masked'.format(seed)] = masked.numpy()
        out['mask{}_replaced'.format(seed)] = repl.numpy()
        out['mask{}_random'.format(seed)] = rnd.numpy()
        out['mask{}_words'.format(seed)] = words.numpy()
    # the raw batches (token strings -> ids in each vocab, plus the static extras)
    def split_ids(vocab, s):
        return [vocab[t] for t in s.split()]
    for name, batch, vocab in (('dyn', batch_dyn, tok_c.vocab), ('static', batch_sta, tok_u.vocab)):
        fa, oa = ragged([split_ids(vocab, b[0]) for b in batch])
        fb, ob = ragged([split_ids(vocab, b[1]) for b in batch])
        out[name + '_a'], out[name + '_a_off'] = fa, oa
        out[name + '_b'], out[name + '_b_off'] = fb, ob
        out[name + '_is_random_next'] = np.asarray([b[2] for b in batch], bool)
    fp, op = ragged([np.load(io.BytesIO(b[3])).tolist() for b in batch_sta], np.uint16)
    fl, ol = ragged([split_ids(tok_u.vocab, b[4]) for b in batch_sta])
    out.update(static_pos=fp, static_pos_off=op, static_lab=fl, static_lab_off=ol,
               vocab_len_cased=np.asarray(len(tok_c.hf)), mask_id_cased=np.asarray(
                   tok_c.hf.convert_tokens_to_ids(tok_c.hf.mask_token)))
    np.savez_compressed(os.path.join(HERE, 'collate.npz'), **out)
    print('collate: dyn batch {}x{}, static batch {}x{}'.format(
        *out['dyn8_input_ids'].shape, *out['static_input_ids'].shape))


def main():
    ref = import_reference()
    tok_u = Tok416(VOCAB_UNCASED, lower=True)
    tok_c = Tok416(VOCAB_CASED, lower=False)
    gen_mt()
    gen_tokenize(tok_u, tok_c)
    lines_u = make_doc_lines(400_000, 5151, 0.03)
    docs_u = gen_documents(ref, tok_u, lines_u, 'uncased')
    lines_c = make_doc_lines(250_000, 6161, 0.03)
    docs_c = gen_documents(ref, tok_c, lines_c, 'cased')
    n = len(docs_u)
    cases = [
        dict(name='s128_mask', partition_sizes=[20, 7, 1, 2, 30], seeds=[1, 2, 3, 4, 12345],
             dup=5, seq=128, short=0.1, masking=True, ratio=0.15),
        dict(name='s128_nomask', partition_sizes=[25, 13], seeds=[7, 8], dup=5, seq=128,
             short=0.1, masking=False, ratio=0.15),
        dict(name='s512_mask', partition_sizes=[40, 15], seeds=[99, 100], dup=3, seq=512,
             short=0.1, masking=True, ratio=0.15),
        dict(name='s512_nomask_short', partition_sizes=[n - 5], seeds=[2024], dup=2, seq=512,
             short=0.5, masking=False, ratio=0.15),
        dict(name='s64_mask_ratio', partition_sizes=[12, 12], seeds=[5, 6], dup=4, seq=64,
             short=0.3, masking=True, ratio=0.2),
    ]
    gen_pairs(ref, tok_u, docs_u, cases)
    gen_binning(ref)
    gen_balance(ref)
    gen_collate(ref, tok_c, tok_u, docs_c, docs_u)


if __name__ == '__main__':
    main()
