"""Build the per-code-point BERT normaliser / pre-tokeniser tables (lddl_amd/assets/bert_norm_*.bin).

The reference tokenizes with `transformers.BertTokenizerFast` (lddl/dask/bert/pretrain.py:584-587,
79-80), whose normaliser and pre-tokeniser live in the HF `tokenizers` Rust crate (not vendored in
the reference; the version installed in this image is tokenizers 0.22.2). Its published algorithm:

  BertNormalizer(clean_text, handle_chinese_chars, strip_accents=None -> lowercase, lowercase):
    clean_text      drop U+0000, U+FFFD and "control" chars (Unicode C* except \\t \\n \\r);
                    map whitespace chars to ' '
    chinese chars   pad CJK ideographs with spaces: c -> ' c '
    strip_accents   NFD, then drop category Mn
    lowercase       char::to_lowercase per char
  BertPreTokenizer: split on whitespace (dropped), isolate every punctuation char.

Applied to ONE code point, the composition yields exactly one of four shapes (verified over all
1,112,064 scalar values by this script): DROP (""), SPACE (" "), ISO (one isolated char, possibly
remapped, e.g. CJK or punctuation) or WORD (1..3 word chars). Except for NFD canonical reordering
across neighbouring code points (only reachable through non-Mn marks with non-zero combining
class, e.g. U+1D165), the whole normaliser is therefore a per-code-point map, which this script
records by probing the installed `tokenizers` directly, so the table IS the dependency's behaviour.

Binary layout (little endian):
  char[4]  magic "LDNT", u32 version=1, u32 lowercase, u32 n_pages, u32 pool_bytes
  u16      l1[4352]                 page index of code points [p*256, p*256+256)
  u32      pages[n_pages][256]      entries
  u8       pool[pool_bytes]         WORD expansions: u8 nbytes, u8 nchars, utf8 bytes
Entry:  bits 31..30 class (0 WORD, 1 DROP, 2 SPACE, 3 ISO), bit 29 IDENT (output == input),
        bit 28 MULTI (pool offset in bits 0..23), otherwise bits 0..20 = the single output cp.
"""
import argparse
import struct

import numpy as np

WORD, DROP, SPACE, ISO = 0, 1, 2, 3
IDENT, MULTI = 1 << 29, 1 << 28


def build(lowercase):
    from tokenizers import normalizers, pre_tokenizers
    norm = normalizers.BertNormalizer(clean_text=True, handle_chinese_chars=True,
                                      strip_accents=None, lowercase=lowercase)
    pre = pre_tokenizers.BertPreTokenizer()
    entries = np.zeros(0x110000, np.uint32)
    pool = bytearray()
    pool_index = {}
    for cp in range(0x110000):
        if 0xD800 <= cp < 0xE000:  # surrogates never occur in valid UTF-8: treat as U+FFFD
            entries[cp] = DROP << 30
            continue
        n = norm.normalize_str(chr(cp))
        if n == '':
            entries[cp] = DROP << 30
        elif n == ' ':
            entries[cp] = SPACE << 30
        else:
            pieces = pre.pre_tokenize_str('a' + n + 'a')
            if len(pieces) == 1:
                cls = WORD
                out = n
            else:
                assert len(pieces) == 3 and pieces[0][0] == 'a' and pieces[2][0] == 'a', (cp, n)
                out = pieces[1][0]
                assert len(out) == 1, (cp, n)
                cls = ISO
            if out == chr(cp):
                entries[cp] = (cls << 30) | IDENT
            elif len(out) == 1:
                entries[cp] = (cls << 30) | ord(out)
            else:
                assert cls == WORD
                if out not in pool_index:
                    b = out.encode('utf-8')
                    pool_index[out] = len(pool)
                    pool += bytes([len(b), len(out)]) + b
                entries[cp] = (cls << 30) | MULTI | pool_index[out]
    # two-level table with deduplicated pages
    pages, page_ids, l1 = [], {}, np.zeros(0x110000 >> 8, np.uint16)
    for p in range(0x110000 >> 8):
        blk = entries[p * 256:(p + 1) * 256].tobytes()
        if blk not in page_ids:
            page_ids[blk] = len(pages)
            pages.append(blk)
        l1[p] = page_ids[blk]
    hdr = b'LDNT' + struct.pack('<IIII', 1, int(lowercase), len(pages), len(pool))
    return hdr + l1.tobytes() + b''.join(pages) + bytes(pool)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--outdir', default='lddl_amd/assets')
    args = ap.parse_args()
    for lower, name in ((True, 'uncased'), (False, 'cased')):
        blob = build(lower)
        path = '{}/bert_norm_{}.bin'.format(args.outdir, name)
        with open(path, 'wb') as f:
            f.write(blob)
        print(path, len(blob), 'bytes')


if __name__ == '__main__':
    main()
