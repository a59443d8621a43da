"""Build the per-code-point character-class table of the GPU Punkt segmenter
(lddl_amd/assets/punkt_props.bin).

The reference splits sentences with `nltk.tokenize.sent_tokenize` (lddl/dask/bert/pretrain.py:86),
i.e. nltk's PunktSentenceTokenizer (nltk 3.6.5, not vendored in the reference; installed in this
image under /opt/conda/lib/python3.9/site-packages). Its regular expressions and token properties
use Python `re` Unicode classes and `str` methods on single code points:

  bit 0  SPACE  re `\\s`            (period-context `\\s+` / `\\S*`, str.strip, str.rstrip)
  bit 1  UPPER  str.isupper()      (PunktToken.first_upper)
  bit 2  LOWER  str.islower()      (PunktToken.first_lower)
  bit 3  ALNOD  re `[^\\W\\d]`       (PunktToken._RE_INITIAL, _RE_ALPHA)
  bit 4  DIGIT  re `\\d`            (PunktToken._RE_NUMERIC)

plus the `str.lower()` map, needed for the token types looked up in trained parameters
(abbreviations, collocations, sentence starters, orthographic context). Every bit is recorded by
asking Python itself, so the table IS the dependency's behaviour for this interpreter's Unicode
version (3.10: Unicode 13.0, the same as the reference's 3.9).

Binary layout (little endian):
  char[4] magic "LDPK", u32 version=1, u32 n_pages, u32 n_lower
  u16     l1[4352]            page of code points [p*256, p*256+256)
  u8      pages[n_pages][256] class bits
  i32     lower[n_lower][2]   (cp, lowercase cp) for every cp whose lower() differs, sorted by cp;
                              lowercase cp -1 marks the one two-code-point expansion
                              (U+0130 -> U+0069 U+0307)
"""
import os
import re
import struct
import sys

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'lddl_amd',
                   'assets', 'punkt_props.bin')


def main(out=OUT):
    sp, alnod, dig = re.compile(r'\s'), re.compile(r'[^\W\d]'), re.compile(r'\d')
    props = np.zeros(0x110000, np.uint8)
    lower = []
    for cp in range(0x110000):
        if 0xD800 <= cp < 0xE000:
            continue
        ch = chr(cp)
        b = 0
        if sp.match(ch):
            b |= 1
        if ch.isupper():
            b |= 2
        if ch.islower():
            b |= 4
        if alnod.match(ch):
            b |= 8
        if dig.match(ch):
            b |= 16
        props[cp] = b
        lo = ch.lower()
        if lo != ch:
            if len(lo) == 1:
                lower.append((cp, ord(lo)))
            else:
                assert cp == 0x130 and lo == 'i̇', (hex(cp), lo)
                lower.append((cp, -1))
    pages, l1 = {}, np.zeros(0x1100, np.uint16)
    blob = []
    for p in range(0x1100):
        key = props[p * 256:(p + 1) * 256].tobytes()
        if key not in pages:
            pages[key] = len(blob)
            blob.append(key)
        l1[p] = pages[key]
    with open(out, 'wb') as f:
        f.write(b'LDPK' + struct.pack('<III', 1, len(blob), len(lower)))
        f.write(l1.tobytes())
        f.write(b''.join(blob))
        f.write(np.asarray(lower, np.int32).tobytes())
    print('{}: {} pages, {} lowercase pairs, {} bytes'.format(out, len(blob), len(lower),
                                                           os.path.getsize(out)))


if __name__ == '__main__':
    main(*sys.argv[1:])
