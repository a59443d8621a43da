"""Input side of the preprocessor: the reference's lddl/dask/readers.py semantics without Dask.

* files: every `*.txt` under the source directory, sorted (readers.py:35-41); Wikipedia adds
  `/<lang>` (readers.py:81-82);
* blocks: `dask.bag.read_text(files, blocksize)` cuts each file into byte blocks of `blocksize`,
  moved forward to the next line start (dask.bytes.read_block with delimiter b'\\n'); no
  blocksize = one block per file; a block is one partition;
* lines are `strip()`ed and empty ones dropped (readers.py:31-32);
* `random_sample(sample_ratio, seed)` keeps a line iff random() < ratio, with the per-partition
  MT states of dask 2021.10's `random_state_data_python` (624 words of randint(0, 2**32) each
  drawn from Random(seed), in partition order).

Blocks are planned from file sizes and a short scan for the newline after each cut
(`plan_blocks`), so a process reads and decodes only the blocks it owns (`read_block`): under
torchrun every rank holds its own share of the corpus, not all of it.
"""
import os
import random
import re
from dataclasses import dataclass


def find_files_under(path, extensions=('.txt',)):
    out = []
    for cur, _, names in os.walk(path):
        for n in names:
            if os.path.splitext(n)[1] in extensions:
                out.append(os.path.join(cur, n))
    return sorted(out)


def total_bytes_of(files):
    return sum(map(os.path.getsize, files))


def estimate_block_size(paths, num_blocks):
    """readers.py:48-57."""
    total = sum(total_bytes_of(find_files_under(p)) for p in paths if p is not None)
    print('total_bytes = {}, num_blocks = {}'.format(total, num_blocks))
    bs = round(total / num_blocks)
    print('block_size = {} bytes'.format(bs))
    return bs


def _block_starts(data, blocksize):
    """Start offsets of dask read_block blocks of `data` (bytes)."""
    n = len(data)
    if not blocksize or n == 0:
        return [0, n]
    starts = [0]
    for off in range(blocksize, n, blocksize):
        j = data.find(b'\n', off - 1)
        s = n if j < 0 else j + 1
        starts.append(s)
    starts.append(n)
    return starts


def _next_line_start(f, off, size, chunk=1 << 13):
    """First byte after the first newline at or after offset off - 1 (dask read_block)."""
    pos = off - 1
    while pos < size:
        f.seek(pos)
        buf = f.read(chunk)
        j = buf.find(b'\n')
        if j >= 0:
            return pos + j + 1
        pos += len(buf)
        if not buf:
            break
    return size


def _file_block_starts(fn, blocksize):
    """_block_starts of the file's bytes, reading only around the cuts."""
    size = os.path.getsize(fn)
    if not blocksize or size == 0:
        return [0, size]
    starts = [0]
    with open(fn, 'rb') as f:
        for off in range(blocksize, size, blocksize):
            starts.append(_next_line_start(f, off, size))
    starts.append(size)
    return starts


@dataclass
class Block:
    """One dask partition before it is read: bytes [start, end) of `path` (empty if end <= start),
    with the MT state of its random_sample as uint32[625] (624 words + index; None: no
    sampling)."""
    path: str
    start: int
    end: int
    mt: object = None
    ratio: float = 1.0

    @property
    def nbytes(self):
        return max(self.end - self.start, 0)

    @property
    def state(self):
        """The state as random.Random.getstate() gives it (None: no sampling)."""
        if self.mt is None:
            return None
        return (3, tuple(int(x) for x in self.mt), None)


def plan_blocks(path, blocksize=None, sample_ratio=1.0, sample_seed=12345):
    """Blocks of one source in partition order (no data read beyond the cut scans)."""
    blocks = []
    for fn in find_files_under(path):
        st = _file_block_starts(fn, blocksize)
        for a, b in zip(st[:-1], st[1:]):
            blocks.append(Block(fn, a, b if (b > a or len(st) <= 2) else a))
    if sample_ratio < 1.0:
        for b, s in zip(blocks, random_state_data(len(blocks), sample_seed)):
            b.mt, b.ratio = s, sample_ratio
    return blocks


def _strip_bytes(raw):
    """str(raw).strip() as UTF-8 bytes. bytes.strip() removes ASCII whitespace only; a line whose
    remaining first or last byte could be other whitespace (\\x1c-\\x1f, non-ASCII: U+0085,
    U+00A0, U+2000.., U+3000 ...) takes the exact str path."""
    s = raw.strip()
    if s and (s[0] >= 0x80 or s[-1] >= 0x80 or 0x1c <= s[0] <= 0x1f or 0x1c <= s[-1] <= 0x1f):
        return raw.decode('utf-8').strip().encode('utf-8')
    return s


def read_block(blk, as_bytes=False):
    """The partition's lines: stripped, non-empty, sampled (readers.py:60-71). as_bytes: the
    lines as bytes, for the GPU path, which validates them as UTF-8 on the device
    (lddl_utf8_check) instead of decoding the corpus into Python strings."""
    if blk.nbytes == 0:
        return []
    with open(blk.path, 'rb') as f:
        f.seek(blk.start)
        data = f.read(blk.end - blk.start)
    if as_bytes:
        lines = [x for x in map(_strip_bytes, data.split(b'\n')) if x]
    else:
        lines = _filter(data.split(b'\n'))
    if blk.state is None:
        return lines
    r = random.Random()
    r.setstate(blk.state)
    kept = []
    for x in lines:
        if r.random() < blk.ratio:
            kept.append(x)
        elif as_bytes:  # dask's read_text decodes every line strictly, sampled out or not; the
            x.decode('utf-8')  # kept ones are checked on the GPU (lddl_utf8_check)
    return kept


def read_blocks(files, blocksize=None):
    """List of blocks; each block is a list of raw lines (bytes, without the delimiter)."""
    blocks = []
    for fn in files:
        with open(fn, 'rb') as f:
            data = f.read()
        st = _block_starts(data, blocksize)
        for a, b in zip(st[:-1], st[1:]):
            if b <= a and len(st) > 2:
                blocks.append([])
                continue
            blocks.append(data[a:b].split(b'\n'))
    return blocks


def random_state_data_python(n, seed):
    """dask 2021.10 dask.utils.random_state_data_python (the per-partition states of
    bag.random_sample), as Random.getstate() tuples."""
    r = random.Random(seed)
    m = 1 << 32
    return [(3, tuple(r.randint(0, m) for _ in range(624)) + (624,), None) for _ in range(n)]


def random_state_data(n, seed):
    """random_state_data_python(n, seed) as uint32[n, 625] (words as setstate stores them), from
    the host library (lddl_random_state_data: 624 x n randint draws in C++ instead of Python)."""
    import numpy as np
    out = np.empty((n, 625), np.uint32)
    if n:
        lib, check = _host_lib()
        if abs(int(seed)) >= 1 << 64:
            raise ValueError('sample seed must be below 2**64 in magnitude')
        check(lib.lddl_random_state_data(n, abs(int(seed)), out.ctypes.data))
    return out


def _filter(block):
    out = []
    for raw in block:
        s = raw.decode('utf-8').strip()
        if s:
            out.append(s)
    return out


def read_bag_of_text(path, blocksize=None, sample_ratio=1.0, sample_seed=12345):
    """readers.py:60-71: partitions of stripped, non-empty lines, optionally sampled."""
    return [read_block(b) for b in plan_blocks(path, blocksize, sample_ratio, sample_seed)]


def wikipedia_dir(path, lang='en'):
    return os.path.join(path, lang)


def read_wikipedia(path, lang='en', blocksize=None, sample_ratio=1.0, sample_seed=12345):
    return read_bag_of_text(wikipedia_dir(path, lang), blocksize, sample_ratio, sample_seed)


def read_books(path, blocksize=None, sample_ratio=1.0, sample_seed=12345):
    return read_bag_of_text(path, blocksize, sample_ratio, sample_seed)


def read_common_crawl(path, blocksize=None, sample_ratio=1.0, sample_seed=12345):
    return read_bag_of_text(path, blocksize, sample_ratio, sample_seed)


def read_open_webtext(path, blocksize=None, sample_ratio=1.0, sample_seed=12345):
    return read_bag_of_text(path, blocksize, sample_ratio, sample_seed)


_WS = re.compile(r'\s')  # str patterns: \s is exactly str.isspace()
_WS_ASCII_B = re.compile(rb'[\t-\r\x1c-\x20]')


def split_id_text(raw_text):
    """readers.py:131-136: id = chars up to the first whitespace char; text = the rest after it."""
    m = _WS.search(raw_text)
    if m is None:
        return raw_text, ''
    return raw_text[:m.start()], raw_text[m.start() + 1:]


def split_id_text_bytes(raw):
    """split_id_text on a UTF-8 line, as bytes. Fast path: the first ASCII whitespace byte, when
    no non-ASCII byte comes before it (a non-ASCII char could itself be whitespace)."""
    m = _WS_ASCII_B.search(raw)
    i = len(raw) if m is None else m.start()
    if max(raw[:i], default=0) < 0x80:
        return raw[:i], raw[i + 1:]
    a, b = split_id_text(raw.decode('utf-8'))
    return a.encode('utf-8'), b.encode('utf-8')


_HOST = None


def _host_lib():
    """liblddl_host.so (lddl_amd/build.py): the reader's entry points without the HIP runtime,
    so they load without torch (the CLI reads while the main thread imports torch)."""
    global _HOST
    if _HOST is None:
        import ctypes
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '_lib',
                            'liblddl_host.so')
        if not os.path.exists(path):
            raise ImportError('{} is missing (run `python -m lddl_amd.build`)'.format(path))
        lib = ctypes.CDLL(path)
        c_i64, c_vp = ctypes.c_int64, ctypes.c_void_p
        lib.lddl_read_groups.restype = ctypes.c_int
        lib.lddl_read_groups.argtypes = [c_i64, c_vp, c_vp, c_vp, c_vp, ctypes.c_double, c_i64,
                                         c_vp, c_vp, ctypes.c_int, ctypes.POINTER(c_vp),
                                         ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), c_vp]
        lib.lddl_read_fill.restype = ctypes.c_int
        lib.lddl_read_fill.argtypes = [c_vp, c_vp, c_vp, c_vp]
        lib.lddl_read_free.restype = ctypes.c_int
        lib.lddl_read_free.argtypes = [c_vp]
        lib.lddl_read_counts.restype = ctypes.c_int
        lib.lddl_read_counts.argtypes = [c_vp, c_vp, c_vp]
        lib.lddl_read_fill_range.restype = ctypes.c_int
        lib.lddl_read_fill_range.argtypes = [c_vp, c_i64, c_i64, c_vp, c_vp]
        lib.lddl_random_state_data.restype = ctypes.c_int
        lib.lddl_random_state_data.argtypes = [c_i64, ctypes.c_uint64, c_vp]
        lib.lddl_last_error.restype = ctypes.c_char_p

        def check(status):
            if status < 0:
                raise RuntimeError('liblddl_host: ' + (lib.lddl_last_error() or b'').decode())
            return status
        _HOST = (lib, check)
    return _HOST


class NativeRead:
    """One lddl_read_groups call (see read_groups_native) whose documents are copied out a range
    at a time: `block_ndocs` / `doc_len` are known as soon as the blocks are read, split, sampled
    and shuffled, and fill(d0, d1) copies documents [d0, d1) (one GPU batch) while later batches
    stay in the reader. close() frees it."""

    def __init__(self, groups, group_seeds, threads=16):
        import ctypes
        import numpy as np
        self._lib, self._check = lib, check = _host_lib()
        blocks = [b for g in groups for b in g]
        n = len(blocks)
        paths = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(b.path) for b in blocks])
        starts = np.asarray([b.start for b in blocks], np.int64)
        ends = np.asarray([max(b.end, b.start) for b in blocks], np.int64)
        ratios = {b.ratio for b in blocks if b.mt is not None}
        if any(b.mt is None for b in blocks) and ratios:
            raise ValueError('blocks mix sampled and unsampled reads')
        if len(ratios) > 1:
            raise ValueError('blocks with different sample ratios')
        states = None
        if ratios:
            states = np.ascontiguousarray(np.stack([b.mt for b in blocks]), np.uint32)
        goff = np.zeros(len(groups) + 1, np.int64)
        np.cumsum([len(g) for g in groups], out=goff[1:])
        seeds = [abs(int(x)) for x in group_seeds]
        if any(x >= 1 << 64 for x in seeds):
            raise ValueError('shuffle seeds must be below 2**64 in magnitude')
        seeds = np.asarray(seeds, np.uint64)
        self._h = ctypes.c_void_p()
        n_docs, n_text = ctypes.c_int64(), ctypes.c_int64()
        bad = np.zeros(2, np.int64)
        st = lib.lddl_read_groups(n, paths, starts.ctypes.data, ends.ctypes.data,
                                  None if states is None else states.ctypes.data,
                                  float(ratios.pop()) if ratios else 1.0, len(groups),
                                  goff.ctypes.data, seeds.ctypes.data, int(threads),
                                  ctypes.byref(self._h), ctypes.byref(n_docs),
                                  ctypes.byref(n_text), bad.ctypes.data)
        if st == -2:
            b = blocks[int(bad[0])]
            off = b.start + int(bad[1])
            with open(b.path, 'rb') as f:
                f.seek(max(off - 8, b.start))
                ctx = f.read(16)
            raise UnicodeDecodeError('utf-8', ctx, min(8, off - b.start),
                                     min(8, off - b.start) + 1,
                                     'invalid UTF-8 at byte {} of {}'.format(off, b.path))
        check(st)
        self.n_docs, self.n_text = n_docs.value, n_text.value
        self.block_ndocs = np.empty(max(n, 1), np.int64)[:n]
        self.doc_len = np.empty(max(self.n_docs, 1), np.int64)[:self.n_docs]
        check(lib.lddl_read_counts(self._h, self.block_ndocs.ctypes.data,
                                   self.doc_len.ctypes.data))

    def fill(self, d0, d1):
        """(text uint8, doc_off int64[d1 - d0 + 1]) of documents [d0, d1)."""
        import numpy as np
        nb = int(self.doc_len[d0:d1].sum())
        text = np.empty(nb, np.uint8)
        doc_off = np.empty(d1 - d0 + 1, np.int64)
        self._check(self._lib.lddl_read_fill_range(self._h, d0, d1, text.ctypes.data,
                                                    doc_off.ctypes.data))
        return text, doc_off

    def close(self):
        if self._h:
            self._lib.lddl_read_free(self._h)
            self._h = None

    def __del__(self):
        self.close()


def read_groups_native(groups, group_seeds, threads=16):
    """The documents of shuffle groups of blocks, read by the library's host reader
    (lddl_read_groups: C++ threads, no per-line Python): for every group, its blocks' lines as
    read_block(as_bytes=True) gives them, shuffled by random.Random(seed).shuffle over the group
    (pretrain.py:100-111 per group) and dealt back (each block keeps its count), each reduced to the
    text after its id (split_id_text_bytes). Returns (text uint8, doc_off int64[n_docs + 1],
    block_ndocs int64[n_blocks]) in block order. Malformed UTF-8 anywhere in a block raises
    UnicodeDecodeError, as dask's strict decode of the block does."""
    r = NativeRead(groups, group_seeds, threads)
    try:
        text, doc_off = r.fill(0, r.n_docs)
        return text, doc_off, r.block_ndocs
    finally:
        r.close()
