"""Device-resident sample table -> the reference's parquet layout.

Counterparts of the reference's output stage:
  * `_to_dataframe_binned` (lddl/dask/bert/binning.py:63-93) -> `bin_partitions` (HIP kernel
    lddl_bin_partitions: per-partition stable regroup by bin_id = min((n-1)//bin_size, nbins-1));
  * the instance dict of `create_pairs_from_document` (lddl/dask/bert/pretrain.py:345-358) ->
    `render` (HIP kernels lddl_render_lengths / lddl_render_write: ' '.join of vocab strings and
    the np.save bytes of masked_lm_positions, lddl/utils.py:98-102);
  * `_save_parquet` / `write_partition_binned` (pretrain.py:444-498, binning.py:353-431) ->
    `write_parquet` (pyarrow, zero-copy Arrow arrays over the rendered buffers; file names
    `part.<i>.parquet` or `part.<i>.parquet_<b>`, one file per (partition, bin) even if empty).

Everything up to the host copy of the rendered bytes runs on the GPU; pyarrow only frames and
writes the buffers.
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import torch

from ._native import lib, check
from .context import _ptr, _stream

try:  # the reference compresses with snappy iff python-snappy is importable (binning.py:42-47)
    import snappy  # noqa: F401
    DEFAULT_COMPRESSION = 'snappy'
except ImportError:
    DEFAULT_COMPRESSION = None


def bin_partitions(ctx, num_tokens, part_off, bin_size, nbins, tok_off=None):
    """num_tokens: int32 cuda [n] (or None with tok_off: a pair table's int64 [n+1] token
    offsets, num_tokens = len(A) + len(B) + 3); part_off: int64 cuda [n_part+1].
    Returns (perm int64 [n], bin_id int64 [n], counts int64 [n_part, nbins]) on the device."""
    n = num_tokens.numel() if num_tokens is not None else tok_off.numel() - 1
    n_part = part_off.numel() - 1
    dev = part_off.device
    perm = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
    bin_id = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
    counts = torch.empty(max(n_part * nbins, 1), dtype=torch.int64, device=dev)[:n_part * nbins]
    check(lib.lddl_bin_partitions(ctx.handle, _stream(), _ptr(num_tokens), _ptr(tok_off), n,
                                  _ptr(part_off), n_part, bin_size, nbins, _ptr(perm),
                                  _ptr(bin_id), _ptr(counts)))
    return perm, bin_id, counts.view(n_part, nbins)


def bin_stable(ctx, num_tokens=None, bin_size=8, nbins=1, tok_off=None, with_bin_id=True):
    """One segment (all rows): (perm, bin_id or None, counts[nbins]) — the tiled multi-workgroup
    regroup used before the load-balance exchange. Rows are given by num_tokens (int32 cuda) or
    by a pair table's tok_off (num_tokens = len(A) + len(B) + 3)."""
    n = num_tokens.numel() if num_tokens is not None else tok_off.numel() - 1
    dev = ctx.device
    perm = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
    bin_id = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n] if with_bin_id else None
    counts = torch.empty(nbins, dtype=torch.int64, device=dev)
    check(lib.lddl_bin_stable(ctx.handle, _stream(), _ptr(num_tokens), _ptr(tok_off), n, bin_size,
                              nbins, _ptr(perm), _ptr(bin_id), _ptr(counts)))
    return perm, bin_id, counts


def scan(ctx, x):
    """Exclusive prefix sum of int64 cuda x -> int64[n + 1] (HIP, lddl_scan_i64)."""
    out = torch.empty(x.numel() + 1, dtype=torch.int64, device=x.device)
    check(lib.lddl_scan_i64(ctx.handle, _stream(), _ptr(x), x.numel(), _ptr(out)))
    return out


@dataclass
class Rendered:
    """Host buffers of the parquet columns of rows 0..n-1 (offsets are int64, global)."""
    a_off: np.ndarray
    a_bytes: np.ndarray
    b_off: np.ndarray
    b_bytes: np.ndarray
    is_random_next: np.ndarray
    num_tokens: np.ndarray
    l_off: np.ndarray = None
    l_bytes: np.ndarray = None
    npy_off: np.ndarray = None
    npy_bytes: np.ndarray = None
    bin_id: np.ndarray = None

    @property
    def n(self):
        return len(self.num_tokens)

    def row(self, r):
        """Python dict of row r, as the reference's instance (for tests / txt output)."""
        d = {'A': bytes(self.a_bytes[self.a_off[r]:self.a_off[r + 1]]).decode('utf-8'),
             'B': bytes(self.b_bytes[self.b_off[r]:self.b_off[r + 1]]).decode('utf-8'),
             'is_random_next': bool(self.is_random_next[r]),
             'num_tokens': int(self.num_tokens[r])}
        if self.l_off is not None:
            d['masked_lm_positions'] = bytes(self.npy_bytes[self.npy_off[r]:self.npy_off[r + 1]])
            d['masked_lm_labels'] = bytes(self.l_bytes[self.l_off[r]:self.l_off[r + 1]]).decode(
                'utf-8')
        if self.bin_id is not None:
            d['bin_id'] = int(self.bin_id[r])
        return d


def render(ctx, pb, rows=None, bin_id=None):
    """Render the parquet columns of PairBatch `pb` for output rows `rows` (int64 cuda tensor of
    pair indices, None = all pairs in order). Returns a host `Rendered`."""
    return render_device(ctx, pb, rows, bin_id).to_host()


@dataclass
class DeviceRendered:
    """render()'s columns still in HBM (device tensors), with the stream event after which they
    are complete: to_host() copies them to pinned host memory on a stream of its own, so the
    copy of one batch overlaps the GPU work of the next (any thread may call it)."""
    cols: dict
    tot: list
    masking: bool
    event: object = None

    @property
    def nbytes(self):
        """Host bytes to_host() pins for this batch."""
        return sum(t.numel() * t.element_size() for t in (self.cols or {}).values() if t is not None)

    def to_host(self, stream=None):
        st = stream if stream is not None else torch.cuda.current_stream()
        if self.event is not None:
            st.wait_event(self.event)
        out = {}
        with torch.cuda.stream(st):
            for k, t in self.cols.items():
                if t is None:
                    out[k] = None
                    continue
                if _PAGEABLE:  # (A/B diagnostics) pageable host buffers
                    h = torch.empty(max(t.numel(), 1), dtype=t.dtype)[:t.numel()]
                    h.copy_(t)
                else:
                    h = torch.empty(max(t.numel(), 1), dtype=t.dtype, pin_memory=True)[:t.numel()]
                    h.copy_(t, non_blocking=True)
                t.record_stream(st)
                out[k] = h
        st.synchronize()
        n = {k: (v.numpy() if v is not None else None) for k, v in out.items()}
        rd = Rendered(n['a_off'], n['a_bytes'], n['b_off'], n['b_bytes'],
                      n['is_rn'].astype(bool), n['num_tokens'].view(np.uint16))
        if self.masking:
            rd.l_off, rd.l_bytes = n['l_off'], n['l_bytes']
            rd.npy_off, rd.npy_bytes = n['npy_off'], n['npy_bytes']
        if n.get('bin_id') is not None:
            rd.bin_id = n['bin_id'].astype(np.int64)
        self.cols = None
        return rd

    _ROW_COLS = ('a_off', 'b_off', 'l_off', 'npy_off', 'is_rn', 'num_tokens', 'bin_id')
    _BYTE_COLS = (('a_off', 'a_bytes'), ('b_off', 'b_bytes'), ('l_off', 'l_bytes'),
                  ('npy_off', 'npy_bytes'))

    def to_host_chunks(self, part_rows, chunk_bytes, stream=None):
        """to_host() in pieces: the per-row columns once, then the string columns of consecutive
        partition groups of about `chunk_bytes` each, yielded as (p0, p1, Rendered) with the
        batch's global row numbers and offsets (the byte columns are addressed through
        `_Shifted`). A pinned allocation holds up every concurrent pageable host copy of the
        process for its whole duration (tools/d2h_probe.py: a 512 MiB H2D 0.010 s alone, 0.18-0.29
        s beside a 4 GiB allocation), so one allocation per batch stalled the next batch's
        pageable copies for ~0.2-0.3 s; chunks bound each stall to a few ms, and the blocks that
        their writes release come back from torch's host cache for the later chunks."""
        st = stream if stream is not None else torch.cuda.current_stream()
        if self.event is not None:
            st.wait_event(self.event)
        cols = self.cols
        host = {}
        with torch.cuda.stream(st):
            for k in self._ROW_COLS:
                t = cols.get(k)
                if t is None:
                    continue
                h = torch.empty(max(t.numel(), 1), dtype=t.dtype, pin_memory=True)[:t.numel()]
                h.copy_(t, non_blocking=True)
                t.record_stream(st)
                host[k] = h
        st.synchronize()
        n = {k: v.numpy() for k, v in host.items()}
        bin_id = n['bin_id'].astype(np.int64) if 'bin_id' in n else None
        byte_cols = [(ok, bk) for ok, bk in self._BYTE_COLS if cols.get(bk) is not None]
        for p0, p1 in chunk_groups(part_rows, [n[ok] for ok, _ in byte_cols], chunk_bytes):
            r0, r1 = int(part_rows[p0]), int(part_rows[p1])
            chunk = {}
            with torch.cuda.stream(st):
                for ok, bk in byte_cols:
                    b0, b1 = int(n[ok][r0]), int(n[ok][r1])
                    t = cols[bk]
                    h = torch.empty(max(b1 - b0, 1), dtype=t.dtype, pin_memory=True)[:b1 - b0]
                    if b1 > b0:
                        h.copy_(t[b0:b1], non_blocking=True)
                    chunk[bk] = _Shifted(h.numpy(), b0)
            st.synchronize()
            rd = Rendered(n['a_off'], chunk['a_bytes'], n['b_off'], chunk['b_bytes'],
                          n['is_rn'].view(bool), n['num_tokens'].view(np.uint16))
            if self.masking:
                rd.l_off, rd.l_bytes = n['l_off'], chunk['l_bytes']
                rd.npy_off, rd.npy_bytes = n['npy_off'], chunk['npy_bytes']
            if bin_id is not None:
                rd.bin_id = bin_id
            yield p0, p1, rd
        for _, bk in byte_cols:
            cols[bk].record_stream(st)
        self.cols = None


def chunk_groups(part_rows, offsets, chunk_bytes):
    """Consecutive partition groups [p0, p1) for DeviceRendered.to_host_chunks: each group adds
    partitions while its bytes (summed over the byte columns, whose row offsets are `offsets`)
    stay <= chunk_bytes; a group holds at least one partition."""
    n_part = len(part_rows) - 1
    out, p0 = [], 0
    while p0 < n_part:
        def span(q):
            r0, r1 = int(part_rows[p0]), int(part_rows[q])
            return sum(int(o[r1]) - int(o[r0]) for o in offsets)
        p1 = p0 + 1
        while p1 < n_part and span(p1 + 1) <= chunk_bytes:
            p1 += 1
        out.append((p0, p1))
        p0 = p1
    return out


class _Shifted:
    """A string column's host bytes [base, base + len) addressed with the batch's global byte
    offsets (what `_var` and `Rendered.row` slice)."""
    __slots__ = ('a', 'base')

    def __init__(self, a, base):
        self.a, self.base = a, base

    def __getitem__(self, s):
        return self.a[s.start - self.base:s.stop - self.base]


def render_device(ctx, pb, rows=None, bin_id=None):
    """The GPU half of render(): kernels only (one host sync for the byte totals)."""
    dev = ctx.device
    n = pb.n_pairs if rows is None else rows.numel()
    masking = pb.pos is not None
    if pb.tokens.element_size() != ctx.id_bytes or (masking and pb.labels.element_size() != ctx.id_bytes):
        raise ValueError('pair table ids are {}-byte, the context renders {}-byte ids'.format(
            pb.tokens.element_size(), ctx.id_bytes))
    st = _stream()
    a_len = torch.empty(max(n, 1), dtype=torch.int64, device=dev)[:n]
    b_len = torch.empty_like(a_len)
    l_len = torch.empty_like(a_len) if masking else None
    npy_len = torch.empty_like(a_len) if masking else None
    lab = pb.labels if masking else None
    pos_off = pb.pos_off if masking else None
    num_tokens = torch.empty(max(n, 1), dtype=torch.int16, device=dev)[:n]  # uint16 storage
    is_rn = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)[:n]
    check(lib.lddl_render_lengths(ctx.handle, st, _ptr(pb.tokens), _ptr(pb.tok_off), _ptr(pb.len_a),
                                  _ptr(lab), _ptr(pos_off), _ptr(rows), n, _ptr(a_len), _ptr(b_len),
                                  _ptr(l_len), _ptr(npy_len), _ptr(pb.is_random_next),
                                  _ptr(num_tokens), _ptr(is_rn)))
    a_off, b_off = scan(ctx, a_len), scan(ctx, b_len)
    l_off = scan(ctx, l_len) if masking else None
    npy_off = scan(ctx, npy_len) if masking else None
    tot = [int(x[-1].item()) if x is not None else 0 for x in (a_off, b_off, l_off, npy_off)]
    bufs = [torch.empty(max(t, 1), dtype=torch.uint8, device=dev) for t in tot]
    check(lib.lddl_render_write(ctx.handle, st, _ptr(pb.tokens), _ptr(pb.tok_off), _ptr(pb.len_a),
                                _ptr(pb.pos) if masking else None, _ptr(lab), _ptr(pos_off),
                                _ptr(rows), n, _ptr(a_off), _ptr(b_off), _ptr(l_off),
                                _ptr(npy_off), _ptr(bufs[0]), _ptr(bufs[1]),
                                _ptr(bufs[2]) if masking else None,
                                _ptr(bufs[3]) if masking else None))

    cols = {'a_off': a_off, 'a_bytes': bufs[0][:tot[0]], 'b_off': b_off,
            'b_bytes': bufs[1][:tot[1]], 'is_rn': is_rn, 'num_tokens': num_tokens}
    if masking:
        cols.update(l_off=l_off, l_bytes=bufs[2][:tot[2]], npy_off=npy_off,
                    npy_bytes=bufs[3][:tot[3]])
    if bin_id is not None:  # a device tensor (or host int64[n])
        cols['bin_id'] = bin_id if torch.is_tensor(bin_id) else torch.from_numpy(
            np.asarray(bin_id, np.int64)).to(dev)
    ev = torch.cuda.Event()
    ev.record()
    return DeviceRendered(cols, tot, masking, ev)


def schema(masking, binned):
    """The reference's parquet schema (pretrain.py:450-468, + bin_id int64 when binned, 496)."""
    fields = [('A', pa.string()), ('B', pa.string()), ('is_random_next', pa.bool_()),
              ('num_tokens', pa.uint16())]
    if masking:
        fields += [('masked_lm_positions', pa.binary()), ('masked_lm_labels', pa.string())]
    if binned:
        fields.append(('bin_id', pa.int64()))
    return pa.schema(fields)


def _var(typ, off, data, r0, r1):
    o = off[r0:r1 + 1]
    b0, b1 = int(o[0]), int(o[-1])
    if b1 - b0 >= (1 << 31):
        raise ValueError('a parquet file would hold >= 2 GiB in one string column; use more '
                         'partitions (--num-blocks / --block-size)')
    rel = (o - b0).astype(np.int32)
    return pa.Array.from_buffers(typ, r1 - r0, [None, pa.py_buffer(rel),
                                                pa.py_buffer(data[b0:b1])])


def table(rd, r0, r1, masking, binned):
    cols = [_var(pa.string(), rd.a_off, rd.a_bytes, r0, r1),
            _var(pa.string(), rd.b_off, rd.b_bytes, r0, r1),
            pa.array(rd.is_random_next[r0:r1], pa.bool_()),
            pa.array(rd.num_tokens[r0:r1], pa.uint16())]
    if masking:
        cols += [_var(pa.binary(), rd.npy_off, rd.npy_bytes, r0, r1),
                 _var(pa.string(), rd.l_off, rd.l_bytes, r0, r1)]
    if binned:
        cols.append(pa.array(rd.bin_id[r0:r1], pa.int64()))
    return pa.Table.from_arrays(cols, schema=schema(masking, binned))


_TRACE = os.environ.get('LDDL_TRACE_PIPELINE')
_PAGEABLE = os.environ.get('LDDL_D2H_PAGEABLE')


def write_table(rd, r0, r1, masking, binned, path, compression=DEFAULT_COMPRESSION):
    """Rows [r0, r1) of a Rendered as one parquet file."""
    if _TRACE:
        import sys
        import time
        t0 = time.perf_counter()
    pq.write_table(table(rd, r0, r1, masking, binned), path, compression=compression)
    if _TRACE:
        sys.stderr.write('[write] %s %.1f MB %.2f ms at %.3f\n' % (
            os.path.basename(path), (rd.a_off[r1] - rd.a_off[r0]) * 2e-6,
            (time.perf_counter() - t0) * 1e3, time.perf_counter()))
    return path


def write_dataset_metadata(outdir, n_part, nbins=None):
    """dask's `_common_metadata` (schema) and `_metadata` (row groups of every partition, in
    partition order, file path `part.<i>.parquet`) next to the part files — ArrowDatasetEngine
    .write_metadata (dask 2021.10, dataframe/io/parquet/arrow.py:712-735) as driven by
    `to_parquet` (pretrain.py:473-478) and `to_parquet_binned` (binning.py:325-339). Binned, each
    partition contributes its LAST bin file's row groups under the unsuffixed name, which is
    what write_partition_binned hands back (binning.py:378-421: `_meta` is overwritten per bin
    and `set_file_path(filename)`)."""
    meta = None
    schema = None
    for p in range(n_part):
        name = 'part.{}.parquet'.format(p)
        fn = os.path.join(outdir, name if nbins is None else '{}_{}'.format(name, nbins - 1))
        md = pq.read_metadata(fn)
        md.set_file_path(name)
        if meta is None:
            meta, schema = md, pq.read_schema(fn)
        else:
            meta.append_row_groups(md)
    if meta is None:
        return None
    pq.write_metadata(schema, os.path.join(outdir, '_common_metadata'))
    meta.write_metadata_file(os.path.join(outdir, '_metadata'))
    return os.path.join(outdir, '_metadata')


def write_parquet(outdir, rd, part_rows, part_index, masking, nbins=None, bin_counts=None,
                  compression=DEFAULT_COMPRESSION, executor=None, futures=None):
    """Write the reference's files for a group of partitions.

    part_rows: int64 [n_part + 1] row ranges of the partitions inside `rd`; part_index: global
    partition number of each (file name part.<i>.parquet); when binned, bin_counts[p, b] are the
    rows of (p, b), laid out bin after bin inside the partition's range. With an `executor`
    (threads: pyarrow encodes and writes without the GIL) the files are written concurrently and
    the futures appended to `futures`; the caller waits for them."""
    paths = []

    def put(r0, r1, binned, fn):
        if executor is None:
            write_table(rd, r0, r1, masking, binned, fn, compression)
        else:
            futures.append(executor.submit(write_table, rd, r0, r1, masking, binned, fn,
                                           compression))
        paths.append(fn)
    for p in range(len(part_rows) - 1):
        r0, r1 = int(part_rows[p]), int(part_rows[p + 1])
        name = os.path.join(outdir, 'part.{}.parquet'.format(part_index[p]))
        if nbins is None:
            put(r0, r1, False, name)
            continue
        b0 = r0
        for b in range(nbins):
            b1 = b0 + int(bin_counts[p, b])
            put(b0, b1, True, '{}_{}'.format(name, b))
            b0 = b1
        assert b0 == r1
    return paths
