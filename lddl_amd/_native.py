"""ctypes binding of include/lddl_amd.h (the C ABI of lddl_amd/_lib/liblddl_amd.so).

There is no fallback: if the library is missing the import fails loudly. Build it with
`python -m lddl_amd.build` (or `__graft_entry__.build()`).
"""
import ctypes
import os

# torch first: its HIP runtime (torch/lib/libamdhip64.so, soname libamdhip64.so.7) must be the
# process's one runtime. Loaded the other way round, liblddl_amd.so would bring in
# /opt/rocm/lib/libamdhip64.so.7 and torch (which asks for "libamdhip64.so") a second copy, and
# the two HIP runtimes do not share devices ("no ROCm-capable device is detected").
import torch  # noqa: F401,E402

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('LDDL_AMD_LIB') or os.path.join(_HERE, '_lib', 'liblddl_amd.so')

c_i64, c_u64, c_i32, c_u32, c_dbl, c_vp = (ctypes.c_int64, ctypes.c_uint64, ctypes.c_int32,
                                           ctypes.c_uint32, ctypes.c_double, ctypes.c_void_p)
c_i64p = ctypes.POINTER(ctypes.c_int64)

# name -> (restype, argtypes); must mirror include/lddl_amd.h exactly
SIGNATURES = {
    'lddl_last_error': (ctypes.c_char_p, []),
    'lddl_build_id': (ctypes.c_char_p, []),
    'lddl_version': (ctypes.c_int, []),
    'lddl_synth_corpus': (c_i64, [c_u64, c_i64, c_i64, c_dbl, c_vp, c_i64, c_vp, c_i64, c_vp, c_i64,
                                  c_i64p, c_i64p, ctypes.c_int]),
    'lddl_read_groups': (ctypes.c_int, [c_i64, c_vp, c_vp, c_vp, c_vp, c_dbl, c_i64, c_vp, c_vp,
                                        ctypes.c_int, ctypes.POINTER(c_vp), c_i64p, c_i64p, c_vp]),
    'lddl_read_fill': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    'lddl_read_free': (ctypes.c_int, [c_vp]),
    'lddl_read_counts': (ctypes.c_int, [c_vp, c_vp, c_vp]),
    'lddl_read_fill_range': (ctypes.c_int, [c_vp, c_i64, c_i64, c_vp, c_vp]),
    'lddl_random_state_data': (ctypes.c_int, [c_i64, c_u64, c_vp]),
    'lddl_ctx_create': (ctypes.c_int, [ctypes.c_int, c_vp, c_i64, c_vp, c_i64,
                                       ctypes.POINTER(c_vp)]),
    'lddl_ctx_destroy': (ctypes.c_int, [c_vp]),
    'lddl_ctx_info': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    'lddl_ctx_id_bytes': (ctypes.c_int, [c_vp]),
    'lddl_ctx_render_table': (ctypes.c_int, [c_vp, ctypes.POINTER(c_vp), ctypes.POINTER(c_vp)]),
    'lddl_synth_doc_text': (c_i64, [c_u64, c_i64, c_i64, c_dbl, c_vp, c_i64, c_vp, c_i64, c_vp,
                                    ctypes.c_int]),
    'lddl_punkt_set_params': (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_i64]),
    'lddl_segment_count': (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_i64,
                                          ctypes.POINTER(c_i64)]),
    'lddl_segment_fill': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    'lddl_tokenize': (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_vp, c_vp]),
    'lddl_pairs_plan': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_vp,
                                       c_vp, c_i64, ctypes.POINTER(c_vp), c_vp]),
    'lddl_pairs_emit': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'lddl_pairs_destroy': (ctypes.c_int, [c_vp, c_vp]),
    'lddl_pairs_part_offsets': (ctypes.c_int, [c_vp, c_vp, c_vp]),
    'lddl_pairs_plan_ms': (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_float)]),
    'lddl_bin_partitions': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_vp, c_i64, c_i32, c_i32,
                                           c_vp, c_vp, c_vp]),
    'lddl_bin_stable': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i32, c_i32, c_vp, c_vp,
                                       c_vp]),
    'lddl_render_lengths': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'lddl_render_write': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                         c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    'lddl_scan_i64': (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp]),
    'lddl_gather_ragged': (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i32, c_vp, c_i64,
                                          c_vp, c_vp]),
    'lddl_take': (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_i32, c_vp, c_i64, c_vp]),
    'lddl_ragged_offsets': (ctypes.c_int, [c_vp, c_vp, c_vp, c_i64, c_vp, c_vp, c_i64, c_vp]),
    'lddl_expand_segments': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, c_vp]),
    'lddl_pairs_meta_pack': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_vp]),
    'lddl_pairs_meta_unpack': (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp]),
    'lddl_ctx_set_allocator': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp]),
    'lddl_collate_encode': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32,
                                           c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                           c_i64]),
    'lddl_utf8_check': (ctypes.c_int, [c_vp, c_vp, c_i64, c_vp]),
    'lddl_collate_encode_masked': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32,
                                                  c_i32, c_vp, c_vp, c_vp, c_vp, ctypes.c_float,
                                                  c_i64, c_i64, c_u64, c_u64]),
    'lddl_mask_dynamic': (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64,
                                         ctypes.c_float, c_i64, c_i64, c_u64, c_u64, c_vp, c_vp,
                                         c_vp, c_vp]),
}


class PairParams(ctypes.Structure):
    """lddl_pair_params (include/lddl_amd.h)."""
    _fields_ = [('seq', ctypes.c_int32), ('dup', ctypes.c_int32), ('masking', ctypes.c_int32),
                ('rng', ctypes.c_int32), ('short_seq_prob', ctypes.c_double),
                ('masked_lm_ratio', ctypes.c_double), ('native_seed', ctypes.c_uint64)]


RNG_REPLAY, RNG_NATIVE = 0, 1


class NativeError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError('lddl_amd native library not built: {} is missing (run `python -m '
                          'lddl_amd.build`). There is no CPU fallback.'.format(LIB_PATH))
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(status):
    """Raise NativeError with the library's thread-local message on a negative status."""
    if status < 0:
        msg = lib.lddl_last_error()
        raise NativeError((msg or b'unknown error').decode())
    return status
