"""The C-ABI library loads without a GPU and exports every entry point include/*.h declares."""
import ctypes
import glob
import os
import re

from conftest import REPO


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, 'include', '*.h')):
        src = open(h).read()
        src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
        for m in re.finditer(r'^[A-Za-z_][\w\s\*]*?\b(lddl_\w+)\s*\(', src, flags=re.M):
            names.add(m.group(1))
    return names


def test_header_declares_functions():
    names = declared_functions()
    assert {'lddl_ctx_create', 'lddl_tokenize', 'lddl_pairs_plan'} <= names


def test_library_exports_every_declared_symbol():
    from lddl_amd import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [n for n in sorted(declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    from lddl_amd import _native
    assert declared_functions() == set(_native.SIGNATURES)


def test_last_error_and_version():
    from lddl_amd._native import lib
    assert lib.lddl_version() >= 1
    assert isinstance(lib.lddl_last_error(), bytes)


def test_synth_deterministic_across_threads():
    from lddl_amd import synth
    a = synth.generate(seed=7, n_bytes=300_000, threads=1)
    b = synth.generate(seed=7, n_bytes=300_000, threads=5)
    assert (a.text == b.text).all() and (a.sent_off == b.sent_off).all()
    assert (a.doc_sent_off == b.doc_sent_off).all()
    c = synth.generate(seed=8, n_bytes=300_000, threads=1)
    assert len(c.text) != len(a.text) or (c.text != a.text).any()


def test_build_id_matches_sources():
    """lddl_build_id() of the loaded library is the hash of the sources in this tree (the
    library is current; bench lines and PMC passes name their build by it)."""
    from lddl_amd import build
    from lddl_amd._native import lib
    assert lib.lddl_build_id().decode() == build.source_id()
