"""In-tree build of the native pieces.

* lddl_amd/_lib/liblddl_amd.so : the product — HIP kernels for gfx950 + C-ABI host code
  (hipcc --offload-arch=gfx950). Cross-compiles without a GPU.
* oracle/_build/liblddl_oracle.so : the CPU restatement used only by tests / bench's cpu_baseline
  (plain gcc, no HIP).

Both are incremental (per-source object files, rebuilt when the source or any header is newer).
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'lddl_amd', 'csrc')
LIBDIR = os.path.join(ROOT, 'lddl_amd', '_lib')
OBJDIR = os.path.join(ROOT, 'build', 'obj')
LIB = os.path.join(LIBDIR, 'liblddl_amd.so')
ORACLE_DIR = os.path.join(ROOT, 'oracle')
ORACLE_LIB = os.path.join(ORACLE_DIR, '_build', 'liblddl_oracle.so')

HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = 'gfx950'


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError('build failed: ' + ' '.join(cmd))
    return r.stdout


BUILD_ID_H = os.path.join(CSRC, 'build_id.h')


def source_id():
    """First 16 hex digits of SHA-256 over the library's sources (csrc/ and include/, names and
    contents, build_id.h itself excluded): the id lddl_build_id() returns."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, '*')) + glob.glob(os.path.join(ROOT, 'include', '*.h')))
    for f in files:
        if os.path.isfile(f) and f != BUILD_ID_H and f.endswith(('.hip', '.cpp', '.h')):
            h.update(os.path.relpath(f, ROOT).encode() + b'\0')
            with open(f, 'rb') as fh:
                h.update(fh.read())
    return h.hexdigest()[:16]


def write_build_id():
    """csrc/build_id.h (generated, not tracked), rewritten only when the id changes so that an
    unchanged tree rebuilds nothing."""
    text = '#pragma once\n#define LDDL_BUILD_ID "{}"\n'.format(source_id())
    try:
        with open(BUILD_ID_H) as f:
            if f.read() == text:
                return
    except OSError:
        pass
    with open(BUILD_ID_H, 'w') as f:
        f.write(text)


def build_product(verbose=False, jobs=8, diag=False, variant=None, defines=()):
    """diag=True builds the stamp-instrumented diagnostic library into lddl_amd/_lib_diag
    (timing shares only; never the shipped library). variant/defines build an experiment library
    into lddl_amd/_lib_<variant> with extra -D flags (A/B measurements only)."""
    write_build_id()
    suffix = '_diag' if diag else ('_' + variant if variant else '')
    libdir = LIBDIR + suffix
    objdir = OBJDIR + suffix
    lib = os.path.join(libdir, 'liblddl_amd.so')
    os.makedirs(libdir, exist_ok=True)
    os.makedirs(objdir, exist_ok=True)
    headers = glob.glob(os.path.join(ROOT, 'include', '*.h')) + glob.glob(os.path.join(CSRC, '*.h'))
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')) + glob.glob(os.path.join(CSRC, '*.cpp')))
    flags = ['-O3', '-std=c++17', '-fPIC', '-Wall', '-Wno-unused-function',
             '-I' + os.path.join(ROOT, 'include'), '-I' + CSRC] + (['-DLDDL_STAMPS'] if diag else []) + \
        ['-D' + d for d in defines] + os.environ.get('LDDL_EXTRA_FLAGS', '').split()
    # a library built with anything but the product flags (diagnostic stamps, variant defines,
    # LDDL_EXTRA_FLAGS) reports lddl_build_id() = source id + '-' + a hash of those flags, so a
    # PMC pass of such a build never passes for the product's
    import hashlib
    extra = flags[flags.index('-I' + CSRC) + 1:]
    if extra:
        fid = hashlib.sha256(' '.join(extra).encode()).hexdigest()[:8]
        flags = flags + ['-DLDDL_BUILD_VARIANT="-{}"'.format(fid)]
    # the objects of a directory are rebuilt whenever its compile flags change
    stamp = os.path.join(objdir, '.flags')
    force = not os.path.exists(stamp) or open(stamp).read() != ' '.join(flags)
    objs, jobs_list = [], []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + '.o')
        objs.append(o)
        if force or _newer(o, [s] + headers):
            if s.endswith('.hip'):
                cmd = [HIPCC, '--offload-arch=' + ARCH, '-x', 'hip'] + flags + ['-c', s, '-o', o]
            else:
                cmd = [HIPCC, '-x', 'c++'] + flags + ['-D__HIP_PLATFORM_AMD__', '-c', s, '-o', o]
            jobs_list.append(cmd)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out:
                print(out)
    with open(stamp, 'w') as f:
        f.write(' '.join(flags))
    if _newer(lib, objs):
        _run([HIPCC, '-shared', '-fPIC', '--offload-arch=' + ARCH, '-o', lib] + objs +
             ['-lpthread'])
    return lib


HOST_LIB = os.path.join(LIBDIR, 'liblddl_host.so')
HOST_SRCS = ('reader.cpp', 'errors.cpp')


def build_host():
    """lddl_amd/_lib/liblddl_host.so: the host-only entry points (the input reader) without the
    HIP runtime, so the CLI's reader thread can load it while the main thread is still importing
    torch (liblddl_amd.so must be loaded after torch: one HIP runtime per process). The same
    sources are also part of liblddl_amd.so."""
    os.makedirs(LIBDIR, exist_ok=True)
    write_build_id()
    srcs = [os.path.join(CSRC, x) for x in HOST_SRCS]
    deps = srcs + glob.glob(os.path.join(ROOT, 'include', '*.h')) + [os.path.join(CSRC, 'common.h'), BUILD_ID_H]
    if _newer(HOST_LIB, deps):
        _run(['g++', '-O3', '-std=c++17', '-fPIC', '-shared', '-Wall', '-I' + os.path.join(ROOT, 'include'),
              '-I' + CSRC, '-o', HOST_LIB] + srcs + ['-lpthread'])
    return HOST_LIB


def build_oracle():
    os.makedirs(os.path.dirname(ORACLE_LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(ORACLE_DIR, '*.c')))
    deps = srcs + glob.glob(os.path.join(ORACLE_DIR, '*.h'))
    if srcs and _newer(ORACLE_LIB, deps):
        _run(['gcc', '-O2', '-std=c11', '-fPIC', '-shared', '-Wall', '-o', ORACLE_LIB] + srcs +
             ['-lm'])
    return ORACLE_LIB


def build_all(verbose=False):
    lib = build_product(verbose=verbose)
    build_host()
    orc = build_oracle()
    return lib, orc


if __name__ == '__main__':
    if '--diag' in sys.argv:
        print(build_product(verbose=True, diag=True))
    elif '--variant' in sys.argv:  # python -m lddl_amd.build --variant NAME DEF=VAL ...
        i = sys.argv.index('--variant')
        print(build_product(verbose=True, variant=sys.argv[i + 1], defines=sys.argv[i + 2:]))
    else:
        print(build_all(verbose=True))
