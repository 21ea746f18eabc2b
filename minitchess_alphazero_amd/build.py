"""Build libmtaz.so (HIP for gfx950) in-tree with hipcc.

Translation units: csrc/mtaz_device.hip (tree kernels + launchers), csrc/mtaz_net16.hip and
csrc/mtaz_net8.hip (network kernels k_net_y, k_net_z), csrc/mtaz_host.cpp (C ABI, numpy-legacy
RNG compiled with -ffp-contract=off, engine driver) and csrc/mtaz_wire.cpp (episode wire
format).  The shared object lands next to this file so it travels to the GPU box with the repo
snapshot.  build(diag=True) makes libmtaz_diag.so with -DMTAZ_NET_DIAG: the network kernels'
A/B and timing-only variants and round 3's k_net_y (csrc/mtaz_net16_r3.hip, variant 3; the
round-3 comparison tests load it in a child process), never loaded by the product path.

Build fingerprint: source_hash() is the sha256 of every file under csrc/, include/mtaz.h and the
compile commands below.  It is compiled into the library (mtaz_version() ends in "src=<hash>"),
build() rebuilds whenever the library does not carry the tree's hash (content, not mtimes), and
_lib.lib() refuses a library whose hash differs from the sources next to it.
"""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, 'csrc')
OUT = os.path.join(HERE, 'libmtaz.so')
BUILD = os.path.join(HERE, '_build')
OUT_DIAG = os.path.join(HERE, 'libmtaz_diag.so')
BUILD_DIAG = os.path.join(HERE, '_build_diag')
INCLUDE = os.path.join(os.path.dirname(HERE), 'include')
ARCH = os.environ.get('MTAZ_OFFLOAD_ARCH', 'gfx950')

SOURCES = [
    ('mtaz_device.hip', ['-O3']),
    # the network kernels' K loops are unrolled by pragma; above LLVM's default pragma threshold
    # (16K) the tail instantiations (fewer boards) were left rolled, and their accumulator arrays
    # went to scratch (round 3: k_net_y<., ., 3> 14x slower)
    ('mtaz_net16.hip', ['-O3', '-mllvm', '-pragma-unroll-threshold=1000000']),
    # round 3's k_net_y (f16x3 variant 3): a bit-identity and batch-dependence reference only, so it
    # is compiled into the diagnostic library alone
    ('mtaz_net16_r3.hip', ['-O3', '-mllvm', '-pragma-unroll-threshold=1000000', 'DIAG_ONLY']),
    ('mtaz_net8.hip', ['-O3', '-mllvm', '-pragma-unroll-threshold=1000000']),
    # numpy's legacy RNG on the device (k_noise, k_choose; glibc's log/pow ported in glibc_math.h,
    # every FMA explicit, no contraction)
    ('mtaz_rng.hip', ['-O3', '-ffp-contract=off', '-fno-fast-math']),
    ('mtaz_host.cpp', ['-O2', '-ffp-contract=off', '-fno-fast-math']),
    ('mtaz_wire.cpp', ['-O2']),
]
HEADERS = ['rules.h', 'engine.h', 'net_common.h', 'glibc_math.h', 'glibc_math_tables.h']


def _hipcc():
    for c in ('/opt/rocm/bin/hipcc', 'hipcc'):
        if os.path.exists(c) or c == 'hipcc':
            return c


def source_hash():
    """sha256 over the library's sources (every file in csrc/, include/mtaz.h) and compile flags."""
    h = hashlib.sha256()
    files = sorted(os.listdir(CSRC))
    for name in files:
        path = os.path.join(CSRC, name)
        if os.path.isfile(path):
            h.update(b'csrc/' + name.encode() + b'\0')
            with open(path, 'rb') as f:
                h.update(f.read())
    with open(os.path.join(INCLUDE, 'mtaz.h'), 'rb') as f:
        h.update(b'include/mtaz.h\0' + f.read())
    h.update(repr((SOURCES, ARCH)).encode())
    return h.hexdigest()


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _tu_key(src, cmd):
    """sha256 of one translation unit's inputs: its source, every header under csrc/, include/mtaz.h
    and the compile command."""
    h = hashlib.sha256(repr(cmd).encode())
    names = [src] + sorted(n for n in os.listdir(CSRC) if n.endswith('.h'))
    for name in names:
        with open(os.path.join(CSRC, name), 'rb') as f:
            h.update(name.encode() + b'\0' + f.read())
    with open(os.path.join(INCLUDE, 'mtaz.h'), 'rb') as f:
        h.update(f.read())
    return h.hexdigest()


def embedded_hash(path):
    """The src=<hash> a built library carries (None if absent)."""
    try:
        with open(path, 'rb') as f:
            data = f.read()
    except OSError:
        return None
    i = data.find(b'mtaz-src-sha256=')
    return data[i + 16:i + 80].decode('ascii', 'replace') if i >= 0 else None


def _stale(out):
    return embedded_hash(out) != source_hash()


def build(force=False, verbose=True, diag=False):
    out, bdir = (OUT_DIAG, BUILD_DIAG) if diag else (OUT, BUILD)
    if not force and not _stale(out):
        return out
    os.makedirs(bdir, exist_ok=True)
    hipcc = _hipcc()
    sha = source_hash()
    objs = []
    procs = []
    for src, flags in SOURCES:
        if 'DIAG_ONLY' in flags:
            if not diag:
                continue
            flags = [f for f in flags if f != 'DIAG_ONLY']
        obj = os.path.join(bdir, src + '.o')
        cmd = [hipcc, '-x', 'hip', '-std=c++17', f'--offload-arch={ARCH}', '-fPIC', '-c',
               os.path.join(CSRC, src), '-o', obj, f'-I{INCLUDE}', '-Wall', '-Wno-unused-function'] + flags
        if src == 'mtaz_host.cpp':   # mtaz_version() carries the whole tree's hash
            cmd.append(f'-DMTAZ_SRC_SHA256="{sha}"')
        if diag:
            cmd.append('-DMTAZ_NET_DIAG')
        objs.append(obj)
        # an object is reused when its source, every header of csrc/ and include/mtaz.h, and its
        # compile command are unchanged (the network TUs take minutes)
        key = _tu_key(src, cmd)
        if not force and os.path.exists(obj) and _read(obj + '.key') == key:
            continue
        if verbose:
            print(' '.join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), cmd, obj, key))
    for p, cmd, obj, key in procs:
        if p.wait() != 0:
            raise RuntimeError('hipcc failed: ' + ' '.join(cmd))
        with open(obj + '.key', 'w') as f:
            f.write(key)
    tmp = out + '.tmp'
    cmd = [hipcc, '-shared', f'--offload-arch={ARCH}', '-o', tmp] + objs + ['-lpthread']
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, out)
    return out


if __name__ == '__main__':
    build(force='--force' in sys.argv, diag='--diag' in sys.argv)
