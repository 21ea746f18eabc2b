#!/usr/bin/env python3
"""Experimental library builds for tools/ab_libs.sh: libmtaz_<name>.so next to libmtaz.so, the
network translation unit (csrc/mtaz_net16.hip) compiled with extra -D flags, every other unit
shared.  Each library embeds the tree's source hash, so the Python binding loads it through
MTAZ_LIB like the product library (same sources, other flags: an A/B of compile-time knobs across
processes on one box).

  python tools/build_exp_libs.py name=FLAGS [name=FLAGS ...]
  e.g. python tools/build_exp_libs.py base= knob="-DSOME_KNOB=0"
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from minitchess_alphazero_amd import build as B  # noqa: E402


def main():
    sha = B.source_hash()
    hipcc = B._hipcc()
    bdir = os.path.join(B.HERE, '_build_exp')
    os.makedirs(bdir, exist_ok=True)
    cfgs = [a.split('=', 1) for a in sys.argv[1:]]

    def cmd(src, flags, obj, extra=()):
        return [hipcc, '-x', 'hip', '-std=c++17', f'--offload-arch={B.ARCH}', '-fPIC', '-c', os.path.join(B.CSRC, src),
                '-o', obj, f'-I{B.INCLUDE}', '-Wall', '-Wno-unused-function', f'-DMTAZ_SRC_SHA256="{sha}"'] + flags + list(extra)

    procs, shared = [], []
    for src, flags in B.SOURCES:
        if src == 'mtaz_net16.hip':
            continue
        obj = os.path.join(bdir, f'{src}.{sha[:12]}.o')
        shared.append(obj)
        if not os.path.exists(obj):
            procs.append(subprocess.Popen(cmd(src, flags, obj)))
    net_flags = dict(B.SOURCES)['mtaz_net16.hip']
    nets = {}
    for name, extra in cfgs:
        obj = os.path.join(bdir, f'net16.{name}.{sha[:12]}.o')
        nets[name] = obj
        procs.append(subprocess.Popen(cmd('mtaz_net16.hip', net_flags, obj, extra.split())))
    for p in procs:
        if p.wait() != 0:
            raise SystemExit('hipcc failed')
    for name, obj in nets.items():
        out = os.path.join(B.HERE, f'libmtaz_{name}.so')
        subprocess.check_call([hipcc, '-shared', f'--offload-arch={B.ARCH}', '-o', out, obj] + shared + ['-lpthread'])
        print('built', out)


if __name__ == '__main__':
    main()
