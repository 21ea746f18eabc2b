"""CPU: the built library's gfx950 code object (no GPU needed).

The network kernels' K loops are unrolled by pragma.  In round 3 a change pushed the tail
instantiations (k_net_y<., 0, 1..3>, now k_net_y_tail) past LLVM's default pragma-unroll threshold: their loops
stayed rolled, the accumulator arrays went to scratch (528 B per lane) and those launches ran 14x
slower, with every output still bitwise correct.  This test reads the kernel metadata of the
product builds out of libmtaz.so and bounds their private (scratch) segment.
"""
import os
import re
import struct
import subprocess
import tempfile

import pytest

from conftest import REPO

LIB = os.path.join(REPO, 'minitchess_alphazero_amd', 'libmtaz.so')
READELF = '/opt/rocm/lib/llvm/bin/llvm-readelf'


def _code_objects():
    """The amdgcn-amd-amdhsa--gfx950 ELFs of the library's clang offload bundles (one per
    translation unit, in .hip_fatbin)."""
    data = open(LIB, 'rb').read()
    magic = b'__CLANG_OFFLOAD_BUNDLE__'
    found = []
    base = data.find(magic)
    while base >= 0:
        n = struct.unpack_from('<Q', data, base + len(magic))[0]
        p = base + len(magic) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from('<QQQ', data, p)
            triple = data[p + 24:p + 24 + tlen].decode(errors='replace')
            p += 24 + tlen
            if 'gfx950' in triple:
                found.append(data[base + off:base + off + size])
        base = data.find(magic, base + len(magic))
    assert found, 'no gfx950 code object in libmtaz.so'
    return found


def _kernel_private_sizes():
    if not os.path.exists(READELF):
        pytest.skip('llvm-readelf not available')
    notes = ''
    for co in _code_objects():
        with tempfile.NamedTemporaryFile(suffix='.co') as f:
            f.write(co)
            f.flush()
            notes += subprocess.run([READELF, '--notes', f.name], capture_output=True, text=True, check=True).stdout
    sizes = {}
    for block in notes.split('  - .agpr_count:')[1:]:
        name = re.search(r'\.name:\s+(\S+)', block)
        priv = re.search(r'\.private_segment_fixed_size:\s+(\d+)', block)
        if name and priv:
            sizes[name.group(1)] = int(priv.group(1))
    return sizes


def test_product_network_kernels_keep_accumulators_in_registers():
    sizes = _kernel_private_sizes()
    product = {k: v for k, v in sizes.items()
               if re.match(r'_ZN4mtaz7k_net_[yz]ILb0ELi0ELi[1-4]E', k) or re.match(r'_ZN4mtaz12k_net_y_tailILi0E', k)}
    # k_net_z: 4 board counts; k_net_y: the 4-board kernel and the tail kernel (1-3 boards)
    assert len(product) == 6, sorted(product)
    # a few spilled registers (bytes per lane) are tolerated; a demoted accumulator array is
    # hundreds of bytes
    assert max(product.values()) <= 64, product
