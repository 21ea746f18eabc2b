"""CPU: k_net_y's tile table and LDS layout properties (csrc/mtaz_net16.hip), no GPU needed.

The class tiles (TMAP4) in the kernel source are the ones tools/net_tiles.py generates and checks
(every tile holds each bank group once; the tap-skip rule of act() / gated() matches the squares'
real sources: 57 of 72 tile-taps), and tools/lds_model_y.py's bank model of the fragment reads
holds the round-4b properties: the 1- and 2-board tail instances read conflict-free, the 4-board
kernel within 10% extra cycles (its padding-square zero cells), the 3-board class tiles within 35%
(their duplicate bank groups: 2-way reads on three of the six tiles)."""
import os
import re
import sys

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, 'tools'))


def _kernel_tmap(name='TMAP4'):
    src = open(os.path.join(REPO, 'minitchess_alphazero_amd', 'csrc', 'mtaz_net16.hip')).read()
    body = re.search(name + r'\[8\]\[16\] = \{(.*?)\};', src, re.S).group(1)
    return [[int(x) for x in row.split(',')] for row in re.findall(r'\{([^{}]*)\}', body)]


def test_kernel_tiles_are_the_generated_ones():
    import net_tiles
    net_tiles.main()                      # asserts the bank groups and the skip rule
    gen = [[b | (p << 2) for b, p in t] for t in net_tiles.build()]
    assert _kernel_tmap('TMAP4') == gen
    gen3 = net_tiles.main3()               # asserts the 3-board skip rule and coverage
    assert _kernel_tmap('TMAP3') == gen3
    import lds_model_y
    assert lds_model_y.TMAP4 == gen and lds_model_y.TMAP3 == gen3


def test_fragment_reads_bank_model():
    import lds_model_y as m
    for nvb in (4, 3, 2, 1):
        tot = ideal = 0
        for tap in range(9):
            for t in range(8):
                if (t & 3) >= nvb or (nvb >= 3 and not m.active(t, tap, nvb)):
                    continue
                for kb in (0, 5):
                    for part in (0, 1):
                        tot += m.cycles([m.entry(nvb, t, l, tap, False) + 1024 * kb + part * m.PART_B
                                         for l in range(64)])
                        ideal += 4
        if nvb < 3:
            assert tot == ideal, nvb
        else:                              # class tiles: a few duplicate bank groups
            assert (tot - ideal) / tot < (0.35 if nvb == 3 else 0.10), nvb
