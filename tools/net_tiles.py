#!/usr/bin/env python3
"""The class tiles of round 4's k_net_y (csrc/mtaz_net16.hip TMAP4): generate and check.

A workgroup's 4 boards x 32 squares (30 on the 6 x 5 board + 2 padding) are the N dimension of the
conv GEMMs, in 8 tiles of 16 (one MFMA column block each).  Round 3 tiled by board; here by the
squares' position class, so that a tile whose 16 squares all read zeros for a tap (their sources
fall off the board) skips that tap:
  tiles 0, 1, 4  interior squares (rows 1-4, files 1-3): all 9 taps
  tile 2  R: file 4, rows 1-4                           no dc = +1 taps
  tile 3  T: row 0, files 0-3 (top-left corner + top)   no dr = -1 taps   (gated per tap row)
  tile 5  L: file 0, rows 1-4                           no dc = -1 taps
  tile 6  X: squares 4, 29 (right corners), 30, 31      no dc = +1 taps
  tile 7  B: row 5, files 0-3                           no dr = +1 taps   (gated per tap row)
Half 0 = tiles 0-3, half 1 = tiles 4-7 (each half-step of the K loop runs one half).  Every tile
holds 16 (board, square) pairs with distinct (square + 4 board) mod 16, the bank group of a cell
in the kernel's image, so a fragment read is conflict-free for every tap.  Lane n of a tile holds
the pair of bank group n.  Prints the C table and checks the skip rule of csrc/mtaz_net16.hip
act() / gated() against the squares' actual sources.
"""
from collections import defaultdict

INTERIOR = [p for p in range(30) if 1 <= p // 5 <= 4 and 1 <= p % 5 <= 3]
T, B = [0, 1, 2, 3], [25, 26, 27, 28]
L, R = [5, 10, 15, 20], [9, 14, 19, 24]
X = [4, 29, 30, 31]


def res(b, p):
    return (p + 4 * b) & 15


def build():
    inner = [[], [], []]
    byres = defaultdict(list)
    for b in range(4):
        for p in INTERIOR:
            byres[res(b, p)].append((b, p))
    for r, items in sorted(byres.items()):
        assert len(items) == 3
        for i, it in enumerate(items):
            inner[i].append(it)
    cls = {name: [(b, p) for b in range(4) for p in sq] for name, sq in (('T', T), ('B', B), ('L', L), ('R', R), ('X', X))}
    tiles = [inner[0], inner[1], cls['R'], cls['T'], inner[2], cls['L'], cls['X'], cls['B']]
    return [sorted(t, key=lambda bp: res(*bp)) for t in tiles]


def valid(p, tap):
    dh, dw = tap // 3 - 1, tap % 3 - 1
    r, c = p // 5 + dh, p % 5 + dw
    return p < 30 and 0 <= r < 6 and 0 <= c < 5


def rule(t, tap):
    """csrc/mtaz_net16.hip act() + gated(): is tile t run at this tap?"""
    dr, dc = tap // 3 - 1, tap % 3 - 1
    return {0: True, 1: True, 2: dc != 1, 3: dr != -1, 4: True, 5: dc != -1, 6: dc != 1, 7: dr != 1}[t]


# The 3-board tail instance (round 4b): 3 x 32 squares in 6 tiles (t = 4 half + i, i < 3).
#   t0, t1  interior squares: all 9 taps
#   t2      T (top row, files 0-3) + 4 of the X squares (4 of board 2, 29-31 of board 0):
#           skips the tap (dr, dc) = (-1, +1)                       (gated in tap row 0)
#   t4      L (file 0, rows 1-4) + 4 interior squares: all 9 taps
#   t5      R (file 4, rows 1-4) + 4 X squares: no dc = +1 taps       (compile-time)
#   t6      B (bottom row, files 0-3) + 4 X squares: skips (+1, +1)   (gated in tap row 2)
# 49 of 54 tile-taps run (per-board tiles: 54 of 54).  With the kernel's bank rotation (square + 4
# board) the classes cannot all hold distinct bank groups (no per-board rotation admits this
# tiling conflict-free: a search over all of them finds none), so t0, t1 and t5 keep 2, 1 and 3
# duplicate bank groups (2-way conflicts on a few fragment-read lane groups).
XT = [(2, 4), (0, 29), (0, 30), (0, 31)]
XB = [(1, 4), (2, 29), (2, 30), (2, 31)]
XR = [(0, 4), (1, 29), (1, 30), (1, 31)]
I4 = [(0, 6), (0, 11), (0, 16), (0, 17)]


def _lanes(items):
    """lane n gets an item of bank group n where one is left, the rest fill the other lanes"""
    lanes, rest = [None] * 16, []
    for it in sorted(items, key=lambda bp: (res(*bp), bp)):
        if lanes[res(*it)] is None:
            lanes[res(*it)] = it
        else:
            rest.append(it)
    for n in range(16):
        if lanes[n] is None:
            lanes[n] = rest.pop(0)
    return lanes


def build3():
    inner = [(b, p) for b in range(3) for p in INTERIOR if (b, p) not in I4]
    a, b_ = [], []
    for it in sorted(inner, key=lambda bp: (res(*bp), bp)):   # alternate within each bank group
        (a if len(a) <= len(b_) and (len({res(*q) for q in a + [it]}) > len({res(*q) for q in a}) or len(b_) >= 16)
         else b_).append(it)
    cls = {name: [(b, p) for b in range(3) for p in sq] for name, sq in (('T', T), ('B', B), ('L', L), ('R', R))}
    tiles = {0: a, 1: b_, 2: cls['T'] + XT, 4: cls['L'] + I4, 5: cls['R'] + XR, 6: cls['B'] + XB}
    assert sorted(len(t) for t in tiles.values()) == [16] * 6
    return {t: _lanes(v) for t, v in tiles.items()}


def rule3(t, tap):
    """csrc/mtaz_net16.hip act() + gated() for 3 boards"""
    dr, dc = tap // 3 - 1, tap % 3 - 1
    return {0: True, 1: True, 2: (dr, dc) != (-1, 1), 4: True, 5: dc != 1, 6: (dr, dc) != (1, 1)}[t]


def main3():
    tiles = build3()
    act = {t: [any(valid(p, tap) for _, p in v) for tap in range(9)] for t, v in tiles.items()}
    assert all(act[t][tap] == rule3(t, tap) for t in tiles for tap in range(9))
    assert sorted(it for v in tiles.values() for it in v) == [(b, p) for b in range(3) for p in range(32)]
    dups = {t: 16 - len({res(*q) for q in v}) for t, v in tiles.items()}
    print('3 boards: tile-taps run:', sum(map(sum, act.values())), 'of', 6 * 9, '; duplicate bank groups', dups)
    rows = [[b | (p << 2) for b, p in tiles[t]] if t in tiles else [0] * 16 for t in range(8)]
    print('__constant__ uint8_t TMAP3[8][16] = {')
    print(',\n'.join('    {' + ', '.join(map(str, r)) + '}' for r in rows) + '};')
    return rows


def main():
    main3()
    tiles = build()
    for t in tiles:
        assert sorted(res(*bp) for bp in t) == list(range(16)), t
    act = [[any(valid(p, tap) for _, p in t) for tap in range(9)] for t in tiles]
    assert all(act[t][tap] == rule(t, tap) for t in range(8) for tap in range(9))
    print('tile-taps run:', sum(map(sum, act)), 'of', 8 * 9)
    print('__constant__ uint8_t TMAP4[8][16] = {')
    print(',\n'.join('    {' + ', '.join(str(b | (p << 2)) for b, p in t) + '}' for t in tiles) + '};')


if __name__ == '__main__':
    main()
