"""The 554-code MinitChess action space (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates exp/generate_moves_list.py:5-57: for every from-square in row-major
order (rank i in 0..5, file j in 0..4) the 8 queen directions x distance 1..5
(off-board entries skipped, :11-22, :40-45), then the 8 knight jumps (:24-34);
white codes use absolute squares (:47-48), black codes the same geometry with
both squares rotated 180 degrees, 29 - sq (:50-57).  The generated JSON must be
byte-identical to the reference's exp/moves_dict.json (its sha256 is pinned in
tests/golden/codec.json).
"""
import json

from .rules import square_name

QDIRS = [[1, 1], [1, 0], [1, -1], [0, 1], [0, -1], [-1, 1], [-1, 0], [-1, -1]]   # :11-12
KDIRS = [[1, 2], [1, -2], [-1, 2], [-1, -2], [2, 1], [2, -1], [-2, 1], [-2, -1]]  # :24-25


def _geometry():
    """(from_sq, to_sq) pairs in code order, as (row, col) -> 5*row + col (:5-9)."""
    movs = []
    for i in range(6):
        for j in range(5):
            for di, dj in QDIRS:
                for dist in range(1, 6):
                    ti, tj = i + dist * di, j + dist * dj
                    movs.append((5 * i + j, 5 * ti + tj if (0 <= ti < 6 and 0 <= tj < 5) else None))
    for i in range(6):
        for j in range(5):
            for di, dj in KDIRS:
                ti, tj = i + di, j + dj
                movs.append((5 * i + j, 5 * ti + tj if (0 <= ti < 6 and 0 <= tj < 5) else None))
    return [(f, t) for f, t in movs if t is not None]


GEOMETRY = _geometry()
NUM_ACTIONS = len(GEOMETRY)   # 554


def moves_dict():
    w = {square_name(f) + square_name(t): code for code, (f, t) in enumerate(GEOMETRY)}
    b = {square_name(29 - f) + square_name(29 - t): code for code, (f, t) in enumerate(GEOMETRY)}
    return {'w': w, 'b': b}


def moves_dict_json():
    """Exactly what exp/generate_moves_list.py:59-60 writes (json.dump defaults)."""
    return json.dumps(moves_dict())


def tables():
    """(encode, decode): encode[side][from*30+to] -> code or -1; decode[side][code] -> (from, to).

    side 0 = white, 1 = black; squares are absolute board squares."""
    enc = [[-1] * 900, [-1] * 900]
    dec = [[None] * NUM_ACTIONS, [None] * NUM_ACTIONS]
    for code, (f, t) in enumerate(GEOMETRY):
        enc[0][f * 30 + t] = code
        dec[0][code] = (f, t)
        enc[1][(29 - f) * 30 + (29 - t)] = code
        dec[1][code] = (29 - f, 29 - t)
    return enc, dec
