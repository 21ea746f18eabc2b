#!/usr/bin/env python3
"""Round 3's k_net_y (f16x3 variant 3) against the product kernel, in a process of its own.

Round 3's kernel keeps one stored-units exponent per workgroup, so past 2^14 its results depend on
the batch: it lives in the diagnostic library only (libmtaz_diag.so, build(diag=True); VERDICT r4
#7), which one process loads instead of libmtaz.so (MTAZ_LIB).  tests/test_gpu_net.py runs these
checks through this script as a child process; it prints one JSON line and exits 0 when every
check holds.

Usage: python tests/diag_round3.py {bit_identical | batch_dependent NET | tiny_mix}
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
DIAG = os.path.join(REPO, 'minitchess_alphazero_amd', 'libmtaz_diag.so')
os.environ['MTAZ_LIB'] = DIAG

import numpy as np  # noqa: E402


def _eng(n_games, sims, net):
    from minitchess_alphazero_amd.engine import Engine
    eng = Engine(n_games=n_games, sims=sims)
    eng.set_precision('f16x3')
    eng.set_weights(net)
    return eng


def _same(a, b):
    return bool(np.array_equal(a.view(np.uint32), b.view(np.uint32)))


def bit_identical():
    """Round 4's k_net_y (class tiles, off-board taps skipped, one exponent per board) computes
    exactly round 3's on nets whose bounds stay below 2^14 (both keep xs = 0 there): logits and
    values bitwise equal, main and tail launches alike."""
    import torch
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.network import Network
    from test_gpu_net import _tiny_activation_net
    from tests_positions import random_fens
    torch.manual_seed(0)
    fens = random_fens(400, seed=5)
    out = {}
    for name, net in (('seed0', Network()), ('tiny', _tiny_activation_net())):
        eng = _eng(4096, 4, net)
        for n in (257, 1024 + 400, 2048 + 900):
            pos = np.stack([pos_from_fen(fens[i % len(fens)]) for i in range(n)])
            eng.set_net_variant(0)
            l0, v0 = eng.evaluate(pos)
            eng.set_net_variant(3)
            l1, v1 = eng.evaluate(pos)
            out[f'{name}/{n}'] = _same(l0, l1) and _same(v0, v1)
        eng.close()
    return all(out.values()), out


def batch_dependent(net_kind):
    """Round 3's kernel on a net whose bound passes 2^14: regrouping the same positions changes
    some boards' bits there; the product kernel (variant 0) changes none."""
    from minitchess_alphazero_amd.environment import pos_from_fen
    from test_gpu_net import _stress_net, _wide_range_net
    from tests_positions import random_fens
    net = {'wide': _wide_range_net, 'stress': _stress_net}[net_kind]()
    pos = np.stack([pos_from_fen(f) for f in random_fens(1300, seed=41)])
    perm = np.random.default_rng(3).permutation(len(pos))
    eng = _eng(4096, 4, net)
    diff = {}
    for var in (3, 0):
        eng.set_net_variant(var)
        l0, v0 = eng.evaluate(pos)
        l1, v1 = eng.evaluate(pos[perm])
        same = (l1.view(np.uint32) == l0[perm].view(np.uint32)).all(axis=1) & (v1.view(np.uint32) == v0[perm].view(np.uint32))
        diff[var] = int((~same).sum())
    eng.close()
    return diff[0] == 0 and diff[3] > 0, {'round3': diff[3], 'round4': diff[0]}


def tiny_mix():
    """k_net_y equals round 3's kernel (whose v_fma_mix epilogue was pinned to its unfused form) on
    the f16-subnormal net."""
    from minitchess_alphazero_amd.environment import pos_from_fen
    from test_gpu_net import _tiny_activation_net
    from tests_positions import random_fens
    eng = _eng(64, 4, _tiny_activation_net())
    pos = np.stack([pos_from_fen(f) for f in random_fens(97, seed=6)])
    eng.set_net_variant(0)
    l0, v0 = eng.evaluate(pos)
    eng.set_net_variant(3)
    l1, v1 = eng.evaluate(pos)
    ok = _same(l0, l1) and _same(v0, v1)
    return ok, {'bitwise_equal': ok}


def main():
    if not os.path.exists(DIAG):
        print(json.dumps({'ok': False, 'error': f'{DIAG} not built (python -m minitchess_alphazero_amd.build --diag)'}))
        return 2
    what = sys.argv[1]
    if what == 'bit_identical':
        ok, info = bit_identical()
    elif what == 'batch_dependent':
        ok, info = batch_dependent(sys.argv[2])
    elif what == 'tiny_mix':
        ok, info = tiny_mix()
    else:
        raise SystemExit(f'unknown check {what}')
    from minitchess_alphazero_amd import _lib
    print(json.dumps({'ok': ok, 'check': sys.argv[1:], 'info': info, 'library': _lib.LIB_PATH}))
    return 0 if ok else 1


if __name__ == '__main__':
    sys.exit(main())
