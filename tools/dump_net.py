#!/usr/bin/env python3
"""Dump the GPU network's logits and values on the stress fixture positions for each
PRECISION:VARIANT (GPU box), for tools/stress_error.py --gpu to compare against fp64 on the CPU.

Usage: python tools/dump_net.py OUT.npz f16x3:0,fp32:0,f16x3:268435456 [--diag]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    out, specs = sys.argv[1], sys.argv[2].split(',')
    if '--diag' in sys.argv:
        from minitchess_alphazero_amd.build import build
        os.environ['MTAZ_LIB'] = build(verbose=False, diag=True)
    from helpers import stress_network
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    z = np.load(os.path.join(ROOT, 'tests', 'golden', 'stress_net.npz'))
    pos = np.stack([pos_from_fen(str(f)) for f in z['fens']])
    eng = Engine(n_games=len(pos), sims=4)
    res = {}
    for s in specs:
        prec, var = s.split(':')
        eng.set_precision(prec)
        eng.set_net_variant(int(var))
        eng.set_weights(stress_network())
        lg, v = eng.evaluate(pos)
        res[f'{prec}_{var}_logits'], res[f'{prec}_{var}_values'] = lg, v
        print(s, 'done', flush=True)
    np.savez_compressed(out, **res)


if __name__ == '__main__':
    main()
