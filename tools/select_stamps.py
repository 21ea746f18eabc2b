#!/usr/bin/env python3
"""Where k_select's time goes: plays --games x --sims self-play with the diagnostic library (whose
k_select sums s_memtime cycles per phase over its waves: hash lookup, PUCT selection + child
apply, legal-move generation, terminal test, insert / edge init / terminal backup) and prints the
per-wave means next to the engine's select_ms.  Diagnostic library only; never the product path."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=4096)
    ap.add_argument('--sims', type=int, default=64)
    ap.add_argument('--lib', default=None, help='library path (default: build the diagnostic one)')
    ap.add_argument('--select-ahead', type=int, default=None,
                    help='Engine.set_select_ahead: only with a library built with profiles/r06/select_ahead/select_ahead.diff')
    args = ap.parse_args()
    if args.lib:
        os.environ['MTAZ_LIB'] = args.lib
    else:
        from minitchess_alphazero_amd.build import build
        os.environ['MTAZ_LIB'] = build(verbose=False, diag=True)
    import torch
    from minitchess_alphazero_amd import _lib
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    L = _lib.lib()
    f = L.mtaz_diag_select_stamps
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    f.restype = ctypes.c_int
    torch.manual_seed(0)
    eng = Engine(n_games=args.games, sims=args.sims)
    eng.set_weights(Network())
    eng.set_timing(True)
    if args.select_ahead is not None:
        eng.set_select_ahead(args.select_ahead)
    out = (ctypes.c_ulonglong * 8)()
    assert f(out, 1) == 0
    st = eng.play()
    assert f(out, 0) == 0
    v = np.array(list(out), dtype=np.float64)
    waves = max(v[0], 1.0)
    names = ['waves', 'find', 'select', 'legal', 'outcome', 'insert_init_backup', 'total', 'depth']
    res = {'games': args.games, 'sims': args.sims, 'select_ahead': args.select_ahead, 'waves': int(v[0]),
           'cycles_per_wave': {n: v[i] / waves for i, n in enumerate(names) if 0 < i < 7},
           'mean_depth': v[7] / waves,
           'select_ms_total': st['select_ms'], 'sims_total': st['sims'], 'plies': st['plies'],
           'select_us_per_launch': 1000.0 * st['select_ms'] / max(st['waves'], 1), 'launches': st['waves']}
    print(json.dumps(res))


if __name__ == '__main__':
    main()
