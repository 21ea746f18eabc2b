#!/usr/bin/env python3
"""Network-only microbenchmark (k_net_x / fp32 path) on n random positions.

Prints the average launch time (HIP events, back-to-back launches), the algorithmic
TFLOP/s (638,245,892 FLOP per board) and, from one launch of the stamp-instrumented
diagnostic build, the per-workgroup cycle shares of stem / conv K loops / conv
epilogues / heads.  Shares only: the stamped build itself is never timed.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--precision', default='f16x3')
    args = ap.parse_args()
    import torch
    from minitchess_alphazero_amd import _lib
    from minitchess_alphazero_amd.engine import Engine, FLOP_PER_EVAL
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.network import Network
    from tests_positions import random_fens
    fens = random_fens(min(args.n, 1024), seed=1)
    pos = np.stack([pos_from_fen(fens[i % len(fens)]) for i in range(args.n)])
    eng = Engine(n_games=args.n if args.precision == 'fp32' else 64, sims=4)
    torch.manual_seed(0)
    eng.set_weights(Network())
    eng.set_precision(args.precision)
    d = torch.from_numpy(pos.view(np.int32)).cuda()
    torch.cuda.synchronize()
    ms = ctypes.c_float()
    nwg = (args.n + 3) // 4
    st = np.zeros(nwg * 4, np.uint64)
    _lib.check(eng.L.mtaz_net_time(eng.h, ctypes.c_void_p(d.data_ptr()), args.n, args.iters, 1,
                                   ctypes.byref(ms), st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
    st = st.reshape(nwg, 4).astype(np.float64)
    tot = st.sum(axis=1)
    shares = (st / tot[:, None]).mean(axis=0)
    out = {'n': args.n, 'precision': args.precision, 'ms': ms.value,
           'tflops_algorithmic': FLOP_PER_EVAL * args.n / (ms.value * 1e-3) / 1e12,
           'wg_cycles_mean': float(tot.mean()),
           'shares': dict(zip(['stem', 'conv_kloop', 'conv_epilogue', 'heads'], shares.round(4).tolist()))}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
