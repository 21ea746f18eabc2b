#!/usr/bin/env python3
"""Network-only microbenchmark and in-process A/B of the network kernels (PRECISION:VARIANT, e.g.
f16f8:0 = the product k_net_z, f16x3:0 = k_net_y).  --diag builds and loads libmtaz_diag.so
(-DMTAZ_NET_DIAG), which also holds the A/B and timing-only variants the product library rejects.

For each variant (interleaved over --rounds, one process, one device; MI355X devices
clock ~10% apart, so only same-process comparisons mean anything):
  * ms: average launch time over --iters back-to-back launches (HIP events)
  * tflops_algorithmic: 638,245,892 FLOP per board / ms
  * from one launch of the stamp-instrumented diagnostic build (shares only, never
    timed): mean per-workgroup cycles, phase shares (stem / conv K loops / conv
    epilogues / heads) and the effective clock (s_memtime / s_memrealtime).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=4096)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--variants', default='0', help='comma list of VARIANT or PRECISION:VARIANT '
                                                   '(e.g. f16x3:0,f16f8:0,f16f8:2048)')
    ap.add_argument('--precision', default='f16f8')
    ap.add_argument('--diag', action='store_true', help='load the diagnostic library (all variants)')
    args = ap.parse_args()
    if args.diag:
        from minitchess_alphazero_amd.build import build
        os.environ['MTAZ_LIB'] = build(verbose=False, diag=True)
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
    variants = [v if ':' in v else f'{args.precision}:{v}' for v in args.variants.split(',')]
    nwg = (args.n + 3) // 4
    res = {v: {'ms': [], 'cycles': [], 'ghz': [], 'shares': []} for v in variants}
    for _ in range(args.rounds):
        for v in variants:
            prec, var = v.split(':')
            eng.set_precision(prec)
            _lib.check(eng.L.mtaz_set_net_variant(eng.h, int(var)))
            ms = ctypes.c_float()
            st = np.zeros(nwg * 10, np.uint64)   # phase stamps [nwg][6], then exponent records [nwg][4]
            _lib.check(eng.L.mtaz_net_time(eng.h, ctypes.c_void_p(d.data_ptr()), args.n, args.iters, 1,
                                           ctypes.byref(ms), st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
            st = st[:nwg * 6].reshape(nwg, 6).astype(np.float64)
            res[v]['ms'].append(ms.value)
            res[v]['cycles'].append(float(st[:, 4].mean()))
            res[v]['ghz'].append(float((st[:, 4] / (st[:, 5] * 10.0)).mean()))   # cycles / (ticks * 10 ns) -> GHz
            res[v]['shares'].append((st[:, :4] / st[:, :4].sum(axis=1, keepdims=True)).mean(axis=0))
    # outputs vs the first variant (64 games' engine evaluates 64 positions at a time)
    ref = None
    check = {}
    for v in variants:
        prec, var = v.split(':')
        eng.set_precision(prec)
        _lib.check(eng.L.mtaz_set_net_variant(eng.h, int(var)))
        lg, vl = eng.evaluate(pos[:64])
        if ref is None:
            ref = (lg, vl)
        check[v] = {'bitwise_equal_to_first': bool(np.array_equal(lg, ref[0]) and np.array_equal(vl, ref[1])),
                    'max_logit_diff': float(np.abs(lg - ref[0]).max()), 'max_value_diff': float(np.abs(vl - ref[1]).max())}
    for v in variants:
        r = res[v]
        ms = float(np.median(r['ms']))
        out = {'variant': v, 'n': args.n, 'ms_median': ms, 'ms_all': r['ms'],
               'tflops_algorithmic': FLOP_PER_EVAL * args.n / (ms * 1e-3) / 1e12,
               'wg_cycles': float(np.median(r['cycles'])), 'clock_ghz_stamped': float(np.median(r['ghz'])),
               'shares': dict(zip(['stem', 'conv_kloop', 'conv_epilogue', 'heads'],
                                  np.mean(r['shares'], axis=0).round(4).tolist())),
               'check': check[v]}
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
