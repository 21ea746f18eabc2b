#!/usr/bin/env python3
"""In-process A/B of per-wave launch overheads on the bench workload (4096 games x 64 sims,
random-init weights, the bench defaults): for each mode, one engine; plays interleaved over
--rounds; wall seconds of one play() and the records checked identical across modes.

A mode is a comma-free token of flags: t<N> = Engine.set_timing(N) (0 off, 1 events every wave),
w<M> = Engine.set_wave_tail(M) (the round-6 experiment of profiles/r06/overhead/wave_tail.diff: a
library built with that diff; the product has no such setter), s<A> = Engine.set_select_ahead(A)
(likewise profiles/r06/select_ahead/select_ahead.diff), l<O> = Engine.set_lag_order(O),
f<S> = Engine.set_schedule(S) (1 = free-running moves), d<D> = Engine.set_defer(D).
Example: --modes t1,t0 or --modes s1,s0
Output: one JSON line per mode (median wall, every run).
"""
import argparse
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def parse(mode):
    d = {'t': 1}
    for k, v in re.findall(r'([a-z])(\d+)', mode):
        d[k] = int(v)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=4096)
    ap.add_argument('--sims', type=int, default=64)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--modes', default='t1,t0')
    ap.add_argument('--weights', default='', help='safetensors state_dict (e.g. tests/golden/c3/c3.safetensors: '
                    'BASELINE config 3) instead of the seed-0 random init')
    args = ap.parse_args()
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    if args.weights:
        from safetensors.torch import load_file
        net.load_state_dict(load_file(args.weights))   # module order (weight_tensors)
    modes = args.modes.split(',')
    engs = {}
    for m in modes:
        f = parse(m)
        e = Engine(n_games=args.games, sims=args.sims, seed_base=0)
        e.set_weights(net)
        e.set_timing(f['t'])
        if 'w' in f:
            e.set_wave_tail(f['w'])
        if 's' in f:
            e.set_select_ahead(f['s'])
        if 'l' in f:
            e.set_lag_order(f['l'])
        if 'f' in f:
            e.set_schedule(f['f'])
        if 'd' in f:
            e.set_defer(f['d'])
        engs[m] = e
    res = {m: [] for m in modes}
    ref = None
    for r in range(args.rounds):
        for m in modes:
            st = engs[m].play()
            rec = engs[m].records()
            if ref is None:
                ref = rec
            same = all(np.array_equal(rec[k], ref[k]) for k in ('plies', 'pos', 'action', 'visits', 'reward'))
            res[m].append({'wall_s': st['wall_ms'] / 1e3, 'trunk_ms': st['trunk_ms'], 'waves': int(st['waves']),
                           'extra_waves': int(st['extra_waves']), 'moves': int(st['moves']),
                           'schedule': int(st['schedule']), 'turn_or_rng_ms': st['rng_dev_ms'],
                           'select_ms': st['select_ms'], 'compact_ms': st['compact_ms'], 'sync_ms': st['sync_ms'],
                           'nn_evals': int(st['nn_evals']), 'memo_hits': int(st['memo_hits']),
                           'same_records': bool(same)})
            print(f'[overhead_ab] round {r} mode {m}: {res[m][-1]}', file=sys.stderr, flush=True)
            if not same:
                print(f'[overhead_ab] RECORDS DIFFER in mode {m}', file=sys.stderr, flush=True)
                sys.exit(4)
    for m in modes:
        rows = res[m]
        print(json.dumps({'mode': m, 'games': args.games, 'sims': args.sims, 'rounds': args.rounds,
                          'weights': args.weights or 'seed-0 random init',
                          'wall_s_median': float(np.median([x['wall_s'] for x in rows])), 'runs': rows}), flush=True)


if __name__ == '__main__':
    main()
