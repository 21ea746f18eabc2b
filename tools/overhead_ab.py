#!/usr/bin/env python3
"""In-process A/B of per-wave launch overheads on the bench workload (4096 games x 64 sims,
random-init weights, the bench defaults): for each mode, one engine; plays interleaved over
--rounds; wall seconds of one play() and the records checked identical across modes.

A mode is a comma-free token of flags: t<N> = Engine.set_timing(N) (0 off, 1 events every wave),
w<M> = Engine.set_wave_tail(M) (the round-6 experiment of profiles/r06/overhead/wave_tail.diff: a
library built with that diff; the product has no such setter), s<A> = Engine.set_select_ahead(A)
(likewise profiles/r06/select_ahead/select_ahead.diff).
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
    args = ap.parse_args()
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
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
                           'nn_evals': int(st['nn_evals']), 'memo_hits': int(st['memo_hits']),
                           'same_records': bool(same)})
            print(f'[overhead_ab] round {r} mode {m}: {res[m][-1]}', file=sys.stderr, flush=True)
            if not same:
                print(f'[overhead_ab] RECORDS DIFFER in mode {m}', file=sys.stderr, flush=True)
                sys.exit(4)
    for m in modes:
        rows = res[m]
        print(json.dumps({'mode': m, 'games': args.games, 'sims': args.sims, 'rounds': args.rounds,
                          'wall_s_median': float(np.median([x['wall_s'] for x in rows])), 'runs': rows}), flush=True)


if __name__ == '__main__':
    main()
