#!/usr/bin/env python3
"""In-process A/B of the simulation-wave schedules on the bench workload: moves in lockstep or
free-running (Engine.set_schedule 0 / 1) x deferred tails (Engine.set_defer 0 / 1 / 2), a mode
written as L<defer> or F<defer> (a bare digit = lockstep, round 5's form).

For each mode (interleaved over --rounds, one engine per mode, same seeds, random-init weights):
wall seconds of one play(), network milliseconds (HIP events per wave), waves and extra waves, and
from the per-wave log (Engine.wave_log) how the evaluated leaves fall into launches: the waves that
ran whole rounds of 4 boards x CUs only, a partial 4-board round (remainder > 3 boards per CU) or a
tail launch (1-3 boards per CU), the boards per launch, and the network milliseconds per
round-equivalent (1,024 boards on 256 CUs).  Records must be identical across modes (checked).
Output: one JSON line per mode.
Usage: python tools/wave_sched.py [--games 4096 --sims 64 --rounds 2 --modes L1,F1,F2]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=4096)
    ap.add_argument('--sims', type=int, default=64)
    ap.add_argument('--rounds', type=int, default=2)
    ap.add_argument('--modes', default='L1,F1')
    ap.add_argument('--memo', type=int, default=2)
    args = ap.parse_args()
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    modes = [m if m[0] in 'LF' else 'L' + m for m in args.modes.split(',')]
    engs = {}
    for m in modes:
        e = Engine(n_games=args.games, sims=args.sims, seed_base=0)
        e.set_weights(net)
        e.set_memo(args.memo)
        e.set_defer(int(m[1:]))
        e.set_schedule(1 if m[0] == 'F' else 0)
        e.set_timing(True)
        engs[m] = e
    cu = torch.cuda.get_device_properties(0).multi_processor_count
    rnd = 4 * cu
    res = {m: [] for m in modes}
    ref = None
    for r in range(args.rounds):
        for m in modes:
            st = engs[m].play()
            log = engs[m].wave_log()
            rec = engs[m].records()
            if ref is None:
                ref = rec
            same = all(np.array_equal(rec[k], ref[k]) for k in ('plies', 'pos', 'action', 'visits', 'reward'))
            ev = log[:, 0].astype(np.int64)
            ev = ev[ev > 0]
            rem = ev % rnd
            res[m].append({'wall_s': st['wall_ms'] / 1e3, 'trunk_ms': st['trunk_ms'], 'waves': int(st['waves']),
                           'schedule': int(st['schedule']), 'turn_ms': st['rng_dev_ms'], 'select_ms': st['select_ms'],
                           'compact_ms': st['compact_ms'], 'sync_ms': st['sync_ms'],
                           'extra_waves': int(st['extra_waves']), 'nn_evals': int(st['nn_evals']), 'same_records': bool(same),
                           'launches': int(len(ev)), 'whole_rounds_only': int((rem == 0).sum()),
                           'partial_round': int((rem > 3 * cu).sum()), 'tail': int(((rem > 0) & (rem <= 3 * cu)).sum()),
                           'boards_per_launch': float(ev.mean()) if len(ev) else 0.0,
                           'ms_per_round_equiv': st['trunk_ms'] / (ev.sum() / rnd) if len(ev) else None})
            print(f'[wave_sched] round {r} mode {m}: {res[m][-1]}', file=sys.stderr, flush=True)
    for m in modes:
        rows = res[m]
        out = {'mode': m, 'games': args.games, 'sims': args.sims, 'rounds': args.rounds,
               'wall_s_median': float(np.median([x['wall_s'] for x in rows])),
               'trunk_ms_median': float(np.median([x['trunk_ms'] for x in rows])), 'runs': rows}
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
