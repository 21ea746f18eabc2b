#!/usr/bin/env python3
"""Duplicate leaves inside one simulation's batch (GPU; measurement only).

Plays one batch of self-play games on the engine one simulation at a time (sim_select ->
leaves -> sim_evaluate -> sim_backup, the kernels of simulate()) and counts, per simulation,
the leaves the network evaluates and the distinct positions among them.  The batch memo
(memo mode 2) only supplies positions evaluated in an EARLIER simulation; a position that
several games reach in the same simulation is evaluated once per game.  The noise and the
action choice are numpy's (not the reference's per-game streams: the statistics, not the
games, are the point).  Prints one JSON line: totals and the per-move profile.
"""
import argparse
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
    ap.add_argument('--memo', type=int, default=2)
    args = ap.parse_args()
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import STARTING_FEN
    from minitchess_alphazero_amd.network import Network
    G, S = args.games, args.sims
    eng = Engine(n_games=G, sims=S)
    torch.manual_seed(0)
    eng.set_weights(Network())
    eng.set_memo(args.memo)
    eng.set_games([STARTING_FEN] * G)
    eng.clear_trees()
    rng = np.random.RandomState(0)
    tot_leaves = tot_distinct = 0
    per_move = []
    while True:
        pos, _ag, act, _oc = eng.games()
        if not act.any():
            break
        k, new = eng.move_begin()
        noise = [rng.dirichlet([0.6] * int(k[g]), size=S - int(new[g]))
                 if act[g] and S - new[g] > 0 else None for g in range(G)]
        eng.set_noise(noise)
        ml = md = 0
        for s in range(S):
            eng.sim_select(s)
            lpos, _lg, lk, _lc = eng.leaves()
            n = len(lk)
            if n:
                d = len(np.unique(np.ascontiguousarray(lpos).view(np.dtype((np.void, lpos.dtype.itemsize * lpos.shape[1])))))
            else:
                d = 0
            ml += n
            md += d
            eng.sim_evaluate()
            eng.sim_backup()
        tot_leaves += ml
        tot_distinct += md
        per_move.append([ml, md])
        codes, visits, _k = eng.move_end()
        actions = np.zeros(G, np.int32)
        for g in range(G):
            if not act[g]:
                continue
            kk = int(k[g])
            N = visits[g][:kk].astype(np.float64)
            actions[g] = int(codes[g][rng.choice(kk, p=N / N.sum())])
        eng.apply(actions)
        print(f'[dup] move {len(per_move)}: {ml} leaves, {md} distinct', file=sys.stderr, flush=True)
    print(json.dumps({'games': G, 'sims': S, 'memo': args.memo, 'leaves': tot_leaves, 'distinct': tot_distinct,
                      'dup_frac': 1 - tot_distinct / max(tot_leaves, 1), 'per_move': per_move}))


if __name__ == '__main__':
    main()
