#!/usr/bin/env python3
"""Round-4 golden fixtures for the STRESS4 checkpoint, made by running the REFERENCE code on the CPU
(build container only; same stubs as make_golden.py: un-vendored erlyx, oracle.rules as `chess`).

VERDICT r3 #3: the round-3 stress checkpoint's value head collapsed to a constant (its self-play
data was almost all draws), so every value check on it passed trivially.  tools/train_stress.py
--endgame-frac 0.5 trained stress4 in the C5 loop with half of each iteration's games started from
random K + heavy pieces v K positions, which end decisively often enough for the value targets to
vary, at lr 0.003, and kept the first network past 20 updates that met the criteria the training
log records: trunk |activation| >= 100 (min_trunk), legal-logit spread >= 8 (min_spread), largest
|logit| <= 3000 and value_std >= 0.05 (iteration 19 of its run: trunk 169, value_std 0.054).  On
the fixture positions below the reference measures trunk |activation| up to 190.6, legal-logit
spreads up to 5.8 (median 0.75), a median top prior of 0.23 and values -0.26 .. 0.33 (std 0.058):
a value head that varies, but NOT the range past 2^14 where k_net_y's per-board stored-units
exponents leave 0 (tools/net_range.py: 0 on every layer and position).  That path is pinned by the
round-3 'stress' net (lightly: one position) and the wide-range test net, and, with varying values,
by round 5's stress5 (make_golden_r5.py).  The checkpoint is data (GPU training is not bitwise
reproducible); this script pins it and records what the reference computes on it:

  stress4.json       sha256 of the checkpoint (oracle.net.state_dict_sha256), the training log
                     (tools/train_stress.py output), the network's ranges on the fixture positions
                     (legal-logit spread, largest prior, trunk |activation| max with forward hooks
                     on the reference modules, value range and standard deviation), and two
                     reference self-play games at 64 sims with the checkpoint (np.random.seed(0)):
                     'game_start' from STARTING_FEN and 'game_end' from an endgame start
  stress4_net.npz    the reference Network.forward (eval mode) on the fixture positions: the
                     positions of both games, 64 endgame starts (make_golden_r2.endgame_starts,
                     seed 44), then sample_positions(64, seed=778): fens, logits [n, 554], values [n]

Usage: python tests/golden/make_golden_r4.py [path/to/train.jsonl]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from make_golden import import_reference, sample_positions  # noqa: E402
from make_golden_r2 import endgame_starts, ref_selfplay  # noqa: E402

THREADS = 8
CKPT = os.path.join(HERE, 'stress4', 'stress4.safetensors')


def main():
    torch.set_num_threads(THREADS)
    renv, rpol, ragent, rcb = import_reference()
    from safetensors.torch import load_file
    from oracle.net import state_dict_sha256
    from oracle.environment import MinitChessEpisode
    t0 = time.time()
    net = rpol.Network()
    net.load_state_dict(load_file(CKPT))
    net.eval()
    sha = state_dict_sha256(net)
    ends = endgame_starts(64, seed=44)
    g_start = ref_selfplay(renv, rpol, ragent, rcb, net, 64, [0])[0]
    print(f'game_start: {len(g_start["moves"])} plies, reward {g_start["moves"][-1]["reward"]} '
          f'({time.time() - t0:.0f} s)', flush=True)
    g_end = None
    for f in ends[:32]:
        try:
            g = ref_selfplay(renv, rpol, ragent, rcb, net, 64, [0], start_fen=f)[0]
        except renv.TerminatedEpisodeStepException:
            # the reference's search steps a finished episode from some starts (exp/agent.py:86 on a
            # position its environment calls over); such a start has no reference game
            print(f'game_end from {f}: the reference raised TerminatedEpisodeStepException', flush=True)
            continue
        print(f'game_end from {f}: {len(g["moves"])} plies, reward {g["moves"][-1]["reward"]}', flush=True)
        if g_end is None or (g['moves'][-1]['reward'] != 0 and g_end['moves'][-1]['reward'] == 0):
            g_end = g
        if g_end['moves'][-1]['reward'] != 0:
            break
    fens = []
    for m in g_start['moves'] + g_end['moves']:
        if m['observation'] not in fens:
            fens.append(m['observation'])
    for f in ends + sample_positions(64, seed=778):
        if f not in fens:
            fens.append(f)
    acts = []
    hooks = [m.register_forward_hook(lambda _m, _i, o: acts.append(float(o.detach().abs().max())))
             for m in net.resbody.modules() if type(m).__name__ in ('ConvBlock', 'ResidualBlock')]
    logits, values, spread, pmax = [], [], [], []
    with torch.no_grad():
        for f in fens:
            p, v = net(rpol.Network.process_observation(f))
            logits.append(p[0].numpy())
            values.append(float(v.item()))
            legal = MinitChessEpisode(f).get_legal_moves()
            if legal:
                lg = p[0][legal].double()
                spread.append(float(lg.max() - lg.min()))
                pmax.append(float(lg.softmax(0).max()))
    for h in hooks:
        h.remove()
    np.savez_compressed(os.path.join(HERE, 'stress4_net.npz'), fens=np.array(fens),
                        logits=np.stack(logits).astype(np.float32), values=np.array(values, dtype=np.float32))
    train = None
    if len(sys.argv) > 1:
        lines = [json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')]
        train = {'summary': lines[-1], 'iterations': [x for x in lines[:-1] if x.get('lr') == lines[-1].get('picked_lr')]}
    out = {'state_dict_sha256': sha, 'checkpoint': 'stress4/stress4.safetensors', 'training': train,
           'positions': len(fens), 'trunk_absmax': max(acts), 'legal_logit_spread_max': max(spread),
           'legal_logit_spread_median': float(np.median(spread)), 'max_prior_median': float(np.median(pmax)),
           'value_range': [float(min(values)), float(max(values))], 'value_std': float(np.std(values)),
           'torch_threads': THREADS, 'torch': torch.__version__, 'game_start': g_start, 'game_end': g_end}
    with open(os.path.join(HERE, 'stress4.json'), 'w') as fh:
        json.dump(out, fh, separators=(',', ':'))
    print(json.dumps({k: v for k, v in out.items() if k not in ('game_start', 'game_end', 'training')}),
          f'({time.time() - t0:.0f} s)')


if __name__ == '__main__':
    main()
