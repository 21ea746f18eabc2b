#!/usr/bin/env python3
"""Round-3 golden fixtures for the STRESS checkpoint, made by running the REFERENCE code on the CPU
(build container only; same stubs as make_golden.py: un-vendored erlyx, oracle.rules as `chess`).

The checkpoint (stress/stress.safetensors) is data: tools/train_stress.py trained it in the C5
self-play loop on one MI355X with the reference learner's update (exp/learner.py:72-94) for
>= 20 updates, to the regime the deployed learner drives toward (peaked priors, trunk
activations in the thousands).  This script pins it and records what the reference computes on it:

  stress.json        sha256 of the checkpoint (oracle.net.state_dict_sha256), the training recipe
                     and measurements (tools/train_stress.py output), the network's ranges on the
                     fixture positions (legal-logit spread, largest prior, trunk |activation| max,
                     measured with forward hooks on the reference modules), and 'stress_64': one
                     reference self-play game at 64 sims with the checkpoint (np.random.seed(0))
  stress_net.npz     the reference Network.forward (eval mode) on the fixture positions: the
                     positions of that game, then sample_positions(96, seed=777) (promotions with
                     repeated codes, mates, both colours): fens, logits [n, 554], values [n]

Usage: python tests/golden/make_golden_r3.py [path/to/train.jsonl]
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
from make_golden_r2 import ref_selfplay  # noqa: E402

THREADS = 8
CKPT = os.path.join(HERE, 'stress', 'stress.safetensors')


def main():
    torch.set_num_threads(THREADS)
    renv, rpol, ragent, rcb = import_reference()
    from safetensors.torch import load_file
    from oracle.net import state_dict_sha256
    t0 = time.time()
    net = rpol.Network()
    net.load_state_dict(load_file(CKPT))
    net.eval()
    sha = state_dict_sha256(net)
    game = ref_selfplay(renv, rpol, ragent, rcb, net, 64, [0])[0]
    print(f'stress_64: {len(game["moves"])} plies, reward {game["moves"][-1]["reward"]} ({time.time() - t0:.0f} s)',
          flush=True)
    fens = []
    for m in game['moves']:
        if m['observation'] not in fens:
            fens.append(m['observation'])
    for f in sample_positions(96, seed=777):
        if f not in fens:
            fens.append(f)
    acts = []
    hooks = [m.register_forward_hook(lambda _m, _i, o: acts.append(float(o.detach().abs().max())))
             for m in net.resbody.modules() if type(m).__name__ in ('ConvBlock', 'ResidualBlock')]
    logits, values, spread, pmax = [], [], [], []
    from oracle.environment import MinitChessEpisode
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
    np.savez_compressed(os.path.join(HERE, 'stress_net.npz'), fens=np.array(fens),
                        logits=np.stack(logits).astype(np.float32), values=np.array(values, dtype=np.float32))
    train = None
    if len(sys.argv) > 1:
        lines = [json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')]
        train = {'summary': lines[-1], 'iterations': [x for x in lines[:-1] if x.get('lr') == lines[-1].get('picked_lr')]}
    out = {'state_dict_sha256': sha, 'checkpoint': 'stress/stress.safetensors', 'training': train,
           'positions': len(fens), 'trunk_absmax': max(acts), 'legal_logit_spread_max': max(spread),
           'legal_logit_spread_median': float(np.median(spread)), 'max_prior_median': float(np.median(pmax)),
           'value_range': [float(min(values)), float(max(values))], 'torch_threads': THREADS,
           'torch': torch.__version__, 'stress_64': game}
    with open(os.path.join(HERE, 'stress.json'), 'w') as fh:
        json.dump(out, fh, separators=(',', ':'))
    print(json.dumps({k: v for k, v in out.items() if k not in ('stress_64', 'training')}), f'({time.time() - t0:.0f} s)')


if __name__ == '__main__':
    main()
