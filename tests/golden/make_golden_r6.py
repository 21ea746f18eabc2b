#!/usr/bin/env python3
"""Round-6 golden fixtures, made by running the REFERENCE code on the CPU (build container only; same
stubs as make_golden.py: un-vendored erlyx, oracle.rules as `chess`).

  trees_r6.json   'net_seed0_36': the reference's self-play with the seed-0 net (torch.manual_seed(0);
                  Network()) at the repo's default 36 sims per move (app/base.py:25), seeds 0-3
                  (np.random.seed(seed) per game, app/base.py:113-120 stack).  The bench's 36-sim
                  engine plays exactly these seeds as its games 0-3.
  stress6.json    VERDICT r5 next #2: stress6 = tools/make_stress6.py (stress4's trunk in 181x larger
                  units, a non-power-of-two gain: new significands).  sha256 of the state_dict, the
                  network's ranges on the fixture positions (trunk |activation| max via forward hooks
                  on the reference modules, legal-logit spread, value range and std), k_net_y's
                  emulated exponents (tools/net_range.py), and one reference self-play game at 64
                  sims from STARTING_FEN (np.random.seed(0)) as 'game_start'.
  stress6_net.npz the reference Network.forward (eval) on stress6 at the fixture positions: the
                  game's positions, stress4's fixture positions, then sample_positions(64, seed=781).
  wide_net.npz    the reference Network.forward (eval) on the 'wide' net of tests/test_gpu_net.py
                  (torch.manual_seed(0); Network(); both BatchNorm gammas of every residual block x 6,
                  trunk activations ~7e6) at tests_positions.random_fens(129, seed=9), plus the
                  state_dict sha256 (compare k_net_y with the reference, not with
                  torch-ROCm).

Usage: python tests/golden/make_golden_r6.py [seed0_36] [stress6] [wide]   (all by default)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tools'))
sys.path.insert(0, os.path.join(REPO, 'tests'))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from make_golden import import_reference, sample_positions  # noqa: E402
from make_golden_r2 import ref_selfplay  # noqa: E402

THREADS = 8


def forward_fixture(rpol, net, fens):
    """Reference outputs + ranges on `fens` (logits [n, 554] f32, values [n] f32)."""
    from oracle.environment import MinitChessEpisode
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
    logits = np.stack(logits).astype(np.float32)
    ranges = {'positions': len(fens), 'trunk_absmax': max(acts), 'legal_logit_spread_max': max(spread),
              'legal_logit_spread_median': float(np.median(spread)), 'max_prior_median': float(np.median(pmax)),
              'logit_absmax': float(np.abs(logits).max()), 'logits_finite': bool(np.isfinite(logits).all()),
              'value_range': [float(min(values)), float(max(values))], 'value_std': float(np.std(values))}
    return logits, np.array(values, dtype=np.float32), ranges


def main():
    parts = sys.argv[1:] or ['seed0_36', 'stress6', 'wide']
    torch.set_num_threads(THREADS)
    renv, rpol, ragent, rcb = import_reference()
    from oracle.net import state_dict_sha256
    t0 = time.time()

    if 'seed0_36' in parts:
        torch.manual_seed(0)
        net0 = rpol.Network().eval()
        games = ref_selfplay(renv, rpol, ragent, rcb, net0, 36, [0, 1, 2, 3])
        print(f'net_seed0_36: plies {[len(g["moves"]) for g in games]} ({time.time() - t0:.0f} s)', flush=True)
        with open(os.path.join(HERE, 'trees_r6.json'), 'w') as fh:
            json.dump({'net_seed0_36': games, 'net_sha256': state_dict_sha256(net0)}, fh, separators=(',', ':'))

    if 'stress6' in parts:
        from make_stress6 import GAIN, stress6_state_dict
        from net_range import fens_profile, summarize
        sd = stress6_state_dict()
        net = rpol.Network()
        net.load_state_dict(sd)
        net.eval()
        sha = state_dict_sha256(net)
        g_start = ref_selfplay(renv, rpol, ragent, rcb, net, 64, [0])[0]
        print(f'stress6 game_start: {len(g_start["moves"])} plies, reward {g_start["moves"][-1]["reward"]} '
              f'({time.time() - t0:.0f} s)', flush=True)
        fens = []
        for m in g_start['moves']:
            if m['observation'] not in fens:
                fens.append(m['observation'])
        for f in np.load(os.path.join(HERE, 'stress4_net.npz'))['fens']:
            if str(f) not in fens:
                fens.append(str(f))
        for f in sample_positions(64, seed=781):
            if f not in fens:
                fens.append(f)
        logits, values, ranges = forward_fixture(rpol, net, fens)
        np.savez_compressed(os.path.join(HERE, 'stress6_net.npz'), fens=np.array(fens), logits=logits, values=values)
        prof = fens_profile(sd, fens)
        xs = summarize(prof)
        xs['min_over_boards_of_max_exponent'] = int(prof['xs'].max(0).min())
        out = {'state_dict_sha256': sha, 'derivation': {'source': 'stress4/stress4.safetensors', 'gain': GAIN,
                                                        'recipe': 'tools/make_stress6.py (stress6_state_dict)'},
               **ranges, 'k_net_y_exponents': xs, 'torch_threads': THREADS, 'torch': torch.__version__,
               'game_start': g_start}
        with open(os.path.join(HERE, 'stress6.json'), 'w') as fh:
            json.dump(out, fh, separators=(',', ':'))
        print('stress6', json.dumps({k: v for k, v in out.items() if k not in ('game_start', 'k_net_y_exponents')}),
              json.dumps({k: v for k, v in xs.items() if k != 'per_layer'}), f'({time.time() - t0:.0f} s)', flush=True)

    if 'wide' in parts:
        from tests_positions import random_fens
        torch.manual_seed(0)
        net = rpol.Network()
        with torch.no_grad():
            for blk in list(net.resbody)[1:]:
                blk.convblock1.layers[1].weight.mul_(6.0)
                blk.convblock2.layers[1].weight.mul_(6.0)
        net.eval()
        fens = random_fens(129, seed=9)
        logits, values, ranges = forward_fixture(rpol, net, fens)
        np.savez_compressed(os.path.join(HERE, 'wide_net.npz'), fens=np.array(fens), logits=logits, values=values,
                            state_dict_sha256=np.array(state_dict_sha256(net)))
        print('wide', json.dumps(ranges), f'({time.time() - t0:.0f} s)', flush=True)


if __name__ == '__main__':
    main()
