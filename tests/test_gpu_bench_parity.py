"""The benched workload itself against the reference.

bench.py's main line is Engine(4096 games, 64 sims, seed_base 0) with the seed-0 net
(torch.manual_seed(0); Network()), k_net_y, the batch memo (2), deferred tails (1) and the device
RNG; its games 0-3 are np.random.seed(0..3) games, exactly the reference's own self-play games in
trees_r2.json 'net_seed0_64' (tests/golden/make_golden_r2.py).  The same engine configuration at the
repo's default 36 sims (app/base.py:25) plays the reference's 'net_seed0_36' games
(tests/golden/make_golden_r6.py), and at BASELINE config 1's 32 sims trees.json 'net_seed0' (seed 0).
Every ply must be identical: observation, legal list, pi, action, reward."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
CASES = {64: ('trees_r2.json', 'net_seed0_64'), 36: ('trees_r6.json', 'net_seed0_36'), 32: ('trees.json', 'net_seed0')}


def _bench_engine(sims, rng_device=1):
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    eng = Engine(n_games=4096, sims=sims, seed_base=0)
    torch.manual_seed(0)
    eng.set_weights(Network())
    eng.set_precision('f16x3')
    eng.set_memo(2)
    eng.set_defer(2)
    eng.set_rng_device(rng_device)
    return eng


def _compare(eng, games):
    got = eng.episodes(len(games))
    rows = []
    for g, ref in enumerate(games):
        assert ref['seed'] == g
        same = sum(1 for a, b in zip(got[g], ref['moves'])
                   if a['observation'] == b['observation'] and a['legal_moves'] == b['legal_moves']
                   and a['pi'] == b['pi'] and a['action'] == b['action'] and a['reward'] == b['reward'])
        rows.append((g, same, len(ref['moves']), len(got[g])))
    return rows


@pytest.mark.parametrize('sims', [64, 36, 32])
def test_benched_workload_games_equal_reference(sims):
    fixture, key = CASES[sims]
    games = json.load(open(os.path.join(GOLDEN, fixture)))[key]
    eng = _bench_engine(sims)
    st = eng.play()
    assert st['rng_device'] == 1 and st['net_precision'] == 1
    rows = _compare(eng, games)
    print(f'{sims} sims, 4096 games: games 0-{len(games) - 1} vs {fixture}:{key}: {rows}; '
          f'waves {st["waves"]:.0f} (extra {st["extra_waves"]:.0f}), memo hits {st["memo_hits"]:.0f}')
    for g, same, n_ref, n_got in rows:
        assert same == n_ref == n_got, (g, same, n_ref, n_got)
    eng.close()


def test_benched_workload_host_rng_36_sims():
    """The same at 36 sims with the host RNG (mtaz_set_rng_device(0))."""
    games = json.load(open(os.path.join(GOLDEN, 'trees_r6.json')))['net_seed0_36']
    eng = _bench_engine(36, rng_device=0)
    st = eng.play()
    assert st['rng_device'] == 0
    for g, same, n_ref, n_got in _compare(eng, games):
        assert same == n_ref == n_got, (g, same, n_ref, n_got)
    eng.close()
