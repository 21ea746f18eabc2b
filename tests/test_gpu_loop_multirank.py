"""GPU: BASELINE config 5 (self-play -> learner -> weights) across ranks, world sizes 2 and 8.

Two ranks started as bench.py --gpus N starts them (minitchess_alphazero_amd.launch), both on cuda:0
of the one-GPU box, gloo for the exchange (records gathered to rank 0, one flat weight broadcast).
Games shard by global id, so two ranks of G games play exactly the games one process plays with 2G,
the learner on rank 0 sees the same rows in the same order, and under deterministic algorithms the
two runs must end with bitwise-identical weights after every iteration's broadcast."""
import json
import os
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('world', [2, 8])
def test_loop_ranks_equal_one_process(tmp_path, world):
    """World 2, and world 8 (config 5's rank count in miniature, eight ranks on the one GPU)."""
    import torch
    from minitchess_alphazero_amd.launch import spawn_ranks
    from minitchess_alphazero_amd.loop import flat_weights, run_loop
    G, sims, iters = 8, 8, 2
    out = str(tmp_path / 'loop.json')
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    rc = spawn_ranks(world, [sys.executable, os.path.join(REPO, 'tests', 'rank_worker_loop.py'), out, str(G), str(sims),
                         str(iters)], env=env)
    assert rc == 0
    res = json.load(open(out))
    prev = (torch.are_deterministic_algorithms_enabled(), torch.backends.cudnn.deterministic,
            torch.backends.cudnn.benchmark)
    torch.use_deterministic_algorithms(True)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        hist, net = run_loop(iters, world * G, sims, batch_size=16, dist=None, device=0, seed=0, log=lambda s: None)
    finally:
        torch.use_deterministic_algorithms(prev[0])
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev[1], prev[2]
    flat, _ = flat_weights(net, 'cpu')
    assert len(res['history']) == iters
    for a, b in zip(res['history'], hist):
        assert a['games'] == b['games'] == world * G
        assert a['rows'] == b['rows']          # (weights_version is a timestamp, app/base.py)
        assert a['loss'] == b['loss'], (a['loss'], b['loss'])
    assert res['head'] == flat[:2000].tolist() and res['tail'] == flat[-2000:].tolist()
    assert res['sum'] == flat.double().sum().item()


@pytest.mark.parametrize('gate', [2.0, -1.0])
def test_loop_arena_gating_two_ranks(tmp_path, gate):
    """C5 with gating (arena_games > 0) at world 2: both ranks play their arena shard,
    the counts are all-reduced, and both keep or revert alike.  gate 2.0 can never pass (score <= 1):
    every update is reverted, so both ranks end on the initial weights (torch.manual_seed(0);
    Network()) bitwise.  gate -1.0 always passes: both ranks end on the same trained weights, which
    differ from the initial ones."""
    import torch
    from minitchess_alphazero_amd.launch import spawn_ranks
    from minitchess_alphazero_amd.loop import flat_weights
    from minitchess_alphazero_amd.network import Network
    G, sims, iters, arena_games = 4, 4, 2, 2
    out = str(tmp_path / 'loop.json')
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    rc = spawn_ranks(2, [sys.executable, os.path.join(REPO, 'tests', 'rank_worker_loop.py'), out, str(G), str(sims),
                         str(iters), str(arena_games), str(gate)], env=env)
    assert rc == 0
    res = json.load(open(out))
    r0, r1 = (json.load(open(f'{out}.rank{r}')) for r in (0, 1))
    assert r0 == r1                                   # same weights on both ranks, bitwise
    assert len(res['history']) == iters
    for h in res['history']:
        a = h['arena']
        assert a['games'] == 2 * 2 * arena_games      # both ranks' games, both sides
        assert a['accepted'] == (gate < 0)
    torch.manual_seed(0)
    init, _ = flat_weights(Network(), 'cpu')
    same_as_init = r0['head'] == init[:2000].tolist() and r0['tail'] == init[-2000:].tolist()
    assert same_as_init == (gate > 1)
