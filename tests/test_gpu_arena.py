"""GPU: two-network play and the arena (commented exp/learner.py:97-145)."""
import numpy as np
import pytest

from helpers import compare_records

pytestmark = pytest.mark.gpu


def _nets():
    import torch
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    a = Network()
    torch.manual_seed(1)
    b = Network()
    return a, b


def test_two_network_play_matches_oracle_pair():
    """Agent 0 searches with net A, agent 1 with net B: the engine's games equal the oracle's
    games driven by the pair (TorchNetEvaluator(A), TorchNetEvaluator(B)): every ply identical
    (L3 with the default k_net_y; rounds 1-2 allowed a late near-tie flip after ply 10)."""
    from minitchess_alphazero_amd.engine import Engine
    from oracle.mcts import TorchNetEvaluator
    from oracle import selfplay
    from oracle.net import Network as ONet
    a, b = _nets()
    eng = Engine(n_games=2, sims=8, seed_base=0)
    eng.set_weights(a, slot=0)
    eng.set_weights(b, slot=1)
    eng.set_agent_networks(0, 1)
    eng.play()
    got = eng.episodes()
    oa, ob = ONet(), ONet()
    oa.load_state_dict(a.state_dict())
    ob.load_state_dict(b.state_dict())
    pair = (TorchNetEvaluator(oa.eval()), TorchNetEvaluator(ob.eval()))
    for g in range(2):
        ref = selfplay.play_games(pair, 1, 8, seed_base=g)[0]
        same, total, first = compare_records(got[g], ref)
        assert first is None, (g, same, total, first)
    # and it is not self-play of A
    eng.set_agent_networks(0, 0)
    eng.play()
    assert any(compare_records(x, y)[2] is not None for x, y in zip(eng.episodes(), got))


def test_arena_counts_and_winner_rule():
    from minitchess_alphazero_amd.arena import DECISIVE, arena, winners
    from minitchess_alphazero_amd.engine import Engine
    a, b = _nets()
    eng = Engine(n_games=8, sims=8)
    res = arena(eng, a, b, seed_base=3)
    assert res['games'] == 16 and res['new_wins'] + res['old_wins'] + res['draws'] == 16
    assert 0.0 <= res['score'] <= 1.0
    # winners() == WinnerRecorder on the episode rewards: decisive iff the last reward != 0
    eng.set_weights(a)
    eng.set_weights(b, slot=1)
    eng.set_agent_networks(0, 1)
    eng.play()
    w = winners(eng.records())
    eps = eng.episodes()
    ref = {False: 0, True: 0}
    for ep in eps:
        if ep[-1]['reward'] != 0:
            ref[bool((len(ep) - 1) % 2)] += 1
    assert w == ref
    eng.set_agent_networks(0, 0)
