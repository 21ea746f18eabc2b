"""GPU: the reference plugin surface (erlyx run_episodes + RoundRobinReferee +
SimpleAlphaZeroAgent + SimpleAlphaZeroPolicy + InfoRecorder + MonteCarloInit, global
np.random) over the HIP engine, vs the batched engine (mtaz_play) on the same seed,
and the SimulatePuppet MQTT payloads (app/base.py:52-70)."""
import json

import numpy as np
import pytest

from helpers import compare_records

pytestmark = pytest.mark.gpu


def _reference_shaped_game(net, sims, seed):
    from minitchess_alphazero_amd import erlyx_compat
    from minitchess_alphazero_amd.agent import RoundRobinReferee, SimpleAlphaZeroAgent
    from minitchess_alphazero_amd.callbacks import InfoRecorder, MonteCarloInit
    from minitchess_alphazero_amd.environment import MinitChessEnvironment
    from minitchess_alphazero_amd.policy import SimpleAlphaZeroPolicy

    class DS:
        def __init__(self):
            self.episodes = []

        def push(self, ep):
            self.episodes.append(ep)

    env = MinitChessEnvironment()
    policy = SimpleAlphaZeroPolicy(network=net)
    agents = [SimpleAlphaZeroAgent(env, policy, sims) for _ in range(2)]
    ds = DS()
    cbs = [InfoRecorder(ds), MonteCarloInit(agents[0]), MonteCarloInit(agents[1])]
    np.random.seed(seed)
    erlyx_compat.run_episodes(env, RoundRobinReferee(agents), 1, callbacks=cbs)
    return ds.episodes[0]


def test_dropin_stack_equals_batched_engine():
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    sims, seed = 12, 21
    a = _reference_shaped_game(net, sims, seed)
    eng = Engine(n_games=1, sims=sims, seed_base=seed)
    eng.set_weights(net)
    eng.play()
    b = eng.episodes()[0]
    assert compare_records(a, b)[2] is None
    assert [r['reward'] for r in a] == [r['reward'] for r in b]


def test_mcts_view_matches_reference_layout():
    import torch
    from minitchess_alphazero_amd.agent import MonteCarloTreeSearch
    from minitchess_alphazero_amd.environment import MinitChessEnvironment, STARTING_FEN
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    m = MonteCarloTreeSearch(MinitChessEnvironment(), Network(), 1)
    np.random.seed(0)
    data = m.simulate(16, STARTING_FEN)
    assert STARTING_FEN in data['visited']
    assert data['N'][STARTING_FEN].sum() == 15          # first sim expands the root
    assert len(data['P'][STARTING_FEN]) == len(data['legal_moves'][STARTING_FEN])
    assert abs(float(np.sum(data['P'][STARTING_FEN])) - 1.0) < 1e-5
    m.simulate(16, STARTING_FEN)                        # table persists across calls
    assert m['N'][STARTING_FEN].sum() == 31


def test_puppet_publishes_reference_payloads():
    from minitchess_alphazero_amd import puppet as pp

    class Client:
        def __init__(self):
            self.msgs = []

        def publish(self, topic, payload, qos=0):
            self.msgs.append((topic, json.loads(payload), qos))

            class I:
                mid = len(self.msgs)
            return I()

    pp.MINITCHESS_ALPHAZERO_VERSION = 'v-test'
    p = pp.SimulatePuppet('u1', 'topic/eps', num_simulations=8)
    p.remote_status = pp.MasterOfPuppetsStatus.SIMULATE
    p.remote_version = 'v-test'
    c = Client()
    np.random.seed(3)
    p.run_episodes(3, c)
    assert len(c.msgs) == 3 and not p.is_simulating()
    topic, msg, qos = c.msgs[0]
    assert topic == 'topic/eps' and qos == 2
    assert set(msg) == {'episode', 'userid', 'weights_version', 'minitchess_alphazero_version'}
    step = msg['episode'][0]
    assert list(step) == ['observation', 'legal_moves', 'pi', 'action', 'reward']
    assert step['observation'] == '2nbk/2ppp/5/5/PPP2/KBN2 w 0 1'
    # gate: wrong status -> nothing published (app/base.py:53-57)
    p.remote_status = pp.MasterOfPuppetsStatus.TRAIN
    p.run_episodes(1, c)
    assert len(c.msgs) == 3
