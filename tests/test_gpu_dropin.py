"""GPU: the reference plugin surface (erlyx run_episodes + RoundRobinReferee +
SimpleAlphaZeroAgent + SimpleAlphaZeroPolicy + InfoRecorder + MonteCarloInit, global
np.random) over the HIP engine, vs the batched engine (mtaz_play) on the same seed,
and the SimulatePuppet MQTT payloads (app/base.py:52-70)."""
import json

import numpy as np
import pytest

from conftest import load_golden
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


def test_mcts_grows_for_more_simulations():
    """A later simulate() may ask for more simulations than the first (exp/agent.py:41-45 has no
    limit): the table moves into a larger engine (mtaz_tree_set) and the search continues exactly
    as in a tree sized for the larger count from the start."""
    import torch
    from minitchess_alphazero_amd.agent import MonteCarloTreeSearch
    from minitchess_alphazero_amd.environment import MinitChessEnvironment, STARTING_FEN, pos_step, pos_from_fen, pos_to_fen
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    fen2 = pos_to_fen(pos_step(pos_from_fen(STARTING_FEN), int(MinitChessEnvironment().new_episode()[0].get_legal_moves()[0])))
    views = []
    for cap in (None, 40):
        m = MonteCarloTreeSearch(MinitChessEnvironment(), net, 1, capacity=cap)
        np.random.seed(5)
        m.simulate(8, STARTING_FEN)
        m.simulate(40, fen2)                       # regrows when capacity is None
        m.simulate(24, STARTING_FEN)
        st = np.random.get_state()
        views.append((m._data, (st[1].tobytes(), st[2])))
    (a, pa), (b, pb) = views
    assert pa == pb                                # same np.random consumption
    assert a['visited'] == b['visited'] and a['terminal'] == b['terminal']
    for fen in b['Q']:
        assert a['legal_moves'][fen] == b['legal_moves'][fen]
        assert np.array_equal(a['N'][fen], b['N'][fen]) and np.array_equal(a['Q'][fen], b['Q'][fen]), fen
        assert np.array_equal(a['P'][fen], b['P'][fen]), fen


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


def test_tree_set_spills_to_the_edge_pool():
    """mtaz_tree_set places a table's edges like k_select does: in the table's own region while
    whole nodes fit, the rest in the shared pool (it used to fail with E_CAPACITY beyond
    the region).  A searched table moved into an engine whose per-table region is far too small
    reads back identically and searches on exactly like the original."""
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import STARTING_FEN
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    engs = []
    for per_tree in (None, 24):
        e = Engine(n_games=1, sims=64)
        e.set_weights(net)
        if per_tree:
            e.set_edge_capacity(per_tree, 1 << 20)
        e.set_games([STARTING_FEN])
        e.clear_trees()
        engs.append(e)
    a, b = engs
    k, new = a.move_begin()
    rng = np.random.RandomState(1)
    noise = [np.stack([rng.dirichlet([0.6] * int(k[0])) for _ in range(64 - int(new[0]))])]
    a.set_noise(noise)
    a.simulate(0, 40)
    ta = a.tree_arrays(0)
    assert int(ta['k'][:ta['n']].astype(np.int64).sum()) > 24     # more edges than b's region
    b.set_tree(0, ta)
    tb = b.tree_arrays(0)
    for key in ('pos', 'e0', 'k', 'term', 'tval', 'codes', 'P', 'Q', 'N'):
        assert np.array_equal(ta[key], tb[key]), key
    kb, newb = b.move_begin()
    assert int(kb[0]) == int(k[0]) and int(newb[0]) == 0      # b finds the root in the moved table
    # simulation s reads draw s - root_new: a's draw s - 1 is b's draw s
    b.set_noise([np.concatenate([noise[0][:1], noise[0]])])
    a.simulate(40, 24)
    b.simulate(40, 24)
    ta, tb = a.tree_arrays(0), b.tree_arrays(0)
    for key in ('pos', 'e0', 'k', 'term', 'tval', 'codes', 'P', 'Q', 'N'):
        assert np.array_equal(ta[key], tb[key]), key


class _Client:
    def __init__(self):
        self.msgs = []

    def publish(self, topic, payload, qos=0):
        self.msgs.append((topic, json.loads(payload), qos))

        class I:
            mid = len(self.msgs)
        return I()


def test_puppet_global_stream_plays_the_reference_sequence():
    """rng_stream='global' (VERDICT r3 #5): the episodes come out in the reference's order, every
    draw from the one global np.random stream (app/base.py:113-120: episodes in sequence, the
    referee's turn carried over).  Episode 1 after np.random.seed(s) is the game the batched engine
    plays for seed s; episode 2 continues the stream (it is the drop-in stack's second episode, not
    a reseeded game); the stream is left exactly where that run leaves it; the payloads carry the
    reference's MQTT fields."""
    import torch
    from minitchess_alphazero_amd import erlyx_compat, puppet as pp
    from minitchess_alphazero_amd.agent import RoundRobinReferee, SimpleAlphaZeroAgent
    from minitchess_alphazero_amd.callbacks import InfoRecorder, MonteCarloInit
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import MinitChessEnvironment
    from minitchess_alphazero_amd.network import Network
    from minitchess_alphazero_amd.policy import SimpleAlphaZeroPolicy
    pp.MINITCHESS_ALPHAZERO_VERSION = 'v-test'
    sims, seed = 8, 11
    torch.manual_seed(0)
    net = Network()
    p = pp.SimulatePuppet('u1', 'topic/eps', num_simulations=sims, rng_stream='global')
    p.load_weights(net.state_dict(), 'w1')
    p.remote_status = pp.MasterOfPuppetsStatus.SIMULATE
    p.remote_version = 'v-test'
    c = _Client()
    np.random.seed(seed)
    p.run_episodes(2, c)
    st_puppet = np.random.get_state()
    assert len(c.msgs) == 2 and not p.is_simulating()
    assert all(m[1]['weights_version'] == 'w1' and m[1]['userid'] == 'u1' for m in c.msgs)
    eps = [m[1]['episode'] for m in c.msgs]

    eng = Engine(n_games=1, sims=sims, seed_base=seed)
    eng.set_weights(net)
    eng.play()
    assert compare_records(eps[0], eng.episodes()[0])[2] is None

    class DS:
        def __init__(self):
            self.episodes = []

        def push(self, ep):
            self.episodes.append(ep)

    env = MinitChessEnvironment()
    policy = SimpleAlphaZeroPolicy(network=net)
    agents = [SimpleAlphaZeroAgent(env, policy, sims) for _ in range(2)]
    ds = DS()
    np.random.seed(seed)
    erlyx_compat.run_episodes(env, RoundRobinReferee(agents), 2,
                              callbacks=[InfoRecorder(ds), MonteCarloInit(agents[0]), MonteCarloInit(agents[1])])
    st_direct = np.random.get_state()
    assert compare_records(eps[1], ds.episodes[1])[2] is None
    assert [r['reward'] for r in eps[1]] == [r['reward'] for r in ds.episodes[1]]
    assert st_puppet[1].tobytes() == st_direct[1].tobytes() and st_puppet[2] == st_direct[2]
    eng2 = Engine(n_games=1, sims=sims, seed_base=seed + 1)
    eng2.set_weights(net)
    eng2.play()
    assert compare_records(eps[1], eng2.episodes()[0])[2] is not None    # not a reseeded game


def test_puppet_global_stream_equals_the_reference_fixture():
    """VERDICT r4 missing #5, pinned to the reference: the drop-in SimulatePuppet with
    rng_stream='global', after ONE np.random.seed(11), plays exactly the two consecutive episodes
    the reference's own exp/* stack played that way (tests/golden/stream.json,
    make_golden_r5_stream.py: app/base.py:108-124's sequence, referee turn carried over), every
    observation, legal list, pi, action and reward, on the GPU engine (k_net_y leaves), and leaves
    the global RandomState where the reference left it."""
    import hashlib
    import torch
    from minitchess_alphazero_amd import puppet as pp
    from minitchess_alphazero_amd.network import Network
    fx = load_golden('stream')
    pp.MINITCHESS_ALPHAZERO_VERSION = 'v-test'
    torch.manual_seed(0)
    net = Network()
    p = pp.SimulatePuppet('u1', 'topic/eps', num_simulations=fx['sims'], rng_stream='global')
    p.load_weights(net.state_dict(), 'w1')
    p.remote_status = pp.MasterOfPuppetsStatus.SIMULATE
    p.remote_version = 'v-test'
    c = _Client()
    np.random.seed(fx['seed'])
    p.run_episodes(len(fx['episodes']), c)
    st = np.random.get_state()
    eps = [m[1]['episode'] for m in c.msgs]
    assert len(eps) == len(fx['episodes'])
    for got, ref in zip(eps, fx['episodes']):
        assert compare_records(got, ref)[2] is None
        assert [r['reward'] for r in got] == [r['reward'] for r in ref]
    assert hashlib.sha256(st[1].tobytes()).hexdigest() == fx['rng_after']['key_sha256']
    assert int(st[2]) == fx['rng_after']['pos']
