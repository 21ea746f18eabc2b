"""Shared test drivers (TEST INFRASTRUCTURE).

drive_engine(): plays games on the GPU engine one MCTS move at a time, with the
reference agent's action selection and numpy RandomState(seed) per game
(exp/agent.py:110-119, :82) implemented here in Python.  Leaves are evaluated
either by the GPU network (evaluator=None) or by a host evaluator (oracle
SyntheticEvaluator / TorchNetEvaluator) so the device tree kernels can be pinned
bit-for-bit against the oracle independently of the network numerics.
"""
import numpy as np

from minitchess_alphazero_amd.environment import STARTING_FEN, pos_to_fen


def drive_engine(eng, n_games, sims, seeds, evaluator=None, tau=6, start_fen=STARTING_FEN, trees_out=None,
                 capture=None):
    """start_fen: one FEN for every game, or a list with one per game.  With the GPU network
    (evaluator=None) and a dict `capture`, each simulation runs as sim_select -> sim_evaluate ->
    sim_backup (the kernels of simulate()) and capture[fen] = (P, v) records the network's
    device-written leaf results."""
    starts = [start_fen] * n_games if isinstance(start_fen, str) else list(start_fen)
    eng.set_games(starts)
    eng.clear_trees()
    rngs = [np.random.RandomState(s) for s in seeds]
    recs = [[] for _ in range(n_games)]
    stats = {'nn_evals': 0, 'sims': 0}
    while True:
        pos, _ag, act, _oc = eng.games()
        if not act[:n_games].any():
            break
        k, new = eng.move_begin()
        noise = []
        for g in range(eng.G):
            if g < n_games and act[g] and sims - new[g] > 0:
                noise.append(np.stack([rngs[g].dirichlet([0.6] * int(k[g])) for _ in range(sims - int(new[g]))]))
            else:
                noise.append(None)
        eng.set_noise(noise)
        for s in range(sims):
            if evaluator is None and capture is not None:
                eng.sim_select(s)
                lpos, _lg, lk, _lc = eng.leaves()
                eng.sim_evaluate()
                P, v = eng.leaf_results()
                for i in range(len(lk)):
                    capture[pos_to_fen(lpos[i])] = (P[i][:lk[i]].copy(), float(v[i]))
                eng.sim_backup()
            elif evaluator is None:
                eng.simulate(s, 1)
            else:
                eng.sim_select(s)
                lpos, _lg, lk, lcodes = eng.leaves()
                P, v = [], []
                for i in range(len(lk)):
                    p, val = evaluator.evaluate(pos_to_fen(lpos[i]), [int(c) for c in lcodes[i][:lk[i]]])
                    P.append(np.asarray(p, np.float32))
                    v.append(val)
                stats['nn_evals'] += len(lk)
                eng.set_leaves(P, v)
                eng.sim_backup()
        codes, visits, _k = eng.move_end()
        actions = np.zeros(n_games, np.int32)
        for g in range(n_games):
            if not act[g]:
                continue
            kk = int(k[g])
            legal = [int(c) for c in codes[g][:kk]]
            N = visits[g][:kk].astype(np.float64)
            pi = N / N.sum()
            num_moves = int(pos[g][4]) >> 16
            if num_moves < tau:
                a = rngs[g].choice(legal, p=pi)
            else:
                maxima = np.where(pi == pi.max())[0]
                a = legal[rngs[g].choice(maxima)]
            actions[g] = int(a)
            recs[g].append({'observation': pos_to_fen(pos[g]), 'legal_moves': legal, 'pi': pi.tolist(),
                            'action': int(a)})
            stats['sims'] += sims
        eng.apply(actions)
    _pos, _ag, _act, oc = eng.games()
    for g in range(n_games):
        reward = 1.0 if oc[g] == 1 else 0.0
        for r in recs[g][::-1]:
            r['reward'] = reward
            reward = -reward
    if trees_out is not None:
        for g in range(n_games):
            trees_out.append((eng.tree(2 * g), eng.tree(2 * g + 1)))
    return recs, stats


def compare_records(got, ref):
    """-> (identical_moves, total_moves, first_mismatch or None)"""
    same, first = 0, None
    n = min(len(got), len(ref))
    for i in range(n):
        a, b = got[i], ref[i]
        ok = (a['observation'] == b['observation'] and list(a['legal_moves']) == list(b['legal_moves'])
              and a['pi'] == b['pi'] and a['action'] == b['action'])
        if ok:
            same += 1
        elif first is None:
            first = i
    if len(got) != len(ref) and first is None:
        first = n
    return same, max(len(got), len(ref)), first


def c3_network():
    """BASELINE config 3's checkpoint (tests/golden/make_golden_r2.py), sha256-checked."""
    import json
    import os
    from safetensors.torch import load_file
    from minitchess_alphazero_amd.network import Network
    from oracle.net import state_dict_sha256
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
    net = Network()
    net.load_state_dict(load_file(os.path.join(here, 'c3', 'c3.safetensors')))
    meta = json.load(open(os.path.join(here, 'c3.json')))
    assert state_dict_sha256(net) == meta['state_dict_sha256'], 'C3 checkpoint does not match its pinned sha256'
    return net.eval()


def stress_network(name='stress'):
    """A trained checkpoint of tests/golden/, sha256-checked against its pinned fixture json.
    'stress' (round 3, tools/train_stress.py, pinned by make_golden_r3.py): 21 reference-learner
    updates in the C5 loop at lr 0.02, trunk activations in the thousands, legal-logit spreads up
    to ~80 on its fixture positions, its value head collapsed to a constant.  'stress4' (round 4,
    pinned by make_golden_r4.py): 20 updates at lr 0.003 with half the games from endgame starts,
    a value head whose outputs vary (-0.26 .. 0.33 on its fixture positions).  'stress5' (round 5,
    tools/make_stress5.py, pinned by make_golden_r5.py): stress4 with its residual trunk in 2^7
    larger units, an exact reparametrisation (the reference's outputs are stress4's bit for bit)
    that puts k_net_y's per-board exponents at 1-4 on every fixture position."""
    import json
    import os
    from safetensors.torch import load_file
    from minitchess_alphazero_amd.network import Network
    from oracle.net import state_dict_sha256
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
    net = Network()
    if name == 'stress6':
        # stress6 (round 6, tools/make_stress6.py, pinned by make_golden_r6.py): stress4 with its trunk in
        # 181x larger units, a non-power-of-two gain (new significands), rebuilt from the committed
        # stress4 and checked against its pinned sha256 below
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(here), '..', 'tools'))
        from make_stress6 import stress6_state_dict
        net.load_state_dict(stress6_state_dict())
    else:
        net.load_state_dict(load_file(os.path.join(here, name, f'{name}.safetensors')))
    meta = json.load(open(os.path.join(here, f'{name}.json')))
    assert state_dict_sha256(net) == meta['state_dict_sha256'], f'{name} checkpoint does not match its pinned sha256'
    return net.eval()


class RecordedEvaluator:
    """Oracle evaluator returning recorded leaf results by FEN (the network is a function of the
    position, so a replay asks only for positions the recorded run evaluated)."""

    def __init__(self, table):
        self.table = table

    def evaluate(self, fen, legal_moves):
        P, v = self.table[fen]
        assert len(P) == len(legal_moves), fen
        return np.asarray(P, np.float32), v


class _LoggingEvaluator:
    """Wraps an oracle evaluator; logs (fen, P, v, number of PUCT selections so far)."""

    def __init__(self, inner, trace):
        self.inner, self.trace, self.log = inner, trace, []

    def evaluate(self, fen, legal_moves):
        P, v = self.inner.evaluate(fen, legal_moves)
        self.log.append((fen, np.asarray(P, np.float64), float(v), len(self.trace)))
        return P, v


def explain_divergence(gpu_leaves, ref_evaluator, sims, seed, gpu_moves, bound_scale=1.0):
    """Why a GPU-network game left the reference game.  Two oracle replays of game `seed`, one with
    the GPU's recorded leaf results (it must reproduce the GPU game exactly) and one with the
    reference network, record every PUCT selection; the first selection where they differ is the
    flip.  Until then both replays expanded the same leaves in the same order with the same
    Dirichlet draws, so the only differences are the leaf results themselves: dP = the largest
    |P_gpu - P_ref| and dv = the largest |v_gpu - v_ref| over the leaves evaluated before the flip,
    MEASURED on this game.  They move u = Q + cpuct*P'*sqrt(S)/(1+N) of a child by at most
    dv + dP*sqrt(S) (Q averages backed-up leaf values; the root mix scales P by 0.75), so the flip
    is explained when the reference margin (u of its choice - u of the GPU's choice) plus the GPU
    run's opposite margin is at most 2*(dv + dP*sqrt(S)) (+1e-12 for the rounding of u itself).
    Returns both margins, dP, dv, the bound, and the bound the 1e-5 north_star tolerance would give.
    bound_scale < 1 shrinks the measured bound (tests/test_explain_cpu.py: the bound is not loose)."""
    from oracle import selfplay
    tr_gpu, tr_ref = [], []
    rec_gpu = selfplay.play_games(RecordedEvaluator(gpu_leaves), 1, sims, seed_base=seed, trace=tr_gpu)[0]
    same, _total, first = compare_records(rec_gpu, gpu_moves)
    assert first is None, f'the oracle replay of the GPU leaves left the GPU game at ply {first}'
    ref_log = _LoggingEvaluator(ref_evaluator, tr_ref)
    selfplay.play_games(ref_log, 1, sims, seed_base=seed, trace=tr_ref)
    for i, (a, b) in enumerate(zip(tr_ref, tr_gpu)):
        if a[0] != b[0] or a[2] != b[2]:
            assert a[0] == b[0], 'the replays reached different nodes without a differing selection'
            u_ref, u_gpu, ar, ag = a[1], b[1], a[2], b[2]
            S = a[3]
            m_ref = float(u_ref[ar] - u_ref[ag])
            m_gpu = float(u_gpu[ag] - u_gpu[ar])
            dP = dv = 0.0
            n_leaves = 0
            for fen, P_ref, v_ref, t in ref_log.log:
                if t > i:
                    break
                P_gpu, v_gpu = gpu_leaves[fen]
                dP = max(dP, float(np.max(np.abs(np.asarray(P_gpu, np.float64) - P_ref))) if len(P_ref) else 0.0)
                dv = max(dv, abs(float(v_gpu) - v_ref))
                n_leaves += 1
            bound = bound_scale * 2 * (dv + dP * np.sqrt(S)) + 1e-12
            return {'selection': i, 'node': a[0], 'ref_choice': ar, 'gpu_choice': ag, 'visits_at_node': S,
                    'margin_ref': m_ref, 'margin_gpu': m_gpu, 'leaves_before_flip': n_leaves,
                    'max_dP': dP, 'max_dv': dv, 'measured_bound': float(bound),
                    'tolerance_bound_1e-5': float(2 * (1e-5 + 1e-5 * np.sqrt(S))),
                    'explained': bool(m_ref >= 0 and m_gpu >= 0 and m_ref + m_gpu <= bound)}
    return None
