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


def drive_engine(eng, n_games, sims, seeds, evaluator=None, tau=6, start_fen=STARTING_FEN, trees_out=None):
    eng.set_games([start_fen] * n_games)
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
            if evaluator is None:
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
