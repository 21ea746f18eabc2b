"""GPU: the search's own inputs and outputs vs the reference, through the C ABI.

  * leaf priors / values: what the fused network writes for the search (D.lf.P, D.lf.v: the legal
    softmax of exp/agent.py:67-68 over the node's legal list, repeated promotion codes included,
    and v.item() of :69) vs the reference's softmax over its own logits, <= 1e-5 (north_star)
  * L3: self-play with the GPU network end to end vs the reference's games (every pi, action and
    reward), seed-0 net at 32 and 64 sims and the C3 net at 256.  Bit-exact move selection is the
    target; a game may leave the reference game only at a near-tie that the leaf deviations
    MEASURED on that game can flip: at the first PUCT selection where an oracle replay of the GPU's
    own leaf results differs from the reference replay, the two margins must sum to at most
    2 (dv + dP sqrt(S)), dP and dv the largest prior and value deviations of the leaves evaluated
    before it (helpers.explain_divergence).  Identity rates, every divergence's margins and its
    measured dP, dv are written to gpurun_out/l3_identity.json
  * the terminal-revisit quirk (exp/agent.py:57-63 vs :75-77) through k_select
  * decisive games (reward back-fill, exp/callbacks.py:49-54; terminal handling) on the GPU
  * BASELINE config 3: the pinned trained checkpoint (tests/golden/make_golden_r2.py): network
    parity, the reference's 256-sim game bit-exact, and a 4096 x 256 play() within capacity
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, REPO, load_golden
from helpers import c3_network, compare_records, drive_engine, explain_divergence
from minitchess_alphazero_amd.environment import STARTING_FEN

pytestmark = pytest.mark.gpu

PRIOR_TOL = 1e-5
VALUE_TOL = 1e-5
PRECISIONS = ['f16f8', 'f16x3']


def _engine(n_games, sims, **kw):
    from minitchess_alphazero_amd.engine import Engine
    return Engine(n_games=n_games, sims=sims, **kw)


def _seed0_network():
    import torch
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    return Network()


def _write_result(name, obj):
    out = os.path.join(REPO, 'gpurun_out')
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, 'l3_identity.json')
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[name] = obj
    with open(path, 'w') as fh:
        json.dump(data, fh, indent=1)


# ---- leaf priors / values the search consumes ------------------------------------------------

@pytest.mark.parametrize('precision', PRECISIONS)
@pytest.mark.parametrize('weights', ['seed0', 'c3'])
def test_leaf_priors_and_values_vs_reference(precision, weights):
    """Every fixture position as a root: sim 0 expands it, the network writes its priors and value
    for the search.  Reference: softmax (torch float32) over the reference's own logits gathered at
    the legal list (exp/agent.py:67-68), and its value (:69)."""
    import torch
    from minitchess_alphazero_amd.environment import pos_from_fen, pos_legal, pos_outcome
    z = np.load(os.path.join(GOLDEN, 'net.npz' if weights == 'seed0' else 'c3_net.npz'))
    fens = [str(f) for f in z['fens']]
    roots = [i for i, f in enumerate(fens) if pos_legal(pos_from_fen(f)) and pos_outcome(pos_from_fen(f)) == 0]
    eng = _engine(len(roots), 4)
    eng.set_precision(precision)
    eng.set_weights(_seed0_network() if weights == 'seed0' else c3_network())
    eng.set_games([fens[i] for i in roots])
    eng.clear_trees()
    eng.move_begin()
    eng.set_noise([None] * eng.G)
    eng.sim_select(0)
    _lpos, lgame, lk, lcodes = eng.leaves()
    assert len(lgame) == len(roots)
    eng.sim_evaluate()
    P, v = eng.leaf_results()
    dup = 0
    worst_p = worst_v = 0.0
    for i in range(len(lgame)):
        j = roots[int(lgame[i])]
        legal = [int(c) for c in lcodes[i][:lk[i]]]
        assert legal == pos_legal(pos_from_fen(fens[j]))
        dup += len(set(legal)) < len(legal)
        ref = torch.from_numpy(z['logits'][j])[legal].softmax(0).numpy()
        worst_p = max(worst_p, float(np.max(np.abs(P[i][:len(legal)].astype(np.float64) - ref))))
        worst_v = max(worst_v, abs(float(v[i]) - float(z['values'][j])))
    print(f'{weights} {precision}: leaves {len(lgame)} (repeated promotion codes in {dup}), '
          f'max |P - ref| {worst_p:.3e}, max |v - ref| {worst_v:.3e}')
    assert dup > 0, 'the fixture must cover legal lists with repeated promotion codes'
    assert worst_p <= PRIOR_TOL
    assert worst_v <= VALUE_TOL
    eng.sim_backup()


# ---- L3: GPU network end to end == the reference's games -------------------------------------

def _l3(name, precision, net, ref_net, games):
    """GPU-network games vs the reference games; every divergence must be an explained near-tie."""
    from oracle.mcts import TorchNetEvaluator
    sims = games[0]['sims']
    eng = _engine(len(games), sims)
    eng.set_precision(precision)
    eng.set_weights(net)
    leaves = {}
    starts = [g.get('start') or STARTING_FEN for g in games]
    recs, _ = drive_engine(eng, len(games), sims, [g['seed'] for g in games], evaluator=None, capture=leaves,
                           start_fen=starts)
    rows = []
    for got, gm in zip(recs, games):
        same, total, first = compare_records(got, gm['moves'])
        row = {'seed': gm['seed'], 'identical_plies': same, 'plies': total, 'first_divergence': first}
        if first is not None:
            row['flip'] = explain_divergence(leaves, TorchNetEvaluator(ref_net), sims, gm['seed'], got)
        else:
            assert [x['reward'] for x in got] == [x['reward'] for x in gm['moves']]
        rows.append(row)
    _write_result(f'{name}/{precision}', rows)
    print(name, precision, rows)
    for r in rows:
        if r['first_divergence'] is not None:
            assert r['flip'] is not None and r['flip']['explained'], r


@pytest.mark.parametrize('precision', PRECISIONS)
@pytest.mark.parametrize('trace', ['net_seed0_32', 'net_seed0_64'])
def test_gpu_net_games_equal_reference(precision, trace):
    from oracle.net import seed0_network
    games = (load_golden('trees')['net_seed0'] if trace == 'net_seed0_32'
             else load_golden('trees_r2')['net_seed0_64'])
    _l3(trace, precision, _seed0_network(), seed0_network(), games)


# ---- terminal-revisit quirk through k_select ------------------------------------------------

def test_terminal_revisit_quirk_on_gpu():
    """quirk.json (the reference's MonteCarloTreeSearch.simulate(1, fen) x 40 after
    np.random.seed(0), synthetic evaluator): the root's Q after every simulation, bit-exact.  The
    mating edge goes +1 -> 0 -> -1/3 (exp/agent.py:57-63, then :75-77 backs up -terminal)."""
    from minitchess_alphazero_amd.environment import pos_to_fen
    from oracle.mcts import SyntheticEvaluator
    ev = SyntheticEvaluator(salt=0)
    for case in load_golden('quirk'):
        f = case['fen']
        eng = _engine(1, 64)          # sqrt(N.sum()) table sized for 64 sims x 30 moves
        eng.set_games([f])
        eng.clear_trees()
        rng = np.random.RandomState(0)
        qs = []
        for _ in range(len(case['Q_after_each_sim'])):
            k, new = eng.move_begin()
            eng.set_noise([rng.dirichlet([0.6] * int(k[0]))[None, :] if not new[0] else None])
            eng.sim_select(0)
            lpos, _g, lk, lcodes = eng.leaves()
            P, v = [], []
            for i in range(len(lk)):
                p, val = ev.evaluate(pos_to_fen(lpos[i]), [int(c) for c in lcodes[i][:lk[i]]])
                P.append(np.asarray(p, np.float32))
                v.append(val)
            eng.set_leaves(P, v)
            eng.sim_backup()
            t = eng.tree(0)
            qs.append([float(x) for x in t['Q'][f]] if f in t['Q'] else None)
        assert qs == case['Q_after_each_sim'], f
        t = eng.tree(0)
        assert [float(x) for x in t['N'][f]] == case['N_final']
        assert t['legal_moves'][f] == case['legal']
        assert {k: float(v) for k, v in t['terminal'].items()} == case['terminal']
        # the quirk itself: some edge's Q sequence contains +1 then 0 then -1/3
        seqs = np.array([q for q in qs if q is not None])
        assert any(1.0 in list(seqs[:, a]) and -1.0 / 3.0 in list(seqs[:, a]) for a in range(seqs.shape[1]))


# ---- decisive games ---------------------------------------------------------------------------

def test_decisive_games_synthetic_vs_reference():
    from oracle.mcts import SyntheticEvaluator
    games = [g for g in load_golden('trees_r2')['decisive'] if g['evaluator'].startswith('synthetic')]
    assert len(games) >= 3 and all(g['moves'][-1]['reward'] == 1.0 for g in games)
    ev = SyntheticEvaluator(salt=0)
    eng = _engine(len(games), games[0]['sims'])
    recs, _ = drive_engine(eng, len(games), games[0]['sims'], [g['seed'] for g in games], evaluator=ev,
                           start_fen=[g['start'] for g in games])
    for got, gm in zip(recs, games):
        assert compare_records(got, gm['moves'])[2] is None, gm['start']
        assert [x['reward'] for x in got] == [x['reward'] for x in gm['moves']]


def test_decisive_games_seed0_net_host_and_gpu():
    """The seed-0 net from endgame starts: host torch leaves (L1, bit-exact) and the GPU network
    through the C++ driver (mtaz_play from the set roots, records and reward back-fill)."""
    from oracle.mcts import TorchNetEvaluator
    from oracle.net import seed0_network
    games = [g for g in load_golden('trees_r2')['decisive'] if g['evaluator'] == 'net_seed0']
    assert any(g['moves'][-1]['reward'] != 0.0 for g in games)
    sims = games[0]['sims']
    eng = _engine(len(games), sims)
    recs, _ = drive_engine(eng, len(games), sims, [g['seed'] for g in games],
                           evaluator=TorchNetEvaluator(seed0_network()), start_fen=[g['start'] for g in games])
    for got, gm in zip(recs, games):
        assert compare_records(got, gm['moves'])[2] is None, gm['start']
        assert [x['reward'] for x in got] == [x['reward'] for x in gm['moves']]
    # GPU network, C++ driver: games with consecutive seeds from their own starts
    rows = []
    for gm in games:
        e1 = _engine(1, sims, seed_base=gm['seed'])
        e1.set_weights(_seed0_network())
        e1.set_games([gm['start']])
        e1.clear_trees()
        e1.play(from_current=True)
        got = e1.episodes()[0]
        same, total, first = compare_records(got, gm['moves'])
        rows.append({'start': gm['start'], 'identical_plies': same, 'plies': total, 'first_divergence': first})
        assert first is None, rows[-1]
        assert [x['reward'] for x in got] == [x['reward'] for x in gm['moves']]
    _write_result('decisive_seed0_32/f16f8/mtaz_play', rows)


# ---- BASELINE config 3 ------------------------------------------------------------------------

def test_c3_checkpoint_pinned():
    c3_network()          # loads and checks the sha256 of make_golden_r2.py's recipe output


def test_c3_host_leaves_256_sims_equal_reference():
    """L1 at config 3's search depth: the reference's 256-sim game with the C3 checkpoint, leaves
    evaluated batch-1 by torch on the host exactly as exp/agent.py:66-69; every pi and action."""
    from oracle.mcts import TorchNetEvaluator
    gm = load_golden('c3')['c3_256'][0]
    eng = _engine(1, gm['sims'])
    recs, _ = drive_engine(eng, 1, gm['sims'], [gm['seed']], evaluator=TorchNetEvaluator(c3_network()))
    assert compare_records(recs[0], gm['moves'])[2] is None
    assert [x['reward'] for x in recs[0]] == [x['reward'] for x in gm['moves']]


@pytest.mark.parametrize('precision', PRECISIONS)
def test_c3_gpu_net_256_sims_vs_reference(precision):
    """L3 at config 3: the GPU network end to end on the C3 checkpoint vs the reference game."""
    _l3('c3_256', precision, c3_network(), c3_network(), load_golden('c3')['c3_256'])


def test_c3_play_4096_games_256_sims():
    """Config 3 at full size through mtaz_play: every game finishes, no device error flag
    (capacity, depth, hash, range), and the trees stay inside their preallocated capacity."""
    eng = _engine(4096, 256)
    eng.set_weights(c3_network())
    st = eng.play()
    assert st['games'] == 4096 and st['plies'] > 4096
    assert st['sims'] == st['plies'] * 256
    nc, ec = st['node_cap'], st['edge_cap']
    assert 0 < st['max_nodes'] <= nc and 0 < st['max_edges'] <= ec
    print({k: st[k] for k in ('plies', 'nn_evals', 'terminal_sims', 'decisive', 'max_nodes', 'max_edges', 'wall_ms')},
          'capacity', nc, ec)
