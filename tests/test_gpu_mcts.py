"""GPU: MCTS kernels vs the CPU oracle / the reference's own traces, bit-exact.

Parity tiers:
  L1  tree + moves bit-exact with a host evaluator (the oracle's SyntheticEvaluator,
      or the batch-1 torch-CPU seed-0 net exactly as the reference evaluates leaves)
  L3  GPU network end to end: move identity rate vs the reference trace, reported
"""
import numpy as np
import pytest

from conftest import load_golden
from helpers import compare_records, drive_engine

pytestmark = pytest.mark.gpu


def _engine(n_games, sims, **kw):
    from minitchess_alphazero_amd.engine import Engine
    return Engine(n_games=n_games, sims=sims, **kw)


def test_select_expand_backup_synthetic_vs_reference_traces():
    """Host evaluator = SyntheticEvaluator: every game of the reference trace fixture."""
    from oracle.mcts import SyntheticEvaluator
    t = load_golden('trees')
    ev = SyntheticEvaluator(salt=t['synthetic_salt'])
    by_sims = {}
    for gm in t['synthetic']:
        by_sims.setdefault(gm['sims'], []).append(gm)
    for sims, games in by_sims.items():
        eng = _engine(len(games), sims)
        recs, _ = drive_engine(eng, len(games), sims, [g['seed'] for g in games], evaluator=ev)
        for got, gm in zip(recs, games):
            same, total, first = compare_records(got, gm['moves'])
            assert first is None, f'seed {gm["seed"]} sims {sims}: first mismatch at ply {first}'
            assert [r['reward'] for r in got] == [r['reward'] for r in gm['moves']]


@pytest.mark.parametrize('memo,spill', [(1, False), (0, False), (1, True), (2, False)],
                         ids=['memo', 'no-memo', 'memo-pool-spill', 'batch-memo'])
def test_trees_bit_exact_vs_oracle(memo, spill):
    """Final transposition tables (Q, N, P, legal_moves, terminal, visited) equal the oracle's,
    with the per-game leaf memo (the default), the per-game + batch memo and without a memo, and
    with table regions of 40 edges so that most nodes take their children from the shared edge
    pool.  The host evaluator sees every leaf the engine asks for: all of the oracle's expansions
    without the memo, fewer with it."""
    from oracle.mcts import SyntheticEvaluator
    from oracle import selfplay
    ev = SyntheticEvaluator(salt=3)
    seeds = [101, 102, 103]
    eng = _engine(len(seeds), 24)
    eng.set_memo(memo)
    if spill:
        eng.set_edge_capacity(40, 1 << 20)
    trees = []
    recs, dst = drive_engine(eng, len(seeds), 24, seeds, evaluator=ev, trees_out=trees)
    ref_evals = 0
    for g, s in enumerate(seeds):
        st = {}
        ref = selfplay.play_games(ev, 1, 24, seed_base=s, stats=st)[0]
        ref_evals += st['nn_evals']
        assert compare_records(recs[g], ref)[2] is None
        for agent in (0, 1):
            mine, theirs = trees[g][agent], st['trees'][0][agent]
            assert mine['visited'] == theirs['visited']
            assert mine['terminal'] == theirs['terminal']
            assert set(mine['Q']) == set(theirs['Q'])
            for fen in theirs['Q']:
                assert mine['legal_moves'][fen] == list(theirs['legal_moves'][fen])
                assert np.array_equal(mine['Q'][fen], theirs['Q'][fen]), fen
                assert np.array_equal(mine['N'][fen], theirs['N'][fen]), fen
                assert np.array_equal(mine['P'][fen], np.asarray(theirs['P'][fen], np.float32)), fen
    if memo:
        assert dst['nn_evals'] < ref_evals
    else:
        assert dst['nn_evals'] == ref_evals


def test_long_legal_lists_trees_bit_exact():
    """Roots with 70-73 legal moves (conftest.LONG_LIST_FENS): move generation ranks more codes
    than a wave has lanes (wave_legal's LDS fallback) and the PUCT argmax holds two children per
    lane; moves, rewards and both final tables equal the oracle's (SyntheticEvaluator, 24 sims)."""
    from conftest import LONG_LIST_FENS
    from oracle.mcts import SyntheticEvaluator
    from oracle import selfplay
    ev = SyntheticEvaluator(salt=5)
    seeds = [201 + i for i in range(len(LONG_LIST_FENS))]
    eng = _engine(len(seeds), 24)
    trees = []
    recs, _ = drive_engine(eng, len(seeds), 24, seeds, evaluator=ev, start_fen=LONG_LIST_FENS, trees_out=trees)
    for g, (s, fen) in enumerate(zip(seeds, LONG_LIST_FENS)):
        st = {}
        ref = selfplay.play_games(ev, 1, 24, seed_base=s, stats=st, start_fen=fen)[0]
        assert len(recs[g][0]['legal_moves']) > 64, fen
        assert compare_records(recs[g], ref)[2] is None, fen
        assert [r['reward'] for r in recs[g]] == [r['reward'] for r in ref], fen
        for agent in (0, 1):
            mine, theirs = trees[g][agent], st['trees'][0][agent]
            assert mine['visited'] == theirs['visited'], fen
            assert set(mine['Q']) == set(theirs['Q']), fen
            for f in theirs['Q']:
                assert mine['legal_moves'][f] == list(theirs['legal_moves'][f]), f
                assert np.array_equal(mine['Q'][f], theirs['Q'][f]), f
                assert np.array_equal(mine['N'][f], theirs['N'][f]), f


def _net(kind):
    """seed0: torch.manual_seed(0); Network().  stress: the round-3 stress checkpoint (trunk
    activations in the thousands; its k_net_y stored-units exponents leave 0 on a few positions).
    stress5: stress4 with its trunk in 2^7 larger units (exponents 1-4 on every position and 18 of
    the 19 trunk layers, a value head whose outputs vary; tests/golden/make_golden_r5.py).  stress6:
    the same with a gain of 181 (new significands, exponents 2-5; tests/golden/make_golden_r6.py)."""
    import torch
    from minitchess_alphazero_amd.network import Network
    from helpers import stress_network
    if kind == 'seed0':
        torch.manual_seed(0)
        return Network()
    return stress_network(kind)


@pytest.mark.parametrize('kind', ['seed0', 'stress', 'stress5', 'stress6'])
def test_leaf_memo_leaves_games_unchanged(kind):
    """The leaf memo changes which leaves the network evaluates, not the games: with the GPU network,
    the per-game memo, the per-game + batch memo and no memo give identical records, and computed +
    memo-supplied evaluations equal the evaluations without the memo (the reference's count: one
    per non-terminal expansion).  The engine is played twice per mode: the batch memo starts empty
    in every play.  On the stress net too (VERDICT r3 #2 / ADVICE r3: a memo hit supplies a result
    computed in another batch, which is exact only because k_net_y's results are per-board)."""
    net = _net(kind)
    out = {}
    for memo in (1, 2, 0):
        eng = _engine(32, 16, seed_base=11)
        eng.set_weights(net)
        eng.set_memo(memo)
        first = eng.play()
        out[memo] = (eng.play(), eng.records())
        assert first['nn_evals'] == out[memo][0]['nn_evals']
    st_off, r_off = out[0]
    assert st_off['memo_hits'] == 0
    for memo in (1, 2):
        st, r = out[memo]
        for key in ('plies', 'pos', 'action', 'k', 'codes', 'visits', 'reward', 'outcome'):
            assert np.array_equal(r[key], r_off[key]), (memo, key)
        assert st['memo_hits'] > 0
        assert st['nn_evals'] + st['memo_hits'] == st_off['nn_evals']
        assert st['terminal_sims'] == st_off['terminal_sims']
        print(f"memo {memo}: {st['memo_hits']:.0f} of {st_off['nn_evals']:.0f} evaluations supplied "
              f"({st['memo_hits'] / st_off['nn_evals']:.1%}; batch memo {st['memo_batch_hits']:.0f})")
    assert out[1][0]['memo_batch_hits'] == 0 and out[2][0]['memo_batch_hits'] > 0


def test_edge_pool_spill_and_exhaustion():
    """Tables that outgrow their edge region continue in the shared pool with unchanged games; an
    exhausted pool fails the call with the edge-capacity flag (exp/agent.py:64-66 never fails, so
    the pool is sized from memory, 8 edges per node per table by default)."""
    import torch
    from minitchess_alphazero_amd import _lib
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    ref = _engine(16, 16, seed_base=3)
    ref.set_weights(net)
    st_ref = ref.play()
    r_ref = ref.records()
    assert st_ref['pool_edges'] == 0
    small = _engine(16, 16, seed_base=3)
    small.set_weights(net)
    small.set_edge_capacity(64, 1 << 21)
    st = small.play()
    r = small.records()
    for key in ('plies', 'pos', 'action', 'k', 'codes', 'visits', 'reward', 'outcome'):
        assert np.array_equal(r[key], r_ref[key]), key
    assert st['pool_edges'] > 0 and st['max_edges'] <= 64
    small.set_edge_capacity(64, 256)
    with pytest.raises(_lib.MtazError, match='edge-capacity'):
        small.play()
    # the state the round-4 fault (r04s) left behind.  After the capacity
    # error the same engine, given its pool back, plays the same games bit-exactly, and a new
    # engine on the same device works: the error is reported and cleared, the context is sound.
    small.set_edge_capacity(64, 1 << 21)
    st2 = small.play()
    r2 = small.records()
    for key in ('plies', 'pos', 'action', 'k', 'codes', 'visits', 'reward', 'outcome'):
        assert np.array_equal(r2[key], r_ref[key]), key
    assert st2['games'] == st_ref['games'] and st2['plies'] == st_ref['plies']
    fresh = _engine(16, 16, seed_base=3)
    fresh.set_weights(net)
    fresh.play()
    r3 = fresh.records()
    for key in ('plies', 'pos', 'action', 'visits', 'reward'):
        assert np.array_equal(r3[key], r_ref[key]), key


def test_numpy1_cast_mode_vs_oracle():
    from oracle.mcts import SyntheticEvaluator
    from oracle import selfplay
    ev = SyntheticEvaluator(salt=5)
    eng = _engine(2, 16, cast_mode=1)
    recs, _ = drive_engine(eng, 2, 16, [7, 8], evaluator=ev)
    for g, s in enumerate([7, 8]):
        ref = selfplay.play_games(ev, 1, 16, seed_base=s, cast_mode=1)[0]
        assert compare_records(recs[g], ref)[2] is None


def test_host_torch_net_matches_reference_trace():
    """L1 with the real network: leaves evaluated batch-1 on the CPU exactly like the
    reference (exp/agent.py:67-69) -> the reference's own seed-0 game, bit-exact."""
    from oracle.mcts import TorchNetEvaluator
    from oracle.net import seed0_network
    gm = load_golden('trees')['net_seed0'][0]
    eng = _engine(1, gm['sims'])
    recs, _ = drive_engine(eng, 1, gm['sims'], [gm['seed']], evaluator=TorchNetEvaluator(seed0_network()))
    assert compare_records(recs[0], gm['moves'])[2] is None


def test_cpp_driver_equals_python_driver():
    """mtaz_play (C++ host RNG + action choice) == the Python/numpy driver, same GPU net."""
    import torch
    from minitchess_alphazero_amd.network import Network
    seeds = [0, 1, 2, 3]
    torch.manual_seed(0)
    net = Network()
    eng = _engine(len(seeds), 12, seed_base=0)
    eng.set_weights(net)
    eng.play()
    got = eng.episodes()
    eng2 = _engine(len(seeds), 12)
    eng2.set_weights(net)
    ref, _ = drive_engine(eng2, len(seeds), 12, seeds, evaluator=None)
    for a, b in zip(got, ref):
        assert compare_records(a, b)[2] is None
        assert [r['reward'] for r in a] == [r['reward'] for r in b]


@pytest.mark.parametrize('kind', ['seed0', 'stress', 'stress5', 'stress6'])
def test_games_independent_of_batch_composition(kind):
    """Per-game results depend only on the game's seed (the multi-GPU sharding contract), also on a
    trained net whose stored-units exponents leave 0: 40 games in one engine (up to
    40 leaves per network launch, 10 workgroups) against games played alone."""
    net = _net(kind)
    big = _engine(40, 8, seed_base=100)
    big.set_weights(net)
    big.play()
    all_eps = big.episodes()
    for g in (0, 3, 5, 22, 39):
        one = _engine(1, 8, seed_base=100 + g)
        one.set_weights(net)
        one.play()
        assert compare_records(one.episodes()[0], all_eps[g])[2] is None


def test_pipelined_groups_equal_single_stream():
    """mtaz_set_pipeline: game groups on separate HIP streams give the same episodes, in the
    same game order, as one stream (the groups are disjoint global game ranges)."""
    import torch
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    one = _engine(8, 8, seed_base=7)
    one.set_weights(net)
    one.play()
    ref = one.episodes()
    two = _engine(8, 8, seed_base=7)
    two.set_weights(net)
    for groups in (2, 4):
        two.set_pipeline(groups)
        st = two.play()
        eps = two.episodes()
        assert len(eps) == len(ref)
        for g in range(len(ref)):
            assert compare_records(eps[g], ref[g])[2] is None, (groups, g)
        assert st['games'] == 8 and st['sims'] == one.stats()['sims']


@pytest.mark.parametrize('kind,memo,mode,G', [('seed0', 2, 2, 4096), ('seed0', 0, 2, 4096), ('seed0', 2, 1, 4096),
                                              ('stress5', 2, 2, 4096), ('stress6', 2, 1, 4096),
                                              ('seed0', 2, 1, 4096 + 700), ('seed0', 0, 2, 4096 + 700)])
def test_deferred_tails_leave_games_unchanged(kind, memo, mode, G):
    """Deferred tails (mtaz_set_defer, the play() default): a wave evaluates only whole rounds of
    4 boards x CUs of its leaves and the rest wait, their games selecting again only after that
    leaf's backup; each move ends with the waves the lagging games need.  Every game still runs its
    simulations in order on the same tables, noise and network results, so the records equal the
    every-leaf-every-wave schedule's bit for bit, and every expansion is evaluated or supplied by
    the memo in both (the reference's count).  4096 games: the waves hold more than one round of
    leaves, so leaves are really deferred (extra_waves > 0).  4796 games: the leaf list
    is built in chunks of 4,096 games (k_leaf_compact's multi-chunk path with one scan per lag bucket)."""
    net = _net(kind)
    out = {}
    for defer in (0, mode):
        eng = _engine(G, 8, seed_base=900)
        eng.set_weights(net)
        eng.set_memo(memo)
        eng.set_defer(defer)
        eng.set_schedule(0)   # moves in lockstep, the default (free-running moves: the test below)
        st = eng.play()
        out[defer] = (st, eng.records())
        eng.close()
    (s0, r0), (s1, r1) = out[0], out[mode]
    for key in ('plies', 'pos', 'action', 'k', 'codes', 'visits', 'reward', 'outcome'):
        assert np.array_equal(r1[key], r0[key]), key
    assert s1['nn_evals'] + s1['memo_hits'] == s0['nn_evals'] + s0['memo_hits']
    assert s1['sims'] == s0['sims'] and s1['terminal_sims'] == s0['terminal_sims']
    assert s0['extra_waves'] == 0 and s1['extra_waves'] > 0
    print(f"{kind} memo {memo} defer {mode}: {s1['extra_waves']:.0f} extra waves over {s1['moves']:.0f} moves; "
          f"waves {s0['waves']:.0f} -> {s1['waves']:.0f}")


@pytest.mark.parametrize('kind,G,defer', [('seed0', 4096, 1), ('seed0', 4096, 0), ('seed0', 4096 + 700, 2),
                                          ('stress5', 4096, 1), ('stress6', 1024, 1)])
def test_free_running_moves_leave_games_unchanged(kind, G, defer):
    """with free-running moves (mtaz_set_schedule 1; lockstep stays the default) a game
    that completes a move records it, chooses, steps and starts its next move on the device (k_turn)
    while the others keep simulating, so games drift onto different moves within one wave.  Every
    game still runs its simulations in order on its own tables with its own RandomState draws and
    the same network results, so every record equals the lockstep schedule's bit for bit (and the
    reference's count of evaluations is unchanged)."""
    net = _net(kind)
    out = {}
    for sched in (0, 1):
        eng = _engine(G, 8, seed_base=300)
        eng.set_weights(net)
        eng.set_memo(2)
        eng.set_defer(defer)
        eng.set_schedule(sched)
        st = eng.play()
        assert st['schedule'] == sched and st['rng_device'] == 1
        out[sched] = (st, eng.records())
        eng.close()
    (s0, r0), (s1, r1) = out[0], out[1]
    for key in ('plies', 'pos', 'action', 'k', 'codes', 'visits', 'reward', 'outcome'):
        assert np.array_equal(r1[key], r0[key]), key
    assert s1['nn_evals'] + s1['memo_hits'] == s0['nn_evals'] + s0['memo_hits']
    assert s1['sims'] == s0['sims'] and s1['terminal_sims'] == s0['terminal_sims']
    assert s1['moves'] == s0['moves'] and s1['plies'] == s0['plies']
    print(f"{kind} G {G} defer {defer}: waves lockstep {s0['waves']:.0f} (extra {s0['extra_waves']:.0f}) -> "
          f"free-running {s1['waves']:.0f} (extra {s1['extra_waves']:.0f})")


@pytest.mark.parametrize('kind,G,sched', [('seed0', 4096, 0), ('seed0', 4096 + 700, 0), ('stress5', 4096, 1)])
def test_lag_order_leaves_games_unchanged(kind, G, sched):
    """Round 6: which leaves a deferred-tail wave evaluates first (mtaz_set_lag_order): the least
    advanced games first (0, the default) or round 5's lag behind the most advanced leaf (1).  Only
    the wave each simulation runs in changes, so the records are identical bit for bit, with the same
    evaluations + memo hits, under the default defer mode 2 (every remainder waits), in lockstep
    (4,096 games; 4,796: the multi-chunk leaf list) and with free-running moves (chunked noise draws)."""
    net = _net(kind)
    out = {}
    for order in (1, 0):
        eng = _engine(G, 8, seed_base=500)
        eng.set_weights(net)
        eng.set_memo(2)
        eng.set_defer(2)
        eng.set_schedule(sched)
        eng.set_lag_order(order)
        st = eng.play()
        assert st['schedule'] == sched
        out[order] = (st, eng.records())
        eng.close()
    (s1, r1), (s0, r0) = out[1], out[0]
    for key in ('plies', 'pos', 'action', 'k', 'codes', 'visits', 'reward', 'outcome'):
        assert np.array_equal(r0[key], r1[key]), key
    assert s0['nn_evals'] + s0['memo_hits'] == s1['nn_evals'] + s1['memo_hits']
    assert s0['sims'] == s1['sims'] and s0['terminal_sims'] == s1['terminal_sims']
    assert s0['extra_waves'] > 0
    print(f"{kind} G {G} schedule {sched}: waves round-5 order {s1['waves']:.0f} (extra {s1['extra_waves']:.0f}) -> "
          f"least advanced first {s0['waves']:.0f} (extra {s0['extra_waves']:.0f})")
