"""World-size-2 and -8 gloo tests of the sharding contract, CPU only.

Each rank plays its shard of seeded games (oracle, synthetic evaluator) and the
gathered records must equal a single-process run of the same global game ids; the
end-of-run reduction must give max(time) and sum(counters)."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, games_per_rank, sims, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from minitchess_alphazero_amd.sharding import reduce_run, shard
    from oracle import selfplay
    from oracle.mcts import SyntheticEvaluator
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    seed_base, n = shard(rank, world, games_per_rank)
    ev = SyntheticEvaluator(salt=1)
    recs = [selfplay.play_games(ev, 1, sims, seed_base=seed_base + g)[0] for g in range(n)]
    gathered = [None] * world
    dist.all_gather_object(gathered, recs)
    secs, tot = reduce_run(float(rank + 1), {'games': n, 'plies': sum(len(r) for r in recs)}, dist)
    if rank == 0:
        q.put((gathered, secs, tot))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,gpr', [(2, 2), (8, 1)])
def test_rank_sharding_matches_single_process(world, gpr):
    """World 2, and world 8 (the node size of BASELINE configs 4 and 5, one game per rank)."""
    from oracle import selfplay
    from oracle.mcts import SyntheticEvaluator
    sims = 4
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, gpr, sims, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, secs, tot = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    flat = [g for rank_recs in gathered for g in rank_recs]
    ev = SyntheticEvaluator(salt=1)
    single = [selfplay.play_games(ev, 1, sims, seed_base=g)[0] for g in range(world * gpr)]
    assert flat == single
    assert secs == float(world)
    assert tot['games'] == world * gpr and tot['plies'] == sum(len(r) for r in single)


def test_shard_bounds():
    from minitchess_alphazero_amd.sharding import shard
    assert shard(3, 8, 4096) == (3 * 4096, 4096)
    with pytest.raises(ValueError):
        shard(8, 8, 4096)


def _loop_worker(rank, world, port, q):
    """The C5 exchange of minitchess_alphazero_amd.loop over gloo: each rank's records reach
    rank 0 in rank order; rank 0 trains (CPU learner) and its new weights reach every rank."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import numpy as np
    import torch
    import torch.distributed as dist
    from minitchess_alphazero_amd.learner import EpisodeRecords, SimpleAlphaZeroLearner
    from minitchess_alphazero_amd.loop import broadcast_weights, flat_weights, gather_records
    from minitchess_alphazero_amd.network import Network
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    rng = np.random.RandomState(rank)
    n = 3 + rank
    k = rng.randint(1, 6, size=n)
    rec = EpisodeRecords(np.tile(np.array([[0x00000000, 0, 0, 0, 1 | (1 << 16)]], np.uint32), (n, 1)), k,
                         rng.randint(0, 554, size=k.sum()), rng.randint(1, 9, size=k.sum()), rng.choice([-1., 0., 1.], n))
    parts = gather_records(rec, dist)
    torch.manual_seed(100 + rank)                  # ranks start from different weights
    net = Network()
    if rank == 0:
        from minitchess_alphazero_amd.environment import STARTING_FEN, pos_from_fen
        allrec = EpisodeRecords.concat(parts)
        allrec.pos[:] = pos_from_fen(STARTING_FEN)
        SimpleAlphaZeroLearner(None, 36, net, 4, 1, {'lr': 0.01}, device='cpu').update(allrec)
    broadcast_weights(net, dist, 'cpu')
    flat, _ = flat_weights(net, 'cpu')
    q.put((rank, parts and [(p.k.tolist(), p.codes.tolist(), p.visits.tolist(), p.reward.tolist()) for p in parts],
           rec.k.tolist(), rec.codes.tolist(), flat.double().sum().item(), flat[:1000].tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 8])
def test_loop_exchange_ranks(world):
    """The C5 exchange at world 2 and 8 (config 5's rank count): records gathered to rank 0 in rank
    order, rank 0's update broadcast to every rank."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_loop_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=300)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    parts = res[0][1]
    assert [p[0] for p in parts] == [res[r][2] for r in range(world)]     # rank order, intact
    assert [p[1] for p in parts] == [res[r][3] for r in range(world)]
    assert all(res[r][1] is None for r in range(1, world))
    assert all(res[0][4] == res[r][4] and res[0][5] == res[r][5] for r in range(world))   # identical weights


def _arena_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from minitchess_alphazero_amd.loop import arena_verdict
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=rank, world_size=world)
    # rank-local arena counts whose LOCAL verdicts disagree: rank 0 alone would keep the new net
    # (3 of 3 decisive games), every other rank alone would revert (0 of 2)
    local = ({'new_wins': 3, 'old_wins': 0, 'draws': 1, 'games': 4} if rank == 0 else
             {'new_wins': 0, 'old_wins': 2, 'draws': 2, 'games': 4})
    out = {th: arena_verdict(local, dist, torch.device('cpu'), th) for th in (0.55, 0.5, 0.3)}
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 8])
def test_arena_gate_same_verdict_on_every_rank(world):
    """C5 gating at world > 1 (loop.run_loop with arena_games > 0): the ranks' arena
    counts are all-reduced and every rank applies the 0.55 gate (app/base.py:194-196) to the same
    sums, so all keep or all revert even when a rank's own games point the other way."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_arena_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nw, ow = 3, 2 * (world - 1)
    for th in (0.55, 0.5, 0.3):
        verdicts = [g[th] for g in gathered]
        assert all(v == verdicts[0] for v in verdicts), th
        v = verdicts[0]
        assert (v['new_wins'], v['old_wins'], v['games']) == (nw, ow, 4 * world)
        assert v['accepted'] == (nw / (nw + ow + 1e-8) > th)
    # the thresholds split the outcomes: at world 2 (score 0.6) 0.55 keeps, at world 8 (score 0.18) it reverts
    assert gathered[0][0.55]['accepted'] == (world == 2)
    assert gathered[0][0.3]['accepted'] == (world == 2)
