"""World-size-2 gloo test of the sharding contract, CPU only.

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


def test_two_rank_sharding_matches_single_process():
    from oracle import selfplay
    from oracle.mcts import SyntheticEvaluator
    world, gpr, sims = 2, 2, 4
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
    assert secs == 2.0
    assert tot['games'] == world * gpr and tot['plies'] == sum(len(r) for r in single)


def test_shard_bounds():
    from minitchess_alphazero_amd.sharding import shard
    assert shard(3, 8, 4096) == (3 * 4096, 4096)
    with pytest.raises(ValueError):
        shard(8, 8, 4096)
