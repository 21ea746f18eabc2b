"""One rank of the engine-level sharding test (tests/test_gpu_multirank.py), started by
minitchess_alphazero_amd.launch.spawn_ranks with RANK / WORLD_SIZE / MASTER_* set.

Every rank plays its shard of global game ids on the engine (seed_base = shard(rank, world, G)),
the episodes are gathered to rank 0 over gloo, and the engine's counters go through reduce_run;
rank 0 writes both to argv[1] (JSON).  All ranks share cuda:0 (one GPU on the test box)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    out, G, sims = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    import torch
    import torch.distributed as dist
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    from minitchess_alphazero_amd.sharding import reduce_run, shard
    dist.init_process_group('gloo')
    rank, world = dist.get_rank(), dist.get_world_size()
    seed_base, n = shard(rank, world, G)
    eng = Engine(n_games=n, sims=sims, device=0, seed_base=seed_base)
    torch.manual_seed(0)
    eng.set_weights(Network())
    st = eng.play()
    eps = eng.episodes()
    gathered = [None] * world
    dist.all_gather_object(gathered, eps)
    keys = ['games', 'plies', 'sims', 'nn_evals', 'terminal_sims', 'decisive']
    secs, tot = reduce_run(float(rank + 1), {k: st[k] for k in keys}, dist)
    if rank == 0:
        with open(out, 'w') as fh:
            json.dump({'episodes': [e for r in gathered for e in r], 'seconds': secs, 'totals': tot,
                       'per_rank_games': n}, fh)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
