"""Multi-GPU sharding of self-play: games are independent units.

Rank r of a world of W processes (one per GPU) plays global games
[r*G, (r+1)*G), each seeded with its global id, so every game's result is the same
at 1, 2, 4 or 8 GPUs.  There is no collective on the data path; the only
collectives are the end-of-run reductions below (max of wall times, sum of counters).
"""


def shard(rank, world, games_per_rank):
    """-> (first global game id = seed_base, number of games) for this rank."""
    if not (0 <= rank < world):
        raise ValueError(f'rank {rank} outside world {world}')
    return rank * games_per_rank, games_per_rank


def reduce_run(seconds, counters, dist=None, device=None):
    """Max of wall seconds and sum of counters over ranks (identity without dist)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds, dict(counters)
    import torch
    keys = sorted(counters)
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    s = torch.tensor([float(counters[k]) for k in keys], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), dict(zip(keys, s.tolist()))
