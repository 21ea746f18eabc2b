"""One rank of the C5 loop test (tests/test_gpu_loop_multirank.py), started by
minitchess_alphazero_amd.launch.spawn_ranks with RANK / WORLD_SIZE / MASTER_* set.

Runs minitchess_alphazero_amd.loop.run_loop over gloo (both ranks on cuda:0 of the one-GPU box) with
deterministic algorithms, so that the learner's update is bitwise reproducible; rank 0 writes the
per-iteration history and the final weights' float64 checksum and first values to argv[1]."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    out, games, sims, iters = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    # optional: arena games per side per rank and the gate threshold (C5 gating at world > 1)
    arena_games = int(sys.argv[5]) if len(sys.argv) > 5 else 0
    gate = float(sys.argv[6]) if len(sys.argv) > 6 else 0.55
    import torch
    import torch.distributed as dist
    from minitchess_alphazero_amd.loop import flat_weights, run_loop
    torch.use_deterministic_algorithms(True)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    dist.init_process_group('gloo')
    hist, net = run_loop(iters, games, sims, batch_size=16, dist=dist, device=0, seed=0, log=lambda s: None,
                         arena_games=arena_games, gate_threshold=gate)
    flat, _ = flat_weights(net, 'cpu')
    if arena_games:   # every rank: its own final weights (all must keep or revert alike)
        with open(f'{out}.rank{dist.get_rank()}', 'w') as fh:
            json.dump({'sum': flat.double().sum().item(), 'head': flat[:2000].tolist(),
                       'tail': flat[-2000:].tolist()}, fh)
    if dist.get_rank() == 0:
        with open(out, 'w') as fh:
            json.dump({'history': hist, 'sum': flat.double().sum().item(), 'head': flat[:2000].tolist(),
                       'tail': flat[-2000:].tolist()}, fh)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
