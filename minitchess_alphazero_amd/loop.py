"""Self-play -> learner -> weights loop: BASELINE config 5 on one node.

The reference runs this as a distributed system: puppets play (app/puppet.py) and publish
each episode over MQTT (app/base.py:52-70), the learner collects them and trains every
`episode_frequency` episodes (app/learner.py:71-98), and rlweb serves the new weights the
puppets download (app/base.py:29-39).  Here one process per GPU does the same exchange over
torch.distributed, with no transport layer between the steps:

  1. every rank plays its G games on its own engine (games sharded by global id; the seeds
     of iteration i, rank r are (i * world + r) * G + g);
  2. the ranks' packed episode records (EpisodeRecords) are gathered to rank 0, the host
     queue of SURVEY 8e;
  3. rank 0's LearnPuppet runs one update (the reference's learner step, app/base.py:188-195,
     on PyTorch-ROCm);
  4. the new weights (the 133 float tensors the engine consumes, 42.8 MB) are broadcast from
     rank 0 as ONE flat float32 buffer (RCCL over xGMI with the nccl backend) and
     every rank uploads them into its engine;
  5. optional gating (--arena-games > 0; the reference's arena and 0.55 gate are commented
     out, exp/learner.py:97-145, app/base.py:194-196, so the default keeps every update):
     every rank plays its shard of arena games new-vs-previous (minitchess_alphazero_amd.arena),
     the win counts are all-reduced, and all ranks keep or revert the weights alike.
Run: python -m minitchess_alphazero_amd.loop [--iterations I --games G --sims S]
     N GPUs: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 -m ...
"""
import argparse
import json
import os
import time

import numpy as np
import torch

from .learner import EpisodeRecords, LearnPuppet
from .network import Network, weight_tensors


def flat_weights(net_or_sd, device):
    """The engine's 133 weight tensors as one flat float32 buffer on `device` (+ their shapes)."""
    ts = [t.detach().to(device, torch.float32).reshape(-1) for t in weight_tensors(net_or_sd)]
    return torch.cat(ts), [t.numel() for t in ts]


def unflat_into(flat, net):
    """Copy a flat buffer (weight_tensors order) into `net`'s parameters and BN buffers."""
    with torch.no_grad():
        o = 0
        for t in weight_tensors(net):
            n = t.numel()
            t.copy_(flat[o:o + n].reshape(t.shape).to(t.device, t.dtype))
            o += n
    return net


def broadcast_weights(net, dist, device, src=0):
    """Rank `src`'s weights into `net` on every rank: one broadcast of the flat buffer."""
    flat, _ = flat_weights(net, device)
    if dist is not None:
        dist.broadcast(flat, src=src)
    unflat_into(flat, net)
    return flat


def gather_records(rec, dist, dst=0):
    """Every rank's EpisodeRecords to rank `dst` (rank order); None on other ranks."""
    if dist is None:
        return [rec]
    world = dist.get_world_size()
    obj = {'pos': rec.pos, 'k': rec.k, 'codes': rec.codes, 'visits': rec.visits, 'reward': rec.reward}
    out = [None] * world if dist.get_rank() == dst else None
    dist.gather_object(obj, out, dst=dst)
    if out is None:
        return None
    return [EpisodeRecords(o['pos'], o['k'], o['codes'], o['visits'], o['reward']) for o in out]


def arena_verdict(res, dist, device, gate_threshold):
    """This rank's arena counts summed over every rank (one all_reduce), the score of
    exp/learner.py:97-145 (new wins / decisive games) and the 0.55 gate of app/base.py:194-196:
    every rank reaches the same verdict from the same sums, so all keep or all revert."""
    cnt = torch.tensor([res['new_wins'], res['old_wins'], res['draws'], res['games']], dtype=torch.float64,
                       device=device)
    if dist is not None:
        dist.all_reduce(cnt)
    nw, ow, dr, ng = cnt.tolist()
    score = nw / (nw + ow + 1e-8)
    return {'new_wins': int(nw), 'old_wins': int(ow), 'draws': int(dr), 'games': int(ng), 'score': score,
            'accepted': score > gate_threshold}


def arena_round(new_net, old_net, games, sims, dist, device, seed_base, gate_threshold=0.55):
    """Sharded arena: each rank plays `games` games per side; counts summed over ranks."""
    from .arena import arena
    from .engine import Engine
    eng = Engine(n_games=games, sims=sims, device=device)
    res = arena(eng, new_net, old_net, seed_base=seed_base)
    eng.close()
    dev = torch.device('cuda', device) if dist is None or dist.get_backend() != 'gloo' else torch.device('cpu')
    return arena_verdict(res, dist, dev, gate_threshold)


def run_loop(iterations, games, sims, batch_size=32, epochs=1, lr=0.2, dist=None, device=0, seed=0,
             log=print, arena_games=0, gate_threshold=0.55, on_iteration=None, starts=None):
    """C5 on this node.  Returns rank 0's per-iteration history (other ranks: []).
    on_iteration(it, net, records, history_entry), rank 0 only, after the weights of
    iteration `it` are in place (tools/train_stress.py measures the network there).
    starts(it, rank, games) -> None (every game from STARTING_FEN, the reference's puppet) or a list
    of `games` FENs to start this iteration's games from (tools/train_stress.py mixes endgame
    starts in, so that the value targets are not all draws)."""
    from .engine import Engine
    rank = dist.get_rank() if dist is not None else 0
    world = dist.get_world_size() if dist is not None else 1
    dev = torch.device('cuda', device)
    torch.manual_seed(seed)
    net = Network()                                   # identical random init on every rank
    learner = LearnPuppet('learner', batch_size, epochs, {'lr': lr}, device=dev) if rank == 0 else None
    if learner is not None:
        learner.weights = net.state_dict()
    broadcast_weights(net, dist, dev)
    eng = Engine(n_games=games, sims=sims, device=device)
    eng.set_weights(net)
    history = []
    for it in range(iterations):
        t0 = time.perf_counter()
        eng.set_seed_base((it * world + rank) * games)
        fens = starts(it, rank, games) if starts is not None else None
        if fens is None:
            st = eng.play()
        else:
            eng.set_games(fens)
            st = eng.play(from_current=True)
        rec = EpisodeRecords.from_engine(eng.records())
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        parts = gather_records(rec, dist)
        t2 = time.perf_counter()
        out = None
        old_sd = {k: v.detach().clone() for k, v in net.state_dict().items()}
        if rank == 0:
            old_version = learner.weights_version
            learner.push_records(EpisodeRecords.concat(parts), games * world)
            learner.train()
            out = learner.update(encode=False)
            learner.simulate()
            net.load_state_dict(out['weights'])
        torch.cuda.synchronize(dev)
        t3 = time.perf_counter()
        broadcast_weights(net, dist, dev)
        verdict = None
        if arena_games > 0:
            prev = Network()
            prev.load_state_dict(old_sd)
            verdict = arena_round(net, prev, arena_games, sims, dist, device,
                                  seed_base=10 ** 9 + (it * world + rank) * 2 * arena_games,
                                  gate_threshold=gate_threshold)
            if not verdict['accepted']:
                net.load_state_dict(old_sd)
                if rank == 0:
                    learner._weights = {k: v.detach().cpu().clone() for k, v in old_sd.items()}
                    learner._weights_version = old_version
        eng.set_weights(net)
        torch.cuda.synchronize(dev)
        t4 = time.perf_counter()
        if rank == 0:
            rows = sum(len(p) for p in parts)
            h = {'iteration': it, 'games': games * world, 'rows': rows, 'loss': out['loss'],
                 'weights_version': out['version'], 'selfplay_s': t1 - t0, 'gather_s': t2 - t1,
                 'train_s': t3 - t2, 'broadcast_s': t4 - t3, 'iteration_s': t4 - t0,
                 'games_per_s': games * world / (t4 - t0), 'samples_per_s_train': rows / (t3 - t2),
                 'plies_per_game': st['plies'] / games, 'decisive_frac': st['decisive'] / games}
            if verdict is not None:
                h['arena'] = verdict
            if on_iteration is not None:
                on_iteration(it, net, EpisodeRecords.concat(parts), h)
            history.append(h)
            log(json.dumps(h))
    return history, net


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--iterations', type=int, default=2)
    ap.add_argument('--games', type=int, default=256, help='games per GPU per iteration')
    ap.add_argument('--sims', type=int, default=64)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--epochs', type=int, default=1)
    ap.add_argument('--lr', type=float, default=0.2)
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--arena-games', type=int, default=0, help='arena games per side per GPU (0: no gating)')
    ap.add_argument('--gate', type=float, default=0.55)
    ap.add_argument('--save', default='', help='write the final state_dict here (torch.save)')
    args = ap.parse_args(argv)
    world = int(os.environ.get('WORLD_SIZE', 1))
    local = int(os.environ.get('LOCAL_RANK', 0))
    from .launch import pin_rank
    torch.set_num_threads(pin_rank(local, int(os.environ.get('LOCAL_WORLD_SIZE', world))))
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    hist, net = run_loop(args.iterations, args.games, args.sims, args.batch, args.epochs, args.lr, dist, local,
                         args.seed, arena_games=args.arena_games, gate_threshold=args.gate)
    if (dist is None or dist.get_rank() == 0) and args.save:
        torch.save(net.state_dict(), args.save)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
