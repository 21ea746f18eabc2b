#!/usr/bin/env python3
"""Learner throughput: one SimpleAlphaZeroLearner.update over self-play rows.

Rows come from the engine (random-init net, --games games at --sims sims).  Timed:
  * product: the resident-batch update (HIP batch encoder once, index-gather batches,
    train-mode forward/backward + AdamW on PyTorch-ROCm)
  * ref_path_gpu: the reference's update structure on the same GPU, a DataLoader with
    collate_fn building every batch on the host (exp/learner.py:73-83)
  * cpu_baseline: the oracle's CPU update on a bounded prefix of the rows (--cpu-rows)
Reference settings: batch 32, 1 epoch, AdamW lr 0.2 (app/learner.py:65-69).
Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--games', type=int, default=256)
    ap.add_argument('--sims', type=int, default=64)
    ap.add_argument('--batch', type=int, default=32)
    ap.add_argument('--lr', type=float, default=0.2)
    ap.add_argument('--cpu-rows', type=int, default=256)
    ap.add_argument('--cpu-threads', type=int, default=16)
    args = ap.parse_args()
    import numpy as np
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.learner import SimpleAlphaZeroLearner, collate_fn, alphazero_loss
    from minitchess_alphazero_amd.network import Network

    torch.manual_seed(0)
    net0 = Network()
    eng = Engine(n_games=args.games, sims=args.sims)
    eng.set_weights(net0)
    eng.play()
    rows = [{k: r[k] for k in ('observation', 'legal_moves', 'pi', 'reward')} for ep in eng.episodes() for r in ep]
    sd0 = {k: v.clone() for k, v in net0.state_dict().items()}

    def fresh():
        n = Network()
        n.load_state_dict(sd0)
        return n

    # warm-up (MIOpen kernel selection) on a throwaway copy
    SimpleAlphaZeroLearner(None, 36, fresh(), args.batch, 1, {'lr': args.lr}, device='cuda').update(rows[:4 * args.batch])
    torch.cuda.synchronize()

    lrn = SimpleAlphaZeroLearner(None, 36, fresh(), args.batch, 1, {'lr': args.lr}, device='cuda')
    torch.manual_seed(1)
    t0 = time.perf_counter()
    lrn.update(rows)
    torch.cuda.synchronize()
    t_prod = time.perf_counter() - t0

    # the reference's structure: host collate per batch through a DataLoader
    model = fresh().train().cuda()
    opt = torch.optim.AdamW(model.parameters(), lr=args.lr)
    torch.manual_seed(1)
    loader = torch.utils.data.DataLoader(rows, batch_size=args.batch, shuffle=True, collate_fn=collate_fn)
    t0 = time.perf_counter()
    for pib, ch, clk, rew in loader:
        loss = alphazero_loss(model, pib.cuda(), ch.cuda(), clk.cuda(), rew.cuda())
        opt.zero_grad()
        loss.backward()
        float(loss.detach().item())
        opt.step()
    torch.cuda.synchronize()
    t_ref = time.perf_counter() - t0

    import oracle.learner as ol
    from oracle.net import Network as ONet
    torch.set_num_threads(args.cpu_threads)
    onet = ONet()
    onet.load_state_dict(sd0)
    ods = ol.Dataset(10 ** 6)
    ods.push(rows[:args.cpu_rows])
    t0 = time.perf_counter()
    ol.update(onet, ods, args.batch, 1, {'lr': args.lr})
    t_cpu = time.perf_counter() - t0

    n = len(rows)
    line = {
        'metric': 'learner samples/s (SimpleAlphaZeroLearner.update, batch 32, AdamW lr 0.2, 1 epoch)',
        'value': n / t_prod, 'unit': 'samples/s', 'higher_is_better': True, 'rows': n,
        'batches': len(lrn.last_losses), 'seconds': t_prod, 'dtype': 'fp32',
        'data': f'self-play rows from {args.games} games at {args.sims} sims, random-init net',
        'ref_path_gpu': {'value': n / t_ref, 'unit': 'samples/s', 'seconds': t_ref,
                         'what': 'DataLoader + host collate_fn per batch, same GPU (the reference structure)'},
        'cpu_baseline': {'value': args.cpu_rows / t_cpu, 'unit': 'samples/s', 'cores': args.cpu_threads,
                         'kind': 'port', 'sample': f'oracle CPU update on the first {args.cpu_rows} rows',
                         'seconds': t_cpu},
        'final_smoothed_loss': float(np.mean(lrn.last_losses[-10:])) if lrn.last_losses else None,
    }
    print(json.dumps(line), flush=True)


if __name__ == '__main__':
    main()
