#!/usr/bin/env python3
"""Train the BASELINE config-3 checkpoint with the full loop (minitchess_alphazero_amd.loop:
self-play -> learner -> weights; reference learner settings: batch 32, AdamW lr 0.2, 1 epoch)
and write it with its sha256.  GPU training is not bitwise deterministic, so the hash belongs to
this file, not to the recipe.
Usage: python tools/make_c3_checkpoint.py --out gpurun_out/c3.pt [--iterations 3 --games 1024 --sims 64]
"""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--iterations', type=int, default=3)
    ap.add_argument('--games', type=int, default=1024)
    ap.add_argument('--sims', type=int, default=64)
    ap.add_argument('--lr', type=float, default=0.2)
    args = ap.parse_args()
    import torch
    from minitchess_alphazero_amd.loop import run_loop
    hist, net = run_loop(args.iterations, args.games, args.sims, lr=args.lr)
    sd = net.state_dict()
    torch.save(sd, args.out)
    h = hashlib.sha256()
    for k, v in sd.items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    meta = {'checkpoint': args.out, 'sha256': h.hexdigest(), 'iterations': args.iterations, 'games': args.games,
            'sims': args.sims, 'lr': args.lr, 'history': hist}
    with open(args.out + '.json', 'w') as f:
        json.dump(meta, f, indent=1)
    print(json.dumps({k: meta[k] for k in ('checkpoint', 'sha256', 'iterations', 'games', 'sims')}))


if __name__ == '__main__':
    main()
