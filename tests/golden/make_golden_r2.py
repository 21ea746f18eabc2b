#!/usr/bin/env python3
"""Round-2 golden fixtures, made by running the REFERENCE code on the CPU (build container only).

Imports the reference's exp/environment.py, exp/policy.py, exp/agent.py, exp/callbacks.py,
exp/dataset.py and exp/learner.py with the stubs of make_golden.py (un-vendored erlyx; oracle.rules
as the `chess` module), then writes:

  c3/c3.safetensors   BASELINE config 3's "trained exp/policy checkpoint", trained by the
                      reference's own loop pieces on the CPU (deterministic in this container):
                        torch.manual_seed(0); net = exp.policy.Network()
                        repeat C3_ITERS times:
                          C3_GAMES reference self-play games (SimulatePuppet's stack, app/base.py:113-120:
                          two SimpleAlphaZeroAgents, RoundRobinReferee, InfoRecorder, MonteCarloInit) at
                          C3_SIMS sims with the current net in eval mode, np.random.seed per game;
                          SimpleAlphaZeroDataset.push(rows); torch.manual_seed(it);
                          SimpleAlphaZeroLearner(env, 36, net, 32, 1, {'lr': C3_LR}).update(dataset)
                          (app/learner.py:65-68 settings, lr see C3_LR; exp/learner.py:70-91 on the
                          CPU: its .cuda() calls are made identity for this script only)
  c3.json             sha256 of the checkpoint (oracle.net.state_dict_sha256), the recipe, the
                      per-update losses, and 'c3_256': one reference self-play game at 256 sims
                      with the checkpoint (BASELINE config 3 search depth)
  c3_net.npz          the reference Network.forward (eval mode) on the C3 checkpoint: logits,
                      values for sample positions
  trees_r2.json       reference self-play traces:
                        net_seed0_64: the seed-0 net, 64 sims, seeds 0-3 (L3 move identity)
                        decisive: games from endgame starts that end decisively (synthetic
                                  evaluator, 6 sims; and the seed-0 net, 32 sims): the reward
                                  back-fill of exp/callbacks.py:49-54 and terminal handling of
                                  exp/agent.py:57-63,75-77 on decisive results
Usage: python tests/golden/make_golden_r2.py [c3|traces]   (both by default; about 10 minutes
on 8 threads)
"""
import json
import logging
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from make_golden import import_reference, sample_positions  # noqa: E402

C3_ITERS, C3_GAMES, C3_SIMS = 3, 10, 16
# AdamW learning rate of the C3 updates.  app/learner.py:69 deploys lr 0.2; three such updates
# leave a degenerate net (policy-head ReLUs dead, value saturated at -1 for every position), whose
# outputs no longer depend on the position, so that neither the network parity nor the search is
# exercised by it.  The C3 checkpoint therefore uses the same update code with AdamW's default lr.
C3_LR = 1e-3
THREADS = 8

DECISIVE_STARTS = [
    'k4/2K2/5/5/5/1Q3 w 0 5',       # KQ v K, mate available
    '3q1/5/5/5/2k2/4K b 0 5',       # the colour-rotated twin, black to move
    '1k3/5/1K3/5/5/R4 w 0 10',      # KR v K
    '4r/5/5/3k1/5/K4 b 0 10',       # KR v K, black to move
    '2k2/Q4/2K2/5/5/5 w 0 8',
    'k4/5/1K3/5/5/3R1 w 0 3',
    '2k2/5/2K2/5/5/3Q1 w 0 15',
    '5/3k1/5/q4/5/3K1 b 0 4',
]


def endgame_starts(n, seed=5):
    """Seeded K + two heavy pieces v K positions (oracle rules: legal, not over), either side to move:
    near-random play (the synthetic evaluator) mates from these often enough."""
    from oracle import rules
    rng = np.random.RandomState(seed)
    out = []
    while len(out) < n:
        sq = rng.choice(30, 4, replace=False)
        strong_white = rng.rand() < 0.5
        board = ['.'] * 30
        board[sq[0]] = 'K' if strong_white else 'k'
        board[sq[1]] = 'k' if strong_white else 'K'
        for j in (2, 3):
            piece = 'Q' if rng.rand() < 0.5 else 'R'
            board[sq[j]] = piece if strong_white else piece.lower()
        rows = []
        for r in range(5, -1, -1):
            row, e = '', 0
            for c in range(5):
                x = board[5 * r + c]
                if x == '.':
                    e += 1
                else:
                    row += (str(e) if e else '') + x
                    e = 0
            rows.append(row + (str(e) if e else ''))
        fen = '/'.join(rows) + (' w ' if rng.rand() < 0.5 else ' b ') + f'0 {1 + rng.randint(5)}'
        try:
            b = rules.Board(fen)
        except Exception:
            continue
        k_idle = rules.king_square(b.board, not b.turn)       # the side not to move must not be in check
        if (b.fen() == fen and b.result() == '*' and b.legal_moves
                and not rules.is_attacked(b.board, k_idle, b.turn)):
            out.append(fen)
    return out


def ref_selfplay(renv, rpol, ragent, rcb, model, sims, seeds, start_fen=None):
    """The reference agent stack of app/base.py:113-120 under the run_episodes stub; one game per
    seed (np.random.seed(seed) at episode start), optionally from `start_fen`
    (MinitChessEnvironment.new_episode(fen), exp/environment.py:88-91)."""
    base_env = renv.MinitChessEnvironment()

    class Env(type(base_env)):
        def new_episode(self, fen=None):
            return super().new_episode(fen=fen or start_fen)

    env = Env() if start_fen else base_env
    policy = rpol.SimpleAlphaZeroPolicy(network=model)
    agents = [ragent.SimpleAlphaZeroAgent(environment=env, policy=policy, num_simulations=sims) for _ in range(2)]
    sink = []

    class DS:
        def push(self, data):
            sink.append(data)

    referee = ragent.RoundRobinReferee(agent_tuple=tuple(agents))
    cbs = [rcb.InfoRecorder(DS()), rcb.MonteCarloInit(agents[0]), rcb.MonteCarloInit(agents[1])]
    games = []
    for s in seeds:
        np.random.seed(s)
        referee.reset()
        sink.clear()
        sys.modules['erlyx'].run_episodes(env, referee, 1, callbacks=cbs)
        rec = sink[0]
        games.append({'seed': int(s), 'sims': sims, 'start': start_fen, 'moves': [
            {'observation': r['observation'], 'legal_moves': [int(x) for x in r['legal_moves']],
             'pi': r['pi'], 'action': r['action'], 'reward': r['reward']} for r in rec]})
    return games


def import_learner():
    logging.getLogger().addHandler(logging.NullHandler())   # exp/learner.py:3 basicConfig -> no-op
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            import exp.learner as rlearn
            import exp.dataset as rdata
        finally:
            os.chdir(cwd)
    return rlearn, rdata


def train_c3(renv, rpol, ragent, rcb, rlearn, rdata):
    # the reference learner moves model and batches to CUDA (exp/learner.py:79,86); on this CPU-only
    # container those calls are made identity so the same update runs on the CPU
    torch.nn.Module.cuda = lambda self, *a, **k: self
    torch.Tensor.cuda = lambda self, *a, **k: self
    losses = []
    orig_acc = rlearn.AvgSmoothLoss.accumulate

    def acc(self, x):
        losses[-1].append(float(x))
        return orig_acc(self, x)

    rlearn.AvgSmoothLoss.accumulate = acc
    torch.manual_seed(0)
    net = rpol.Network()
    env = renv.MinitChessEnvironment()
    learner = rlearn.SimpleAlphaZeroLearner(env, 36, net, 32, 1, {'lr': C3_LR})
    last_games = None
    for it in range(C3_ITERS):
        net.eval()
        games = ref_selfplay(renv, rpol, ragent, rcb, net, C3_SIMS, [1000 * it + g for g in range(C3_GAMES)])
        ds = rdata.SimpleAlphaZeroDataset(max_length=1_000_000)
        for g in games:
            ds.push([dict(m) for m in g['moves']])
        losses.append([])
        torch.manual_seed(it)
        learner.update(ds)
        print(f'c3 iteration {it}: {len(ds)} rows, plies/game {np.mean([len(g["moves"]) for g in games]):.1f}, '
              f'loss {np.mean(losses[-1]):.3f}', flush=True)
        last_games = games
    rlearn.AvgSmoothLoss.accumulate = orig_acc
    return net.eval(), losses, last_games


def main():
    parts = sys.argv[1:] or ['c3', 'traces']
    torch.set_num_threads(THREADS)
    renv, rpol, ragent, rcb = import_reference()
    rlearn, rdata = import_learner()
    from oracle import mcts as omcts
    from oracle.net import state_dict_sha256
    t0 = time.time()
    out = {}

    if 'c3' in parts:
        net_c3, losses, last_games = train_c3(renv, rpol, ragent, rcb, rlearn, rdata)
        from safetensors.torch import save_file
        os.makedirs(os.path.join(HERE, 'c3'), exist_ok=True)
        sd = {k: v.detach().contiguous() for k, v in net_c3.state_dict().items()}
        save_file(sd, os.path.join(HERE, 'c3', 'c3.safetensors'))
        sha = state_dict_sha256(net_c3)
        fens = sample_positions(64, seed=321)
        logits, values = [], []
        with torch.no_grad():
            for f in fens:
                p, v = net_c3(rpol.Network.process_observation(f))
                logits.append(p[0].numpy())
                values.append(float(v.item()))
        np.savez_compressed(os.path.join(HERE, 'c3_net.npz'), fens=np.array(fens),
                            logits=np.stack(logits).astype(np.float32), values=np.array(values, dtype=np.float32))
        print(f'c3 checkpoint sha256 {sha} ({time.time() - t0:.0f} s)', flush=True)
        c3_256 = ref_selfplay(renv, rpol, ragent, rcb, net_c3, 256, [0])
        print(f'c3_256: {len(c3_256[0]["moves"])} plies ({time.time() - t0:.0f} s)', flush=True)
        out['c3'] = {'state_dict_sha256': sha, 'iterations': C3_ITERS, 'games_per_iteration': C3_GAMES,
                     'selfplay_sims': C3_SIMS, 'batch_size': 32, 'epochs': 1, 'optim_params': {'lr': C3_LR},
                     'torch_threads': THREADS, 'torch': torch.__version__, 'losses': losses,
                     'last_iteration_plies': [len(g['moves']) for g in last_games], 'c3_256': c3_256}

    if 'traces' in parts:
        torch.manual_seed(0)
        net0 = rpol.Network().eval()
        trees = {'net_seed0_64': ref_selfplay(renv, rpol, ragent, rcb, net0, 64, [0, 1, 2, 3])}
        print(f'net_seed0_64 done ({time.time() - t0:.0f} s)', flush=True)
        synth = omcts.SyntheticEvaluator(salt=0)
        decisive = []
        for i, f in enumerate(DECISIVE_STARTS + endgame_starts(400)):
            # 6 sims: the sign quirk (exp/agent.py:75-77) turns a mating edge's Q to 0 and -1/3 on
            # revisits, so deeper searches seldom keep a mate; sampled moves (fullmove < 6) at 6 sims do
            g = ref_selfplay(renv, rpol, ragent, rcb, synth, 6, [50 + i], start_fen=f)[0]
            g['evaluator'] = 'synthetic:0'
            if g['moves'] and g['moves'][-1]['reward'] != 0.0:
                decisive.append(g)
                if len(decisive) == 8:
                    break
        for i, f in enumerate(DECISIVE_STARTS[:4]):
            g = ref_selfplay(renv, rpol, ragent, rcb, net0, 32, [70 + i], start_fen=f)[0]
            g['evaluator'] = 'net_seed0'
            decisive.append(g)
        trees['decisive'] = decisive
        print(f'decisive: {sum(1 for g in decisive if g["moves"][-1]["reward"] != 0)} of {len(decisive)} decisive '
              f'({time.time() - t0:.0f} s)', flush=True)
        trees['synthetic_salt'] = 0
        out['trees_r2'] = trees

    for name, obj in out.items():
        with open(os.path.join(HERE, f'{name}.json'), 'w') as fh:
            json.dump(obj, fh, separators=(',', ':'))
    print('wrote', sorted(out), f'in {time.time() - t0:.0f} s')


if __name__ == '__main__':
    main()
