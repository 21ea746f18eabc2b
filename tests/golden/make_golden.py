#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by running the REFERENCE code.

Runs only in the build container (needs /root/reference, read-only).  It imports
the reference's own exp/environment.py, exp/policy.py, exp/agent.py and
exp/callbacks.py with
  * stub `erlyx.*` modules (the un-vendored RL framework), and
  * oracle.rules injected as the `chess` module (the un-vendored python-chess
    fork; rules content is the build's RULES.md - "parity unpinned"),
then records what the reference computes.  The reference's source never
leaves this container; only these data files are committed.

Outputs:
  codec.json    sha256 of exp/moves_dict.json
  encoder.json  FEN -> (tokens, clock) from exp/policy.py:96-105
  env.json      per-position legal codes / reward / done from exp/environment.py
  rng.json      numpy legacy RandomState streams (dirichlet, choice) as used by exp/agent.py
  net.npz       seed-0 reference Network outputs (logits, values) for sample positions
  trees.json    seeded self-play games through the reference MCTS/agent/referee/
                InfoRecorder: per move root codes, N, pi, chosen action, rewards
  quirk.json    terminal-revisit sign quirk (exp/agent.py:75-77) Q sequence
Usage: python tests/golden/make_golden.py  (takes ~1-2 minutes)
"""
import hashlib
import json
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def install_stubs():
    """Stub erlyx (contract from call sites) and use oracle.rules as chess."""
    from collections import namedtuple
    import oracle.rules as rules
    mods = {}
    for name in ['erlyx', 'erlyx.agents', 'erlyx.types', 'erlyx.policies', 'erlyx.environment',
                 'erlyx.learners', 'erlyx.callbacks']:
        mods[name] = types.ModuleType(name)
        sys.modules[name] = mods[name]

    class BaseAgent:
        pass

    class PolicyAgent(BaseAgent):
        def __init__(self, policy):
            self._policy = policy

        @property
        def policy(self):
            return self._policy

    mods['erlyx.agents'].BaseAgent = BaseAgent
    mods['erlyx.agents'].PolicyAgent = PolicyAgent
    mods['erlyx.types'].ActionData = namedtuple('ActionData', ['action', 'info'])
    mods['erlyx.types'].EpisodeStatus = namedtuple('EpisodeStatus', ['observation', 'reward', 'done'])
    mods['erlyx.policies'].Policy = type('Policy', (), {})
    mods['erlyx.environment'].BaseEnvironment = type('BaseEnvironment', (), {})
    mods['erlyx.environment'].Episode = type('Episode', (), {})
    mods['erlyx.learners'].BaseLearner = type('BaseLearner', (), {})
    mods['erlyx.callbacks'].BaseCallback = type('BaseCallback', (), {
        'on_episode_begin': lambda self, o: None, 'on_step_end': lambda self, *a: None,
        'on_episode_end': lambda self: None})

    def run_episodes(env, agent, num_episodes, callbacks=(), use_tqdm=False, on_start=None):
        for ep in range(num_episodes):
            if on_start:
                on_start(ep)
            episode, obs = env.new_episode()
            for cb in callbacks:
                cb.on_episode_begin(obs)
            done = False
            while not done:
                action = agent.select_action(obs)
                obs, reward, done = episode.step(action.action)
                for cb in callbacks:
                    cb.on_step_end(action, obs, reward, done)
            for cb in callbacks:
                cb.on_episode_end()

    mods['erlyx'].run_episodes = run_episodes
    sys.modules['chess'] = rules


def import_reference():
    install_stubs()
    sys.path.insert(1, REF)
    cwd = os.getcwd()
    os.chdir(os.path.join(REF, 'exp'))       # exp/environment.py:16 opens moves_dict.json from CWD
    try:
        import exp.environment as renv
        import exp.policy as rpol
        import exp.agent as ragent
        import exp.callbacks as rcb
    finally:
        os.chdir(cwd)
    return renv, rpol, ragent, rcb


def sample_positions(n, seed=123):
    """Random-walk positions under oracle rules (both colours, promotions, mates)."""
    from oracle import rules
    rng = np.random.RandomState(seed)
    out, seen = [], set()
    fens = [rules.STARTING_FEN, '4k/5/5/5/5/K4 w 0 1', '4k/P4/5/5/4p/K4 w 3 12',
            '4k/P4/5/5/4p/K4 b 3 12', 'k4/2Q2/1K3/5/5/5 w 0 20', '1k3/P4/1K3/5/5/5 w 0 9',
            '2k2/5/2K2/5/5/3Q1 w 0 15', 'nbk2/ppp2/5/5/2PPP/2KBN b 0 1']
    for f in fens:
        if f not in seen:
            seen.add(f)
            out.append(f)
    while len(out) < n:
        b = rules.Board(rules.STARTING_FEN)
        for _ in range(rng.randint(1, 70)):
            moves = b.legal_moves
            if not moves or b.result() != '*':
                break
            b.push(moves[rng.randint(len(moves))])
            f = b.fen()
            if f not in seen and rng.rand() < 0.3:
                seen.add(f)
                out.append(f)
    return out[:n]


def main():
    renv, rpol, ragent, rcb = import_reference()
    from oracle import mcts as omcts
    golden = {}

    # ---- codec ---------------------------------------------------------------------
    raw = open(os.path.join(REF, 'exp', 'moves_dict.json'), 'rb').read()
    golden['codec'] = {'sha256': hashlib.sha256(raw).hexdigest(), 'num_actions': renv.NUM_ACTIONS}

    # ---- encoder + env -------------------------------------------------------------
    fens = sample_positions(600)
    enc = []
    envrows = []
    for f in fens:
        ch, clk = rpol.Network.process_observation(f)
        enc.append({'fen': f, 'tokens': ch.reshape(-1).tolist(), 'clock': float(clk.item())})
        ep = renv.MinitChessEpisode(f)
        envrows.append({'fen': f, 'legal': list(ep.get_legal_moves()), 'reward': ep.get_reward(),
                        'done': bool(ep.is_done()), 'turn': bool(ep.turn)})
    # step round trips: every legal code of a subset of positions -> next FEN
    steps = []
    for f in fens[:150]:
        ep0 = renv.MinitChessEpisode(f)
        if ep0.is_done():
            continue
        for code in sorted(set(ep0.get_legal_moves())):
            ep = renv.MinitChessEpisode(f)
            st = ep.step(code)
            steps.append({'fen': f, 'code': code, 'next': st.observation, 'reward': st.reward, 'done': bool(st.done)})
    golden['encoder'] = enc
    golden['env'] = {'positions': envrows, 'steps': steps}

    # ---- RNG streams (numpy legacy, exp/agent.py:82,115,118) ----------------------------
    rngrows = []
    for seed in range(12):
        rs = np.random.RandomState(seed)
        row = {'seed': seed, 'ops': []}
        for j in range(25):
            k = 1 + (seed * 7 + j * 3) % 19
            d = rs.dirichlet([0.6] * k)
            row['ops'].append({'op': 'dirichlet', 'k': k, 'out': [float(x) for x in d]})
            p = d / d.sum()
            c = rs.choice(list(range(100, 100 + k)), p=p)
            row['ops'].append({'op': 'choice_p', 'p': [float(x) for x in p], 'out': int(c)})
            m = 1 + (seed + j) % 5
            c2 = rs.choice(np.arange(m))
            row['ops'].append({'op': 'choice_m', 'm': m, 'out': int(c2)})
        st = rs.get_state()
        row['final_pos'] = int(st[2])
        row['final_key_head'] = [int(x) for x in st[1][:4]]
        rngrows.append(row)
    golden['rng'] = rngrows

    # ---- net: seed-0 reference Network outputs -------------------------------------
    torch.manual_seed(0)
    net = rpol.Network().eval()
    from oracle.net import state_dict_sha256
    sd_hash = state_dict_sha256(net)
    nfens = fens[:48]
    logits, values = [], []
    with torch.no_grad():
        for f in nfens:
            p, v = net(rpol.Network.process_observation(f))
            logits.append(p[0].numpy())
            values.append(float(v.item()))
    np.savez_compressed(os.path.join(HERE, 'net.npz'), fens=np.array(nfens), logits=np.stack(logits).astype(np.float32),
                        values=np.array(values, dtype=np.float32))
    golden['net'] = {'state_dict_sha256': sd_hash, 'n': len(nfens)}

    # ---- seeded self-play through the reference agent stack ------------------------
    def ref_selfplay(model, sims, seeds):
        env = renv.MinitChessEnvironment()
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
            tr0, tr1 = agents[0]._mcts, agents[1]._mcts
            games.append({'seed': s, 'sims': sims, 'moves': [
                {'observation': r['observation'], 'legal_moves': [int(x) for x in r['legal_moves']],
                 'pi': r['pi'], 'action': r['action'], 'reward': r['reward']} for r in rec],
                'tree_sizes': [len(tr0['visited']), len(tr1['visited'])],
                'nn_nodes': [len(tr0['P']), len(tr1['P'])]})
        return games

    synth = omcts.SyntheticEvaluator(salt=0)
    trees = {'synthetic': ref_selfplay(synth, 32, [0, 1, 2, 3]) + ref_selfplay(synth, 64, [10, 11]),
             'synthetic_salt': 0}
    trees['net_seed0'] = ref_selfplay(net, 32, [0])
    golden['trees'] = trees

    # ---- terminal revisit quirk (exp/agent.py:57-63 vs :75-77) ---------------------------
    # Mate-in-1 positions (Qb1-b6#, and its colour-rotated twin Qd6-d1#): the mating
    # edge's Q must go +1, 0, -1/3 over its first three visits.
    quirk = []
    for f in ['k4/2K2/5/5/5/1Q3 w 0 5', '3q1/5/5/5/2k2/4K b 0 5']:
        env = renv.MinitChessEnvironment()
        np.random.seed(0)
        m = ragent.MonteCarloTreeSearch(env, synth, 1)
        qs = []
        for _ in range(40):
            m.simulate(1, f)
            qs.append([float(x) for x in m['Q'][f]] if f in m['Q'] else None)
        terms = {k: float(v) for k, v in m['terminal'].items()}
        quirk.append({'fen': f, 'Q_after_each_sim': qs, 'N_final': [float(x) for x in m['N'][f]],
                      'legal': [int(x) for x in m['legal_moves'][f]], 'terminal': terms})
    golden['quirk'] = quirk

    for name in ('codec', 'encoder', 'env', 'rng', 'trees', 'quirk', 'net'):
        with open(os.path.join(HERE, f'{name}.json'), 'w') as fh:
            json.dump(golden[name], fh, separators=(',', ':'))
    print('wrote', sorted(golden))


if __name__ == '__main__':
    main()
