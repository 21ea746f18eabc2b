#!/usr/bin/env python3
"""Round-5 golden fixture: the reference puppet's sequential global random stream (VERDICT r4 missing #5).

SimulatePuppet.run_episodes (/root/reference/app/base.py:108-124) plays its episodes one after the
other through erlyx.run_episodes with ONE RoundRobinReferee and the one global legacy np.random
stream: nothing reseeds between episodes, and the referee's turn carries over.  This script runs
the REFERENCE agent stack that way (exp/agent.py, exp/environment.py, exp/policy.py,
exp/callbacks.py under the same stubs as make_golden.py: the un-vendored erlyx loop restated from
its call sites, oracle.rules as `chess`) for two consecutive episodes after one np.random.seed(11),
with the reference Network at torch.manual_seed(0) initialisation and 8 simulations per move, and
records:

  stream.json   seed, sims, both episodes' InfoRecorder records (observation, legal_moves, pi,
                action, reward per move), and the global RandomState position after the second
                episode (the sha256 of its key array and its index), so that a drop-in puppet with
                rng_stream='global' can be checked draw for draw (tests/test_gpu_dropin.py)

Usage: python tests/golden/make_golden_r5_stream.py   (build container only; about a minute)
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from make_golden import import_reference  # noqa: E402

SEED, SIMS, EPISODES = 11, 8, 2


def main():
    torch.set_num_threads(8)
    renv, rpol, ragent, rcb = import_reference()
    t0 = time.time()
    torch.manual_seed(0)
    net = rpol.Network()
    net.eval()
    env = renv.MinitChessEnvironment()
    policy = rpol.SimpleAlphaZeroPolicy(network=net)
    agents = [ragent.SimpleAlphaZeroAgent(environment=env, policy=policy, num_simulations=SIMS) for _ in range(2)]
    sink = []

    class DS:
        def push(self, data):
            sink.append(data)

    callbacks = [rcb.InfoRecorder(DS()), rcb.MonteCarloInit(agents[0]), rcb.MonteCarloInit(agents[1])]
    np.random.seed(SEED)
    with torch.no_grad():
        sys.modules['erlyx'].run_episodes(env, ragent.RoundRobinReferee(agent_tuple=tuple(agents)), EPISODES,
                                          callbacks=callbacks, use_tqdm=False)
    st = np.random.get_state()
    eps = [[{'observation': r['observation'], 'legal_moves': [int(x) for x in r['legal_moves']], 'pi': r['pi'],
             'action': r['action'], 'reward': r['reward']} for r in rec] for rec in sink]
    out = {'seed': SEED, 'sims': SIMS, 'episodes': eps, 'weights': 'torch.manual_seed(0); Network()',
           'rng_after': {'key_sha256': hashlib.sha256(st[1].tobytes()).hexdigest(), 'pos': int(st[2])}}
    with open(os.path.join(HERE, 'stream.json'), 'w') as fh:
        json.dump(out, fh, separators=(',', ':'))
    print(json.dumps({'episodes': [len(e) for e in eps], 'rewards': [e[-1]['reward'] for e in eps],
                      'rng_pos': int(st[2]), 'seconds': round(time.time() - t0, 1)}))


if __name__ == '__main__':
    main()
