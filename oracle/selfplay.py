"""The app/puppet self-play loop on the CPU (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates what SimulatePuppet.run_episodes (app/base.py:108-124) drives:
two SimpleAlphaZeroAgents sharing one network, a RoundRobinReferee,
InfoRecorder + MonteCarloInit callbacks (exp/callbacks.py:31-62), and the
erlyx episode loop (un-vendored; contract inferred from the callback
signatures).  This is also bench.py's `cpu_baseline` leg
(batch-1 torch-CPU forward per leaf, FEN-keyed dict tables, Python rules).

Harness seeding: game g runs with RandomState(seed) where
seed = seed_base + g, equivalent to np.random.seed(seed) at episode start.
"""
import time

import numpy as np

from .environment import MinitChessEnvironment
from .mcts import RoundRobinReferee, SimpleAlphaZeroAgent, SimpleAlphaZeroPolicy


class InfoRecorder:
    """exp/callbacks.py:31-54 (records + alternating-sign reward back-fill)."""

    def __init__(self, sink):
        self._sink = sink

    def on_episode_begin(self, initial_observation):
        self._episode_record = []
        self._observation = initial_observation
        self._episode_reward = None

    def on_step_end(self, action, observation, reward, done):
        info = {'observation': self._observation}
        info.update(action.info)
        info['action'] = int(action.action)
        info['pi'] = info['pi'].tolist()
        self._episode_record.append(info)
        self._episode_reward = reward
        self._observation = observation

    def on_episode_end(self):
        reward = self._episode_reward
        for info in self._episode_record[::-1]:
            info['reward'] = reward
            reward = -reward
        self._sink.append(self._episode_record)


def run_episodes(env, agent, num_episodes, callbacks, on_episode_start=None):
    """erlyx.run_episodes contract (app/base.py:116-120)."""
    for ep in range(num_episodes):
        if on_episode_start is not None:
            on_episode_start(ep)
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


class _MCInit:
    def __init__(self, agent):
        self.agent = agent

    def on_episode_begin(self, obs):
        self.agent.init_mcts()

    def on_step_end(self, *a):
        pass

    def on_episode_end(self):
        pass


def play_games(evaluator, num_games, sims, seed_base=0, cpuct=1, tau_change=6, cast_mode=2,
               record=None, stats=None, trace=None, start_fen=None):
    """Play `num_games` seeded self-play games; return the list of episode records.
    `evaluator` may be a pair: agent 0 (first mover, exp/agent.py:11-14) uses the first, agent 1
    the second (the arena of the commented exp/learner.py:97-145)."""
    env = MinitChessEnvironment()
    if start_fen is not None:
        # every episode from start_fen (exp/environment.py new_episode's fen argument)
        base_new = env.new_episode
        env.new_episode = lambda fen=None: base_new(fen or start_fen)
    rng = np.random.RandomState(seed_base)
    evs = tuple(evaluator) if isinstance(evaluator, (tuple, list)) else (evaluator, evaluator)
    agents = [SimpleAlphaZeroAgent(env, SimpleAlphaZeroPolicy(evs[i]), sims, cpuct, tau_change, rng=rng,
                                   cast_mode=cast_mode, record=record, trace=trace) for i in range(2)]
    sink = []
    referee = RoundRobinReferee(agents)
    callbacks = [InfoRecorder(sink), _MCInit(agents[0]), _MCInit(agents[1])]

    def start(ep):
        rng.seed(seed_base + ep)
        referee.reset()

    t0 = time.perf_counter()
    evals = [0]
    terms = [0]

    class _Count:
        def on_episode_begin(self, obs):
            pass

        def on_step_end(self, *a):
            pass

        def on_episode_end(self):
            evals[0] += agents[0].mcts.nn_evals + agents[1].mcts.nn_evals
            terms[0] += agents[0].mcts.terminal_hits + agents[1].mcts.terminal_hits
            if stats is not None:
                # agent i's table; agent 0 moved first because the referee is reset per game
                stats.setdefault('trees', []).append((agents[0].mcts._data, agents[1].mcts._data))

    run_episodes(env, referee, num_games, callbacks + [_Count()], on_episode_start=start)
    if stats is not None:
        stats['seconds'] = time.perf_counter() - t0
        stats['nn_evals'] = evals[0]
        stats['terminal_hits'] = terms[0]
        stats['plies'] = sum(len(r) for r in sink)
    return sink
