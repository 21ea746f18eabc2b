"""erlyx plugin surface (the reference's un-vendored RL framework, README.md:7).

erlyx is not installable offline.  Its contract is inferred from the reference's
call sites: app/base.py:14,116-120 (run_episodes) and the base classes
imported by exp/agent.py:1-2, exp/environment.py:2-4, exp/policy.py:1,
exp/callbacks.py:4, exp/learner.py:8.  `install()` registers these as the `erlyx`
package when the real one is absent, so reference-style imports keep working.
"""
import sys
import types
from collections import namedtuple

ActionData = namedtuple('ActionData', ['action', 'info'])
EpisodeStatus = namedtuple('EpisodeStatus', ['observation', 'reward', 'done'])


class BaseAgent:
    def select_action(self, observation):
        raise NotImplementedError


class PolicyAgent(BaseAgent):
    def __init__(self, policy):
        self._policy = policy

    @property
    def policy(self):
        return self._policy


class Policy:
    pass


class BaseEnvironment:
    def new_episode(self, fen=None):
        raise NotImplementedError


class Episode:
    pass


class BaseLearner:
    pass


class BaseCallback:
    def on_episode_begin(self, initial_observation):
        pass

    def on_step_end(self, action, observation, reward, done):
        pass

    def on_episode_end(self):
        pass


def run_episodes(environment, agent, num_episodes, callbacks=(), use_tqdm=False):
    """Episode loop: new_episode -> on_episode_begin -> [select_action -> step ->
    on_step_end]* -> on_episode_end (callback signatures exp/callbacks.py:13-24,35-54)."""
    for _ in range(num_episodes):
        episode, observation = environment.new_episode()
        for cb in callbacks:
            cb.on_episode_begin(observation)
        done = False
        while not done:
            action = agent.select_action(observation)
            observation, reward, done = episode.step(action.action)
            for cb in callbacks:
                cb.on_step_end(action, observation, reward, done)
        for cb in callbacks:
            cb.on_episode_end()


def install(force=False):
    """Expose this module as `erlyx` (+ submodules) unless a real erlyx is importable."""
    if not force:
        try:
            import erlyx  # noqa: F401
            return False
        except ImportError:
            pass
    me = sys.modules[__name__]
    root = types.ModuleType('erlyx')
    root.run_episodes = run_episodes
    subs = {
        'agents': {'BaseAgent': BaseAgent, 'PolicyAgent': PolicyAgent},
        'types': {'ActionData': ActionData, 'EpisodeStatus': EpisodeStatus},
        'policies': {'Policy': Policy},
        'environment': {'BaseEnvironment': BaseEnvironment, 'Episode': Episode},
        'learners': {'BaseLearner': BaseLearner},
        'callbacks': {'BaseCallback': BaseCallback},
    }
    sys.modules['erlyx'] = root
    for name, attrs in subs.items():
        m = types.ModuleType('erlyx.' + name)
        for k, v in attrs.items():
            setattr(m, k, v)
        setattr(root, name, m)
        sys.modules['erlyx.' + name] = m
    del me
    return True
