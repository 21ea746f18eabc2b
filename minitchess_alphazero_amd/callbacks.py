"""Self-play callbacks with the reference's hook contract (exp/callbacks.py).

On the self-play path: InfoRecorder (exp/callbacks.py:31-54: one record per step,
reward back-filled from the last step with alternating sign, then dataset.push) and
MonteCarloInit (:57-62: fresh tree per episode).  WinnerRecorder, RefereeInit and
WeightUpdater (:7-28, :64-83) are bookkeeping kept for API completeness.

Records keep the reference's key order (observation, legal_moves, pi, action, reward)
so JSON payloads serialise identically.
"""
from .erlyx_compat import BaseCallback


def backfill_rewards(records, last_reward):
    """records[-1] gets last_reward, records[-2] its negation, ... (-0.0 for draws, as
    the reference's repeated `reward = -reward`)."""
    r = last_reward
    for rec in reversed(records):
        rec['reward'] = r
        r = -r
    return records


class InfoRecorder(BaseCallback):
    def __init__(self, dataset):
        self._sink = dataset
        self._steps = []
        self._before = None
        self._final = None

    def on_episode_begin(self, initial_observation):
        self._steps, self._before, self._final = [], initial_observation, None

    def on_step_end(self, action, observation, reward, done):
        rec = dict(observation=self._before, **action.info)
        rec['action'] = int(action.action)
        rec['pi'] = rec['pi'].tolist()
        self._steps.append(rec)
        self._before, self._final = observation, reward

    def on_episode_end(self):
        return self._sink.push(backfill_rewards(self._steps, self._final))


class MonteCarloInit(BaseCallback):
    def __init__(self, agent):
        self._agent = agent

    def on_episode_begin(self, initial_observation):
        self._agent.init_mcts()


class RefereeInit(BaseCallback):
    def __init__(self, referee):
        self._referee = referee

    def on_episode_begin(self, initial_observation):
        self._referee.reset()


class WinnerRecorder(BaseCallback):
    """Counts decisive games per side: the winner is the side that made the last move."""

    def __init__(self, referee):
        self._referee = referee
        self._wins = {False: 0, True: 0}
        self._end_reward = None

    def on_episode_begin(self, initial_observation):
        self._end_reward = None

    def on_step_end(self, action, observation, reward, done):
        if done:
            self._end_reward = reward

    def on_episode_end(self):
        assert self._end_reward is not None
        if self._end_reward != 0:
            side = not self._referee.turn
            self._wins[side] += 1

    @property
    def results(self):
        return dict(self._wins)


class WeightUpdater(BaseCallback):
    """Calls learner.update(dataset) every `update_interval` episodes after `init_episodes`."""

    def __init__(self, learner, dataset, update_interval, init_episodes=0):
        self._learner, self._dataset = learner, dataset
        self._every = update_interval
        self._seen = -init_episodes

    def on_episode_end(self):
        self._seen += 1
        if self._seen > 0 and self._seen % self._every == 0:
            self._seen = 0
            self._learner.update(self._dataset)
