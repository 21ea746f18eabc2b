"""Drop-in for the reference's exp/agent.py (RoundRobinReferee, MonteCarloTreeSearch,
SimpleAlphaZeroAgent) with the search running in the HIP engine.

Semantics kept from the reference:
  * one transposition table per MonteCarloTreeSearch object, persisting across moves
    until init_mcts() (exp/agent.py:25-39, :105-108);
  * `simulate(n, fen)` runs n sequential simulations from `fen` (exp/agent.py:41-45);
  * root Dirichlet noise and the action choice draw from the GLOBAL np.random, in the
    reference's order (exp/agent.py:82, :115, :118), so a caller that seeds
    np.random gets the reference's stream;
  * `mcts['Q'|'N'|'P'|'legal_moves'|'terminal'|'visited']` views keyed by FEN.
"""
import numpy as np

from .erlyx_compat import ActionData, BaseAgent, PolicyAgent
from .environment import pos_from_fen


class RoundRobinReferee(BaseAgent):
    """exp/agent.py:6-21: agent 0 moves when turn is False, then the turn flips.
    (app/puppet never resets it between episodes; both agents are identical there.)"""

    def __init__(self, agent_tuple):
        self._agents = tuple(agent_tuple)
        self._turn = False

    def select_action(self, observation):
        mover = self._agents[1 if self._turn else 0]
        chosen = mover.select_action(observation)
        self._turn = not self._turn
        return chosen

    def reset(self):
        self._turn = False

    @property
    def turn(self):
        return self._turn


def _weights_key(model):
    return (id(model), tuple(t._version for t in model.state_dict().values()))


class MonteCarloTreeSearch:
    """exp/agent.py:24-88 on the GPU: a one-game engine whose table 0 is this tree."""

    def __init__(self, environment, model, cpuct, device=0, cast_mode=2, capacity=None):
        self._environment = environment
        self._model = model
        self._cpuct = cpuct
        self._device = device
        self._cast_mode = cast_mode
        self._capacity = capacity     # simulations per move the engine is first sized for (None: the first call's)
        self._engine = None
        self._sims = None
        self._wkey = None
        self._view = None

    def _engine_for(self, n):
        """The one-game engine, sized for n simulations per move.  A later call with more
        simulations than the engine was sized for (the reference has no such limit,
        exp/agent.py:41-45) moves the table into a larger engine (mtaz_tree_set)."""
        from .engine import Engine
        if self._engine is None or n > self._sims:
            sims = max(n, self._capacity or 0)
            eng = Engine(n_games=1, sims=sims, device=self._device, cpuct=self._cpuct, cast_mode=self._cast_mode)
            eng.clear_trees()
            if self._engine is not None:
                eng.set_tree(0, self._engine.tree_arrays(0))
                self._engine.close()
            self._engine, self._sims, self._wkey = eng, sims, None
        key = _weights_key(self._model)
        if key != self._wkey:
            self._engine.set_weights(self._model)
            self._wkey = key
        return self._engine

    def simulate(self, num_simulations, observation):
        eng = self._engine_for(num_simulations)
        eng.set_games([pos_from_fen(observation)], agents=[0])
        k, new = eng.move_begin()
        k, new = int(k[0]), int(new[0])
        draws = num_simulations - new
        noise = np.stack([np.random.dirichlet([0.6] * k) for _ in range(draws)]) if draws > 0 else None
        eng.set_noise([noise])
        eng.simulate(0, num_simulations)
        self._view = None
        return self._data

    @property
    def _data(self):
        if self._view is None:
            self._view = self._engine.tree(0) if self._engine is not None else {
                'Q': {}, 'N': {}, 'P': {}, 'terminal': {}, 'visited': set(), 'legal_moves': {}}
        return self._view

    def __getitem__(self, item):
        return self._data.get(item, None)


class SimpleAlphaZeroAgent(PolicyAgent):
    """exp/agent.py:91-119: search, then sample a move proportionally to the root visit
    counts while the fullmove number is below tau_change, else play a most-visited move
    (ties broken uniformly at random)."""

    def __init__(self, environment, policy, num_simulations, cpuct=1, tau_change=6, device=0):
        super().__init__(policy)
        self._environment = environment
        self._num_simulations = num_simulations
        self._cpuct = cpuct
        self._tau_change = tau_change
        self._device = device     # (not in the reference: the GPU the one-game engines run on)
        self.init_mcts()

    def init_mcts(self):
        self._mcts = MonteCarloTreeSearch(self._environment, self.policy.model, self._cpuct, device=self._device)

    def select_action(self, observation):
        dist = self.policy.get_distribution(observation, self._mcts, self._num_simulations)
        moves, pi = dist['legal_moves'], dist['pi']
        if int(observation.split()[3]) < self._tau_change:
            chosen = np.random.choice(moves, p=pi)
        else:
            best = np.flatnonzero(pi == pi.max())
            chosen = moves[np.random.choice(best)]
        return ActionData(action=chosen, info=dist)
