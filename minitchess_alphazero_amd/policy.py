"""Drop-in for the reference's exp/policy.py: Network + SimpleAlphaZeroPolicy.

Network is the weight container of network.py (same state_dict as the reference);
SimpleAlphaZeroPolicy.get_distribution keeps exp/policy.py:115-122: run the search,
then pi = N / N.sum() over the root's legal list.
"""
from .erlyx_compat import Policy
from .network import EMBEDDING_DIM, MAX_NUM_MOVES_ALLOWED, NUM_ACTIONS, Network  # noqa: F401

CODES = {v: k for k, v in enumerate('0prbnqk')}   # exp/policy.py:7


class SimpleAlphaZeroPolicy(Policy):
    def __init__(self, network=None):
        self._network = network or Network()

    @property
    def model(self):
        return self._network

    def get_distribution(self, observation, mcts, num_simulations):
        mcts.simulate(num_simulations, observation)
        legal_moves = mcts['legal_moves'][observation]
        N = mcts['N'][observation]
        return {'legal_moves': legal_moves, 'pi': N / N.sum()}

    def num_actions(self):
        return NUM_ACTIONS
