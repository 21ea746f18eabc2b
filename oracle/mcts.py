"""MCTS / agent / referee / policy restatement (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates exp/agent.py:6-119 and exp/policy.py:107-125 with two additions that
the reference does not have but the parity tests need:
  * `rng`: a numpy RandomState standing in for the global np.random the
    reference calls (exp/agent.py:82,115,118); RandomState(s) == np.random.seed(s).
  * `cast_mode`: 2 = numpy>=2 (NEP 50) promotion, the semantics the reference
    gets in this container; 1 = numpy 1.x value-based casting, the semantics of
    the deployed reference (py3.8).  They differ only in `P * sqrt(N.sum())`
    at non-root nodes (float64 vs float32) - SURVEY 8a-11.
  * `evaluator`: object with evaluate(fen, legal_moves) -> (P float32[k], v float)
    (the reference inlines this at exp/agent.py:67-69).  `record` optionally
    logs every expansion for replay fixtures.
"""
import numpy as np


class TorchNetEvaluator:
    """Batch-1 torch CPU leaf evaluation exactly as exp/agent.py:67-69."""

    def __init__(self, network):
        import torch
        from .encoder import process_observation
        self.torch = torch
        self.net = network.eval()
        self._proc = process_observation

    def evaluate(self, fen, legal_moves):
        with self.torch.no_grad():
            p, v = self.net(self._proc(fen))
            P = p[0][legal_moves].softmax(0).data.numpy()
            return P, v.item()


class SyntheticEvaluator:
    """Deterministic cheap stand-in net: logits/value are a hash of the FEN.

    Presents both the oracle interface (evaluate) and the reference model
    interface (process_observation + __call__ -> (p[1,554], v[1,1])) so the
    imported reference MCTS can run on it (tests/golden/make_golden.py).
    It draws from its own PCG64 generator, never from the global np.random."""

    def __init__(self, salt=0, scale=2.0):
        import torch
        self.torch = torch
        self.salt = salt
        self.scale = scale

    def raw(self, fen):
        import hashlib
        h = int.from_bytes(hashlib.blake2b(f'{self.salt}|{fen}'.encode(), digest_size=8).digest(), 'little')
        g = np.random.Generator(np.random.PCG64(h))
        logits = (g.standard_normal(554) * self.scale).astype(np.float32)
        v = np.float32(np.tanh(g.standard_normal()))
        return logits, v

    # reference model interface
    def process_observation(self, fen):
        return fen

    def __call__(self, fen):
        logits, v = self.raw(fen)
        return self.torch.from_numpy(logits).reshape(1, 554), self.torch.tensor([[v]], dtype=self.torch.float32)

    def eval(self):
        return self

    def cpu(self):
        return self

    # oracle interface
    def evaluate(self, fen, legal_moves):
        p, v = self(fen)
        return p[0][legal_moves].softmax(0).data.numpy(), v.item()


class MonteCarloTreeSearch:
    """exp/agent.py:24-88 (FEN-keyed transposition DAG)."""

    def __init__(self, environment, evaluator, cpuct, rng=None, cast_mode=2, record=None, trace=None):
        self._environment = environment
        self._evaluator = evaluator
        self._cpuct = cpuct
        self._rng = rng if rng is not None else np.random.mtrand._rand
        self._cast_mode = cast_mode
        self._record = record
        # test instrumentation: every PUCT selection as (node, u, chosen index, N.sum())
        self._trace = trace
        self._data = {'Q': {}, 'N': {}, 'P': {}, 'terminal': {}, 'visited': set(), 'legal_moves': {}}
        self.nn_evals = 0
        self.terminal_hits = 0

    def __getitem__(self, item):                                                  # :38-39
        return self._data.get(item, None)

    def simulate(self, num_simulations, observation):                             # :41-45
        for _ in range(num_simulations):
            episode, _ = self._environment.new_episode(fen=observation)
            self._search(episode, [])
        return self._data

    def _backprop(self, value, chain):                                             # :47-52
        Qd, Nd = self._data['Q'], self._data['N']
        for node, action in chain[::-1]:
            value = -value
            Q, N = Qd[node], Nd[node]
            Q[action] = (N[action] * Q[action] + value) / (N[action] + 1)
            N[action] += 1

    def _puct(self, Q, N, P, root, node=None):                                     # :79-85
        if root:
            k = len(Q)
            P = 0.75 * P + 0.25 * self._rng.dirichlet([0.6] * k)                 # :81-82
        s = np.sqrt(N.sum())
        cp = self._cpuct * P
        if self._cast_mode == 1 and cp.dtype == np.float32:
            # numpy 1.x: float64 scalar x float32 array stays float32 (value-based casting)
            t = cp * np.float32(s)
        else:
            t = cp * s
        u = Q + t / (1 + N)
        a = u.argmax()
        if self._trace is not None:
            self._trace.append((node, u.copy(), int(a), float(N.sum())))
        return a

    def _search(self, episode, chain):                                             # :54-88
        d = self._data
        while True:
            node = episode.get_observation()
            if node not in d['visited']:
                d['visited'].add(node)
                if episode.is_done():
                    value = -episode.get_reward()
                    d['terminal'][node] = value
                    self.terminal_hits += 1
                    self._backprop(value, chain)
                    return
                legal_moves = episode.get_legal_moves()
                d['Q'][node] = np.zeros(len(legal_moves))
                d['N'][node] = np.zeros(len(legal_moves))
                P, v = self._evaluator.evaluate(node, legal_moves)
                self.nn_evals += 1
                if self._record is not None:
                    self._record.append((node, list(legal_moves), np.asarray(P, np.float32).copy(), float(v)))
                d['P'][node] = P
                d['legal_moves'][node] = legal_moves
                self._backprop(v, chain)
                return
            if node in d['terminal']:
                self.terminal_hits += 1
                self._backprop(-d['terminal'][node], chain)                        # sign quirk, SURVEY a-12
                return
            Q, N, P = d['Q'][node], d['N'][node], d['P'][node]
            legal_moves = d['legal_moves'][node]
            action = self._puct(Q, N, P, len(chain) == 0, node)
            episode.step(legal_moves[action], return_status=False)
            chain.append((node, action))


class ActionData:
    __slots__ = ('action', 'info')

    def __init__(self, action, info):
        self.action = action
        self.info = info


class SimpleAlphaZeroPolicy:
    """exp/policy.py:107-125 (get_distribution: pi = N_root / sum N_root)."""

    def __init__(self, evaluator):
        self.evaluator = evaluator

    @property
    def model(self):
        return self.evaluator

    def get_distribution(self, observation, mcts, num_simulations):
        mcts.simulate(num_simulations, observation)
        legal_moves = mcts['legal_moves'][observation]
        N = mcts['N'][observation]
        return {'legal_moves': legal_moves, 'pi': N / N.sum()}

    def num_actions(self):
        return 554


class SimpleAlphaZeroAgent:
    """exp/agent.py:91-119."""

    def __init__(self, environment, policy, num_simulations, cpuct=1, tau_change=6,
                 rng=None, cast_mode=2, record=None, trace=None):
        self._environment = environment
        self.policy = policy
        self._num_simulations = num_simulations
        self._cpuct = cpuct
        self._tau_change = tau_change
        self._rng = rng if rng is not None else np.random.mtrand._rand
        self._cast_mode = cast_mode
        self._record = record
        self._trace = trace
        self.init_mcts()

    def init_mcts(self):
        self._mcts = MonteCarloTreeSearch(self._environment, self.policy.model, self._cpuct,
                                          rng=self._rng, cast_mode=self._cast_mode, record=self._record,
                                          trace=self._trace)

    @property
    def mcts(self):
        return self._mcts

    def select_action(self, observation):
        info = self.policy.get_distribution(observation, self._mcts, self._num_simulations)
        num_moves = int(observation.split()[3])
        if num_moves < self._tau_change:
            action = self._rng.choice(info['legal_moves'], p=info['pi'])
        else:
            maxima = np.where(info['pi'] == info['pi'].max())[0]
            action = info['legal_moves'][self._rng.choice(maxima)]
        return ActionData(action=action, info=info)


class RoundRobinReferee:
    """exp/agent.py:6-21."""

    def __init__(self, agent_tuple):
        self._agent_tuple = tuple(agent_tuple)
        self._turn = False

    def select_action(self, observation):
        action = self._agent_tuple[int(self._turn)].select_action(observation)
        self._turn = not self._turn
        return action

    def reset(self):
        self._turn = False

    @property
    def turn(self):
        return self._turn
