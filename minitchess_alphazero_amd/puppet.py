"""The app/puppet self-play entry point on the GPU: drop-in for app/base.py's
SimulatePuppet / MQTTDataset / MasterOfPuppetsStatus (app/base.py:41-132).

Same constructor, properties and methods as the reference's SimulatePuppet
(userid, publish_topic, weights_version, remote_status [setter asserts the enum],
remote_version, remote_weights_version, run_episodes(num_episodes, mqtt_client),
load_weights(weights, version), is_simulating()).  The difference is inside
run_episodes: instead of erlyx.run_episodes playing the episodes one after another
on the CPU (app/base.py:116-120), all num_episodes games run in parallel in the HIP
engine, then each episode's InfoRecorder records (exp/callbacks.py:31-54) are
pushed through the same MQTT payload and gates as the reference's MQTTDataset
(app/base.py:52-70); the payloads of a batch are serialized natively from the packed
records (minitchess_alphazero_amd.wire.episode_payloads), byte-identical to json.dumps.

Weights from rlweb: `load_weights_blob(body)` decodes the reference's download_weights body
(zlib + json + jsonpickle, app/base.py:31-39) without unpickling (wire.load_weights_blob).

RNG: the reference plays its episodes one after another, every draw from the global np.random
(app/base.py:113-120).  rng_stream='batched' (the default) plays them in parallel instead, every
game on its own numpy-legacy stream seeded from one np.random.randint draw per batch, so seeding
np.random still makes a run reproducible (game i of a batch plays as the reference does after
np.random.seed(seed_base + i)).  rng_stream='global' keeps the reference's stream exactly: the
episodes run in sequence through the drop-in agent stack (erlyx run_episodes + RoundRobinReferee +
SimpleAlphaZeroAgent + InfoRecorder + MonteCarloInit, app/base.py:112-120 line for line), one game
at a time on the GPU engine, so the payloads are those the reference publishes after the same
np.random.seed (as fast as one game's search allows, not the batched throughput).

Command line (no MQTT broker needed):
    python -m minitchess_alphazero_amd.puppet --episodes 64 --sims 36 --out episodes.jsonl
"""
import json
import logging
import os
from enum import IntEnum

import numpy as np

from .network import Network

NUM_SIMULATIONS = 36                                                   # app/base.py:25
MINITCHESS_ALPHAZERO_VERSION = os.getenv('MINITCHESS_ALPHAZERO_VERSION')


class MasterOfPuppetsStatus(IntEnum):                                  # app/base.py:41-44
    OFF = 1
    SIMULATE = 2
    TRAIN = 3


class MQTTDataset:
    """app/base.py:47-70: publish one episode per push, gated on status and version."""

    def __init__(self, mqtt_client, puppet):
        self._puppet = puppet
        self._client = mqtt_client

    def _gate(self):
        p = self._puppet
        if p.remote_status != MasterOfPuppetsStatus.SIMULATE:
            logging.info('Not pushing episode. Master Status is not SIMULATE')
            return False
        if p.remote_version != MINITCHESS_ALPHAZERO_VERSION:
            logging.info('Not pushing episode. Master version differs')
            return False
        return True

    def push(self, data):
        if not self._gate():
            return True
        p = self._puppet
        payload = {'episode': data, 'userid': p.userid, 'weights_version': p.weights_version,
                   'minitchess_alphazero_version': MINITCHESS_ALPHAZERO_VERSION}
        self.push_payload(json.dumps(payload), gated=True)

    def push_payload(self, payload, gated=False):
        """push() for a payload already serialized (wire.episode_payloads writes the same bytes
        json.dumps would); same gates."""
        if not gated and not self._gate():
            return True
        info = self._client.publish(self._puppet.publish_topic, payload, qos=2)
        logging.info(f'published episode with mid={getattr(info, "mid", None)}')


class SimulatePuppet:
    def __init__(self, userid, publish_topic, num_simulations=NUM_SIMULATIONS, device=0, max_parallel=4096,
                 rng_stream='batched'):
        if rng_stream not in ('batched', 'global'):
            raise ValueError(f"rng_stream must be 'batched' or 'global', not {rng_stream!r}")
        self._rng_stream = rng_stream
        self._network = Network().eval()
        self._userid = userid
        self._publish_topic = publish_topic
        self._is_simulating = False
        self._weights_version = None
        self._remote_status = None
        self.remote_weights_version = None
        self.remote_version = None
        self._sims = num_simulations
        self._device = device
        self._max_parallel = max_parallel
        self._engine = None
        self._engine_games = 0
        self._weights_dirty = True

    @property
    def userid(self):
        return self._userid

    @property
    def publish_topic(self):
        return self._publish_topic

    @property
    def weights_version(self):
        return self._weights_version

    @property
    def remote_status(self):
        return self._remote_status

    @remote_status.setter
    def remote_status(self, status):
        assert isinstance(status, MasterOfPuppetsStatus)
        self._remote_status = status

    def load_weights(self, weights, version):
        logging.info(f'Loading weights {version} ...')
        self._network.load_state_dict(weights)
        self._weights_version = version
        self._weights_dirty = True

    def load_weights_blob(self, blob):
        """download_weights() + load_weights(): the rlweb /get_weights body, decoded safely."""
        from .wire import load_weights_blob
        content = load_weights_blob(blob)
        self.load_weights(content['weights'], content['version'])
        return content['version']

    def is_simulating(self):
        return self._is_simulating

    def _engine_for(self, n_games, seed_base):
        from .engine import Engine
        if self._engine is None or self._engine_games < n_games:
            self._engine = Engine(n_games=n_games, sims=self._sims, device=self._device, seed_base=seed_base)
            self._engine_games = n_games
            self._weights_dirty = True
        self._engine.set_seed_base(seed_base)
        if self._weights_dirty:
            self._engine.set_weights(self._network)
            self._weights_dirty = False
        return self._engine

    def _batches(self, num_episodes):
        left = num_episodes
        while left > 0:
            n = min(left, self._max_parallel)
            seed_base = int(np.random.randint(0, 2 ** 31 - n))
            eng = self._engine_for(n, seed_base)
            eng.play(n_games=n)
            yield eng, n
            left -= n

    def play(self, num_episodes):
        """Play num_episodes games in parallel batches; returns InfoRecorder records."""
        out = []
        for eng, n in self._batches(num_episodes):
            out.extend(eng.episodes()[:n])
        return out

    def play_payloads(self, num_episodes):
        """The games of play() as MQTT payloads, written natively (wire.episode_payloads):
        the bytes MQTTDataset.push would publish for each episode."""
        from .wire import episode_payloads
        for eng, n in self._batches(num_episodes):
            yield from episode_payloads(eng.records(), self.userid, self.weights_version,
                                        MINITCHESS_ALPHAZERO_VERSION)[:n]

    def _run_sequential(self, num_episodes, dataset):
        """rng_stream='global': app/base.py:112-120 over the drop-in stack, episodes in sequence."""
        import torch
        from .agent import RoundRobinReferee, SimpleAlphaZeroAgent
        from .callbacks import InfoRecorder, MonteCarloInit
        from .environment import MinitChessEnvironment
        from .erlyx_compat import run_episodes
        from .policy import SimpleAlphaZeroPolicy
        env = MinitChessEnvironment()
        policy = SimpleAlphaZeroPolicy(network=self._network)
        agents = [SimpleAlphaZeroAgent(environment=env, policy=policy, num_simulations=self._sims,
                                       device=self._device) for _ in range(2)]
        callbacks = [InfoRecorder(dataset), MonteCarloInit(agents[0]), MonteCarloInit(agents[1])]
        with torch.no_grad():
            run_episodes(env, RoundRobinReferee(agent_tuple=tuple(agents)), num_episodes, callbacks=callbacks,
                         use_tqdm=False)

    def run_episodes(self, num_episodes, mqtt_client):
        """app/base.py:108-124: any Exception is logged and swallowed; the
        BaseException game errors propagate, as in the reference."""
        try:
            self._is_simulating = True
            logging.info('Starting simulations')
            dataset = MQTTDataset(mqtt_client, self)
            if self._rng_stream == 'global':
                self._run_sequential(num_episodes, dataset)
                return
            for payload in self.play_payloads(num_episodes):
                dataset.push_payload(payload)
        except Exception as e:
            logging.error(f'Exception occurred: {e}')
        finally:
            self._is_simulating = False


class _JsonlClient:
    """Stand-in MQTT client for the command line: appends payloads to a file."""

    class _Info:
        mid = 0

    def __init__(self, path):
        self._fh = open(path, 'a')

    def publish(self, topic, payload, qos=0):
        self._fh.write(payload + '\n')
        self._fh.flush()
        return self._Info()


def main(argv=None):
    import argparse
    import torch
    ap = argparse.ArgumentParser(description='GPU self-play puppet (app/puppet drop-in)')
    ap.add_argument('--episodes', type=int, default=10)                  # app/puppet.py:72
    ap.add_argument('--sims', type=int, default=NUM_SIMULATIONS)
    ap.add_argument('--device', type=int, default=0)
    ap.add_argument('--weights', help='torch state_dict file (weights_only load)')
    ap.add_argument('--seed', type=int, default=None)
    ap.add_argument('--out', default='episodes.jsonl')
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if args.seed is not None:
        np.random.seed(args.seed)
        torch.manual_seed(args.seed)
    global MINITCHESS_ALPHAZERO_VERSION
    MINITCHESS_ALPHAZERO_VERSION = MINITCHESS_ALPHAZERO_VERSION or 'local'
    puppet = SimulatePuppet(os.getenv('USERID', 'local'), 'episodes', num_simulations=args.sims, device=args.device)
    if args.weights:
        puppet.load_weights(torch.load(args.weights, map_location='cpu', weights_only=True), 'file')
    puppet.remote_status = MasterOfPuppetsStatus.SIMULATE
    puppet.remote_version = MINITCHESS_ALPHAZERO_VERSION
    puppet.run_episodes(args.episodes, _JsonlClient(args.out))


if __name__ == '__main__':
    main()
