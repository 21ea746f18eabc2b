"""GPU: the wire formats on engine output.  Episode payloads written natively
from a batch of GPU self-play games are byte-identical to the reference's json.dumps of the
same InfoRecorder records (oracle/wire.py, app/base.py:63-69); a weights blob (zlib + json +
jsonpickle document) loaded into a puppet drives the engine exactly like the original weights."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_engine_payloads_equal_reference_json():
    import oracle.wire as ow
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    from minitchess_alphazero_amd.wire import episode_payloads
    torch.manual_seed(0)
    eng = Engine(n_games=256, sims=8)
    eng.set_weights(Network())
    eng.play()
    t0 = time.perf_counter()
    got = episode_payloads(eng.records(), 'gpu-puppet', '20240101120000', 'v1')
    t1 = time.perf_counter()
    eps = eng.episodes()
    want = [ow.episode_payload(ep, 'gpu-puppet', '20240101120000', 'v1') for ep in eps]
    t2 = time.perf_counter()
    assert len(got) == len(want) == 256
    for g in range(256):
        assert got[g] == want[g], g
    print(f'payloads: native {t1 - t0:.3f}s, episodes()+json.dumps {t2 - t1:.3f}s')


def test_puppet_native_payloads_equal_python_path():
    import oracle.wire as ow
    from minitchess_alphazero_amd import puppet as pp
    pp.MINITCHESS_ALPHAZERO_VERSION = 'v-test'
    p = pp.SimulatePuppet('u1', 'topic/eps', num_simulations=8)
    np.random.seed(5)
    native = list(p.play_payloads(7))
    np.random.seed(5)
    eps = p.play(7)
    assert len(native) == len(eps) == 7
    for a, ep in zip(native, eps):
        assert a == ow.episode_payload(ep, 'u1', None, 'v-test')


def test_weights_blob_into_puppet_engine():
    from minitchess_alphazero_amd import puppet as pp
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import STARTING_FEN, pos_from_fen
    from minitchess_alphazero_amd.learner import LearnPuppet
    from minitchess_alphazero_amd.wire import weights_blob
    torch.manual_seed(2)
    lp = LearnPuppet('learner', 32, 1, {'lr': 0.2}, device='cuda')
    blob = weights_blob(lp.get_weights_dict())
    p = pp.SimulatePuppet('u1', 'topic', num_simulations=8)
    assert p.load_weights_blob(blob) == lp.weights_version
    pos = np.stack([pos_from_fen(STARTING_FEN)] * 4)
    a = Engine(n_games=8, sims=4)
    a.set_weights(lp.weights)
    b = Engine(n_games=8, sims=4)
    b.set_weights(p._network)
    la, va = a.evaluate(pos)
    lb, vb = b.evaluate(pos)
    assert np.array_equal(la, lb) and np.array_equal(va, vb)
