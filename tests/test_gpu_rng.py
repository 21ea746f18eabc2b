"""numpy's legacy RandomState on the device (SURVEY a-14): csrc/mtaz_rng.hip.

The Dirichlet sampler the engine's k_noise runs (exp/agent.py:82: np.random.dirichlet([0.6] * k)) is
checked draw for draw against numpy.random.RandomState on more than 10^6 vectors (k = 1 .. 73, many
seeds), including the stream position after the draws; play() with the device RNG (the default)
gives the games of the host RNG bit for bit; and the reference's own games through play() are in
tests/test_gpu_bench_parity.py."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _draw(seeds, ks, n_vec, alpha):
    from minitchess_alphazero_amd import _lib
    L = _lib.lib()
    seeds = np.ascontiguousarray(seeds, np.uint32)
    ks = np.ascontiguousarray(ks, np.int32)
    out = np.zeros(max(1, int(ks.sum()) * n_vec), np.float64)
    tail = np.zeros(len(ks), np.float64)
    _lib.check(L.mtaz_rng_dirichlet_device(0, _lib.ptr(seeds, ctypes.c_uint32), _lib.ptr(ks, ctypes.c_int32), len(ks),
                                           int(n_vec), float(alpha), _lib.ptr(out, ctypes.c_double),
                                           _lib.ptr(tail, ctypes.c_double)))
    return out, tail


def _check(seeds, ks, n_vec, alpha):
    out, tail = _draw(seeds, ks, n_vec, alpha)
    off, bad = 0, []
    for s, (seed, k) in enumerate(zip(seeds, ks)):
        rs = np.random.RandomState(int(seed))
        ref = rs.dirichlet([alpha] * int(k), size=n_vec)
        got = out[off:off + int(k) * n_vec].reshape(n_vec, int(k))
        off += int(k) * n_vec
        if not np.array_equal(got.view(np.uint64), ref.view(np.uint64)):
            i = int(np.argmax((got.view(np.uint64) != ref.view(np.uint64)).any(1)))
            bad.append((int(seed), int(k), i))
        elif tail[s].view(np.uint64) != np.float64(rs.random_sample()).view(np.uint64):
            bad.append((int(seed), int(k), 'tail'))
    return bad


def test_device_dirichlet_equals_numpy_1e6_vectors():
    """1,022,000 Dirichlet(0.6 x k) vectors, k = 1 .. 73 (20 seeds each, seeds 0 .. 3 and 2^32 - 1
    among them), 700 vectors per stream: every double bit-identical to RandomState(seed).dirichlet,
    and the next random_sample() after them too (the stream ends where numpy's does)."""
    ks = np.repeat(np.arange(1, 74), 20)
    seeds = (np.arange(len(ks), dtype=np.uint64) * 7919 + 12345) % (1 << 32)
    seeds[:4] = [0, 1, 2, 3]
    seeds[4] = (1 << 32) - 1
    bad = _check(seeds, ks, 700, 0.6)
    print(f'{len(ks)} streams x 700 vectors: {len(bad)} streams differ', bad[:5])
    assert not bad


@pytest.mark.parametrize('alpha', [0.03, 0.3, 0.9, 0.999])
def test_device_dirichlet_other_alphas(alpha):
    """Other concentrations below 1 (the sampler's two branches in other proportions)."""
    ks = np.repeat(np.array([1, 2, 7, 30, 73, 256]), 8)
    seeds = np.arange(len(ks)) * 31 + 7
    assert not _check(seeds, ks, 64, alpha)


@pytest.mark.parametrize('kind', ['seed0', 'stress5'])
def test_play_device_rng_equals_host_rng(kind):
    """play() with the device RNG (k_noise / k_choose, the default) and with the host RNG: every
    record identical (observations, legal lists, visit counts, actions, rewards), both through the
    sampled opening moves (fullmove < 6: choice with p) and the later argmax picks (randint among
    the maxima)."""
    from minitchess_alphazero_amd.engine import Engine
    from helpers import stress_network
    import torch
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network() if kind == 'seed0' else stress_network('stress5')
    eng = Engine(n_games=96, sims=12, seed_base=17)
    eng.set_weights(net)
    recs = []
    for on in (0, 1):
        eng.set_rng_device(on)
        st = eng.play()
        assert st['rng_device'] == on
        recs.append(eng.records())
    for key in recs[0]:
        assert np.array_equal(recs[0][key], recs[1][key]), key
    assert recs[0]['plies'].sum() > 96 * 20
