"""GPU: the HBM replay ring (exp/dataset.py:6-20 + collate_fn rows,
exp/learner.py:23-37).  Ingest is checked bit-exact against the reference's own collate output
(tests/golden/learner.npz, made by running the reference's collate_fn) and against the host
path (EpisodeRecords -> dense pi / encoder); the deque(maxlen) semantics across wrap-around,
growth and oversize pushes; an update read from the ring equals one from host records."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import REPO, GOLDEN

pytestmark = pytest.mark.gpu


def _visits_from_pi(pi):
    for s in range(1, 5000):
        n = [round(p * s) for p in pi]
        if sum(n) == s and all(x / s == p for x, p in zip(n, pi)):
            return n
    raise AssertionError('no integer visit vector reproduces pi')


def _records_from_rows(rows):
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.learner import EpisodeRecords
    return EpisodeRecords(np.stack([pos_from_fen(r['observation']) for r in rows]),
                          [len(r['legal_moves']) for r in rows],
                          np.concatenate([np.asarray(r['legal_moves'], np.uint16) for r in rows]),
                          np.concatenate([np.asarray(_visits_from_pi(r['pi']), np.uint32) for r in rows]),
                          np.asarray([r['reward'] for r in rows], np.float32))


def _engine_records(n_games=24, sims=8, seed=0):
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.learner import EpisodeRecords
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(seed)
    eng = Engine(n_games=n_games, sims=sims)
    eng.set_weights(Network())
    eng.set_seed_base(seed * 1000)
    eng.play()
    return EpisodeRecords.from_engine(eng.records())


def _rows_of(buf, n):
    i = torch.arange(n, device='cuda')
    return [t.cpu() for t in buf.gather(i)]


def test_ring_ingest_matches_reference_collate():
    from minitchess_alphazero_amd.learner import ReplayBuffer
    meta = json.load(open(os.path.join(GOLDEN, 'learner.json')))
    z = np.load(os.path.join(GOLDEN, 'learner.npz'))
    rec = _records_from_rows(meta['batch'])
    buf = ReplayBuffer(1000, 'cuda')
    buf.push_records(rec)
    pib, tok, clk, rew = _rows_of(buf, 32)
    assert np.array_equal(pib.numpy(), z['pib'])                  # incl. repeated promotion codes
    assert np.array_equal(tok.numpy(), z['channels'].astype(np.int64))
    assert np.array_equal(clk.numpy(), z['clock'])
    assert np.array_equal(rew.numpy(), z['reward'])


def test_ring_equals_host_rows_through_wraparound():
    from minitchess_alphazero_amd.learner import EpisodeRecords, ReplayBuffer, ResidentBatches
    rec = _engine_records()
    n = len(rec)
    assert n > 300
    buf = ReplayBuffer(250, 'cuda', initial=16)              # grows 16 -> ... -> 250, then wraps
    host = EpisodeRecords.concat([])
    cuts = [0, 7, 100, 101, 260, n]
    for a, b in zip(cuts[:-1], cuts[1:]):
        part = _slice(rec, a, b)
        buf.push_records(part)
        host = EpisodeRecords.concat([host, part]).tail(250)
        assert len(buf) == len(host)
        ref = ResidentBatches(host, 'cuda')
        got = _rows_of(buf, len(buf))
        want = [t.cpu() for t in ref.gather(torch.arange(len(host), device='cuda'))]
        for g, w in zip(got, want):
            assert torch.equal(g, w)
    assert buf.cap == 250 and buf.head != 0                  # the ring did wrap
    # one push larger than max_length keeps only its newest rows
    buf.push_records(rec)
    ref = ResidentBatches(rec.tail(250), 'cuda')
    for g, w in zip(_rows_of(buf, 250), [t.cpu() for t in ref.gather(torch.arange(250, device='cuda'))]):
        assert torch.equal(g, w)
    buf.clear()
    assert len(buf) == 0


def _slice(rec, a, b):
    from minitchess_alphazero_amd.learner import EpisodeRecords
    e = np.concatenate([[0], np.cumsum(rec.k)])
    return EpisodeRecords(rec.pos[a:b], rec.k[a:b], rec.codes[e[a]:e[b]], rec.visits[e[a]:e[b]], rec.reward[a:b])


def test_update_from_ring_equals_update_from_records():
    """The ring feeds update() the same batches, in the same order, as the host records.
    With lr=0 the weights never move, so every batch's loss depends only on its rows: the two
    runs must agree to 1e-6 on all 5 batches.  With lr=1e-3 the first loss is bitwise equal and
    the rest drift by the GPU backward's non-deterministic reductions, which drift the host-record
    path against itself by the same order (test_learner_drift_is_nondeterministic_reduction, which
    also shows the two paths bitwise equal under deterministic algorithms), hence rtol=1e-2 there."""
    from minitchess_alphazero_amd.learner import ReplayBuffer, SimpleAlphaZeroLearner
    from minitchess_alphazero_amd.network import Network
    rec = _engine_records(16, 8, seed=1)
    rec = _slice(rec, 0, 150)

    def run(data, lr):
        torch.manual_seed(0)
        lrn = SimpleAlphaZeroLearner(None, 36, Network(), 32, 1, {'lr': lr}, device='cuda')
        torch.manual_seed(7)
        lrn.update(data)
        return np.array(lrn.last_losses)

    buf = ReplayBuffer(1000, 'cuda')
    buf.push_records(rec)
    a, b = run(rec, 0.0), run(buf, 0.0)
    assert len(a) == len(b) == 5
    assert np.allclose(a, b, rtol=1e-6, atol=0)
    a, b = run(rec, 1e-3), run(buf, 1e-3)
    assert len(a) == len(b) == 5
    assert abs(a[0] - b[0]) <= 1e-6 * abs(a[0]) and np.allclose(a, b, rtol=1e-2)


def test_learner_drift_is_nondeterministic_reduction(record_property):
    """Where the lr > 0 drift between the ring and the host records comes from.  (1) The host-record
    path run twice against itself drifts by the same order (the GPU backward's reductions are not
    bitwise reproducible).  (2) Under torch.use_deterministic_algorithms(True) with deterministic
    MIOpen convolutions, two runs of one path are bitwise equal, and the ring equals the host
    records bitwise: the two paths feed identical batches, and the drift is the reductions'."""
    from minitchess_alphazero_amd.learner import ReplayBuffer, SimpleAlphaZeroLearner
    from minitchess_alphazero_amd.network import Network
    rec = _slice(_engine_records(16, 8, seed=1), 0, 150)
    buf = ReplayBuffer(1000, 'cuda')
    buf.push_records(rec)

    def run(data):
        torch.manual_seed(0)
        lrn = SimpleAlphaZeroLearner(None, 36, Network(), 32, 1, {'lr': 1e-3}, device='cuda')
        torch.manual_seed(7)
        lrn.update(data)
        return np.array(lrn.last_losses)

    a1, a2 = run(rec), run(rec)
    self_drift = float(np.max(np.abs(a1 - a2) / np.abs(a1)))
    prev = (torch.are_deterministic_algorithms_enabled(), torch.backends.cudnn.deterministic,
            torch.backends.cudnn.benchmark)
    torch.use_deterministic_algorithms(True)
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        d1, d2, d3 = run(rec), run(rec), run(buf)
    finally:
        torch.use_deterministic_algorithms(prev[0])
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = prev[1], prev[2]
    msg = (f'records vs records, default algorithms: max relative loss drift {self_drift:.3e}; '
           f'deterministic: {d1.tolist()} / ring {d3.tolist()}')
    record_property('drift', msg)
    print(msg)
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(REPO, 'gpurun_out', 'learner_drift.txt'), 'w') as fh:
        fh.write(msg + '\n')
    assert np.array_equal(d1, d2)
    assert np.array_equal(d1, d3)


def test_learn_puppet_uses_ring():
    from minitchess_alphazero_amd.learner import LearnPuppet
    rec = _engine_records(8, 8, seed=2)
    lp = LearnPuppet('learner', 32, 1, {'lr': 0.02}, device='cuda')
    lp.push_records(rec, 8)
    assert lp._replay is not None and len(lp._replay) == len(rec)
    out = lp.update(encode=False)
    assert np.isfinite(out['loss']) and len(lp._replay) == 0


def test_both_push_paths_share_the_ring_in_arrival_order():
    """A GPU LearnPuppet puts push_data rows (dict rows, the MQTT path) and push_records rows
    (packed engine rows) into one HBM ring in push order: the ring equals the reference collate of
    the rows in that order (exp/dataset.py:12-13 keeps one dataset), with no host copy kept."""
    from minitchess_alphazero_amd.learner import LearnPuppet, ResidentBatches
    rec = _engine_records(6, 8, seed=4)
    rows = rec.to_rows()
    n = len(rows)
    a, b = n // 3, 2 * n // 3
    lp = LearnPuppet('learner', 32, 1, {'lr': 0.02}, device='cuda', max_length=n - 5)
    lp.push_data(rows[:a])
    lp.push_records(rec.slice(a, b), 1)
    lp.push_data(rows[b:])
    assert lp._arrivals == [] and len(lp._replay) == n - 5       # deque(maxlen): the 5 oldest fell out
    ref = ResidentBatches(rows[5:], 'cuda')
    got = _rows_of(lp._replay, n - 5)
    want = [t.cpu() for t in ref.gather(torch.arange(n - 5, device='cuda'))]
    for g, w in zip(got, want):
        assert torch.equal(g, w)
