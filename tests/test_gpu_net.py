"""GPU: HIP network (fp32 MFMA trunk) vs the reference's torch-CPU forward.

Tolerance (north_star): priors and values within 1e-5 (fp32).  Priors are the
legal-code softmax of the logits (exp/agent.py:68); we also bound the raw
logits at 1e-4 absolute."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_golden

pytestmark = pytest.mark.gpu

PRIOR_TOL = 1e-5
VALUE_TOL = 1e-5
LOGIT_TOL = 1e-4


def _softmax(x):
    x = x.astype(np.float64)
    e = np.exp(x - x.max())
    return e / e.sum()


# f16x3 = product fused kernel k_net_y (16x16x32 MFMA) and its A/B schedules (4, 64, 128);
# f16x3-x* = k_net_x (32x32x16 MFMA, variant bit 512) and its schedules; fp32 = fp32 MFMA path
NET_KERNELS = {'f16x3': ('f16x3', 0), 'fp32': ('fp32', 0), 'f16x3-y4': ('f16x3', 4), 'f16x3-y128': ('f16x3', 128),
               'f16x3-y64': ('f16x3', 64), 'f16x3-x': ('f16x3', 512)}


@pytest.fixture(scope='module', params=list(NET_KERNELS))
def engine(request):
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.network import Network
    import torch
    eng = Engine(n_games=64, sims=8)
    prec, var = NET_KERNELS[request.param]
    eng.set_precision(prec)
    eng.set_net_variant(var)
    torch.manual_seed(0)
    net = Network()
    eng.set_weights(net)
    return eng


def test_seed0_weights_match_reference_hash():
    import torch
    from minitchess_alphazero_amd.network import Network
    from oracle.net import state_dict_sha256
    torch.manual_seed(0)
    assert state_dict_sha256(Network()) == load_golden('net')['state_dict_sha256']


def test_net_vs_reference_outputs(engine):
    from minitchess_alphazero_amd.environment import pos_from_fen, pos_legal
    z = np.load(os.path.join(GOLDEN, 'net.npz'))
    fens = [str(f) for f in z['fens']]
    pos = np.stack([pos_from_fen(f) for f in fens])
    logits, values = engine.evaluate(pos)
    assert np.max(np.abs(logits - z['logits'])) <= LOGIT_TOL
    assert np.max(np.abs(values - z['values'])) <= VALUE_TOL
    for i, f in enumerate(fens):
        legal = pos_legal(pos[i])
        if not legal:
            continue
        ref = _softmax(z['logits'][i][legal])
        got = _softmax(logits[i][legal])
        assert np.max(np.abs(got - ref)) <= PRIOR_TOL


def test_net_vs_torch_cpu_many_positions(engine):
    """Larger random sample: batch sizes that are odd / exceed the engine slots."""
    import torch
    from minitchess_alphazero_amd.environment import pos_from_fen
    from oracle.encoder import process_observation
    from oracle.net import seed0_network
    from tests_positions import random_fens
    fens = random_fens(301, seed=11)
    pos = np.stack([pos_from_fen(f) for f in fens])
    logits, values = engine.evaluate(pos)
    net = seed0_network()
    worst = 0.0
    with torch.no_grad():
        for i, f in enumerate(fens):
            p, v = net(process_observation(f))
            worst = max(worst, float(np.max(np.abs(p[0].numpy() - logits[i]))))
            assert abs(float(v.item()) - float(values[i])) <= VALUE_TOL
    assert worst <= LOGIT_TOL


def test_mix_epilogue_bit_identical():
    """k_net_y's product epilogue (v_fma_mix forms) stores exactly the bits of the unfused
    expressions (variant 1024): logits and values of the two builds must be bitwise equal."""
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.network import Network
    from tests_positions import random_fens
    import torch
    eng = Engine(n_games=64, sims=8)
    torch.manual_seed(0)
    eng.set_weights(Network())
    pos = np.stack([pos_from_fen(f) for f in random_fens(257, seed=5)])
    eng.set_net_variant(0)
    l0, v0 = eng.evaluate(pos)
    eng.set_net_variant(1024)
    l1, v1 = eng.evaluate(pos)
    assert np.array_equal(l0.view(np.uint32), l1.view(np.uint32))
    assert np.array_equal(v0.view(np.uint32), v1.view(np.uint32))
