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


# every build the product library accepts (mtaz_set_net_variant): f16f8 = k_net_z (an option,
# within 1e-5 on the seed-0 and C3 nets only), f16f6 = k_net_z with e2m3 cross terms, f16x3 =
# k_net_y (the default), fp32 = the fp32 MFMA path
NET_KERNELS = {'f16f8': ('f16f8', 0), 'f16f6': ('f16f8', 8192), 'f16x3': ('f16x3', 0), 'fp32': ('fp32', 0)}


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


def _diag_child(*args):
    """Run a round-3 comparison of tests/diag_round3.py in a child process on the diagnostic library
    (round 3's kernel is not in the product library); returns its JSON line."""
    import json
    import subprocess
    import sys
    from conftest import REPO
    r = subprocess.run([sys.executable, os.path.join(REPO, 'tests', 'diag_round3.py'), *args], cwd=REPO,
                       capture_output=True, text=True, timeout=240)
    lines = [x for x in r.stdout.splitlines() if x.startswith('{')]
    assert lines, f'diag_round3.py {args}: rc {r.returncode}\n{r.stderr[-3000:]}'
    out = json.loads(lines[-1])
    assert out.get('library', '').endswith('libmtaz_diag.so'), out
    return r.returncode, out


def test_y_bit_identical_to_round3():
    """Round 4's k_net_y (class tiles with the off-board taps skipped, one stored-units exponent per
    board) computes exactly round 3's k_net_y (variant 3, diagnostic library) on nets whose
    activations stay below 2^14 (both keep xs = 0 there): logits and values bitwise equal, main and
    tail launches alike (tests/diag_round3.py bit_identical)."""
    rc, out = _diag_child('bit_identical')
    assert rc == 0 and out['ok'], out


def test_product_library_rejects_untested_variants():
    """Only parity-tested builds are selectable; the timing-only diagnostic variants (wrong results
    by construction) and round 3's batch-dependent kernel (f16x3 variant 3) are not in the product
    library."""
    from minitchess_alphazero_amd import _lib
    from minitchess_alphazero_amd.engine import Engine
    eng = Engine(n_games=4, sims=2)
    for prec, good, bad in (('f16f8', [0, 1, 8192, 2097152, 25165824, 33554432, 58720256],
                             [16384, 32768, 65536, 131072, 2048, 4194304, 8388608, 16777216]),
                            ('f16x3', [0, 1, 2, 5],
                             [3, 512, 4, 8, 1024, 114688, 16777216, 2048, 8192, 4096, 268435456, 16384, 32768])):
        eng.set_precision(prec)
        for v in good:
            eng.set_net_variant(v)
        for v in bad:
            with pytest.raises(_lib.MtazError):
                eng.set_net_variant(v)


def test_z_mix_epilogue_bit_identical():
    """k_net_z's product epilogue (scaled conversions for the Xl8 / Xh8 copies and the residual
    seed's decode, v_fma_mix for the exact differences) stores the same values as the unfused form
    (variant 2097152) and as the round-2 form (v_fma_mix scalings, variant 33554432): logits and
    values of the builds must be bitwise equal, on an ordinary and on a wide-range net."""
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.network import Network
    from tests_positions import random_fens
    import torch
    for net in (None, _wide_range_net()):
        eng = Engine(n_games=64, sims=8)
        eng.set_precision('f16f8')
        if net is None:
            torch.manual_seed(0)
            net = Network()
        eng.set_weights(net)
        pos = np.stack([pos_from_fen(f) for f in random_fens(257, seed=7)])
        eng.set_net_variant(0)
        l0, v0 = eng.evaluate(pos)
        for var in (2097152, 33554432):
            eng.set_net_variant(var)
            l1, v1 = eng.evaluate(pos)
            assert np.array_equal(l0.view(np.uint32), l1.view(np.uint32)), var
            assert np.array_equal(v0.view(np.uint32), v1.view(np.uint32)), var


def test_z_loop_forms_bit_identical():
    """k_net_z's tap-major K loop with buffer-loaded weights (the product) computes exactly the
    round-2 loop (per-step fragment addresses, 64-bit global weight addresses; variant 25165824):
    logits and values bitwise equal on an ordinary, a wide-range and a tiny-activation net."""
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.network import Network
    from tests_positions import random_fens
    import torch
    torch.manual_seed(0)
    pos = np.stack([pos_from_fen(f) for f in random_fens(259, seed=13)])
    for net in (Network(), _wide_range_net(), _tiny_activation_net()):
        eng = Engine(n_games=64, sims=4)
        eng.set_precision('f16f8')
        eng.set_weights(net)
        eng.set_net_variant(0)
        l0, v0 = eng.evaluate(pos)
        eng.set_net_variant(25165824)
        l1, v1 = eng.evaluate(pos)
        assert np.array_equal(l0.view(np.uint32), l1.view(np.uint32))
        assert np.array_equal(v0.view(np.uint32), v1.view(np.uint32))


def test_y_tap_skip_bit_identical():
    """Skipping the off-board taps (variant 0) changes no bit: the class-tiled kernel with every MFMA
    run (variant 2) gives bitwise the same logits and values, on an ordinary, a wide-range (xs > 0)
    and a tiny-activation net.  1024 boards = one full round of 4 boards per workgroup."""
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.network import Network
    from tests_positions import random_fens
    import torch
    torch.manual_seed(0)
    pos = np.stack([pos_from_fen(f) for f in random_fens(1024, seed=17)])
    for net in (Network(), _wide_range_net(), _tiny_activation_net()):
        eng = Engine(n_games=1024, sims=4)
        eng.set_precision('f16x3')
        eng.set_weights(net)
        eng.set_net_variant(0)
        l0, v0 = eng.evaluate(pos)
        eng.set_net_variant(2)
        l1, v1 = eng.evaluate(pos)
        assert np.array_equal(l0.view(np.uint32), l1.view(np.uint32))
        assert np.array_equal(v0.view(np.uint32), v1.view(np.uint32))
        eng.close()


@pytest.mark.parametrize('precision,net_kind', [('f16f8', 'seed0'), ('f16f8', 'tiny'), ('f16x3', 'seed0'),
                                               ('f16x3', 'tiny'), ('f16x3', 'wide'), ('f16x3', 'stress'),
                                               ('f16x3', 'stress5'), ('f16x3', 'stress6')])
def test_tail_launches_bit_identical(net_kind, precision):
    """The tail-balanced board assignment (k_net_z, k_net_y: the boards beyond the full rounds of
    4 x CUs go to workgroups of 1, 2 or 3 boards) computes every board exactly as 4 boards per
    workgroup do (variant 1): batch sizes whose tails take each of the three tail builds and none.
    k_net_y's tails read off-board sources from zeroed cells of the unused board 3 on the source's
    own bank group and load weights 5 / 3 / 2 k-blocks ahead; variant 5 keeps the first round-4
    tails (off-board cells on the padding squares, 2-way bank conflicts for half the tail's fragment
    reads; weights one k-block ahead): bitwise the same.
    k_net_y keeps one stored-units exponent per board, so this holds for nets whose activations
    pass 2^14 too (wide, stress); k_net_z's is per workgroup (tested below 2^14 only)."""
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from minitchess_alphazero_amd.network import Network
    from tests_positions import random_fens
    import torch
    torch.manual_seed(0)
    net = {'seed0': Network, 'wide': _wide_range_net, 'tiny': _tiny_activation_net,
           'stress': _stress_net, 'stress5': lambda: _stress_net('stress5'),
           'stress6': lambda: _stress_net('stress6')}[net_kind]()
    fens = random_fens(400, seed=29)
    eng = Engine(n_games=4096, sims=4)
    eng.set_precision(precision)
    eng.set_weights(net)
    for n in (1024 + 100, 1024 + 400, 1024 + 700, 2048 + 900, 37):
        pos = np.stack([pos_from_fen(fens[i % len(fens)]) for i in range(n)])
        eng.set_net_variant(0)
        l0, v0 = eng.evaluate(pos)
        # 1: no tail launch; 5 (k_net_y): the tails' off-board cells on the padding squares
        for var in ((1, 5) if precision == 'f16x3' else (1,)):
            eng.set_net_variant(var)
            l1, v1 = eng.evaluate(pos)
            assert np.array_equal(l0.view(np.uint32), l1.view(np.uint32)), (n, var)
            assert np.array_equal(v0.view(np.uint32), v1.view(np.uint32)), (n, var)


def _tiny_activation_net(scale=2.0 ** -20):
    """Random-init net with every BatchNorm gamma and beta x `scale` (stem and both convs of every
    block): folded weights and biases shrink with it, so the trunk's activations sit around
    1e-6, in f16's subnormal range, where the v_fma_mix forms read subnormal halves."""
    import torch
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    with torch.no_grad():
        bns = [net.resbody[0].layers[1]]
        for blk in list(net.resbody)[1:]:
            bns += [blk.convblock1.layers[1], blk.convblock2.layers[1]]
        for bn in bns:
            bn.weight.mul_(scale)
            bn.bias.mul_(scale)
    return net.eval()


@pytest.mark.parametrize('precision,var0,var1', [('f16f8', 0, 2097152), ('f16f8', 0, 33554432), ('f16x3', 0, 3)])
def test_mix_epilogue_bit_identical_tiny_activations(precision, var0, var1):
    """The v_fma_mix epilogues equal their unfused forms bitwise also when the activations are
    f16-subnormal (the mix path's exactness precondition); k_net_y equals round 3's
    kernel (whose epilogue was pinned to its unfused form that way) on the same net, in a child
    process on the diagnostic library (tests/diag_round3.py tiny_mix)."""
    if precision == 'f16x3':
        rc, out = _diag_child('tiny_mix')
        assert rc == 0 and out['ok'], out
        return
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from tests_positions import random_fens
    eng = Engine(n_games=64, sims=4)
    eng.set_precision(precision)
    eng.set_weights(_tiny_activation_net())
    pos = np.stack([pos_from_fen(f) for f in random_fens(97, seed=6)])
    eng.set_net_variant(var0)
    l0, v0 = eng.evaluate(pos)
    eng.set_net_variant(var1)
    l1, v1 = eng.evaluate(pos)
    assert np.array_equal(l0.view(np.uint32), l1.view(np.uint32))
    assert np.array_equal(v0.view(np.uint32), v1.view(np.uint32))


def _wide_range_net(gain=6.0):
    """Random-init net whose residual blocks amplify: both BatchNorm gammas of every block x
    `gain`, so the trunk's activations reach ~7e6 (f16's max is 65504)."""
    import torch
    from minitchess_alphazero_amd.network import Network
    torch.manual_seed(0)
    net = Network()
    with torch.no_grad():
        for blk in list(net.resbody)[1:]:
            blk.convblock1.layers[1].weight.mul_(gain)
            blk.convblock2.layers[1].weight.mul_(gain)
    return net.eval()


@pytest.mark.parametrize('precision,var', [('f16x3', 0), ('f16f8', 0), ('f16f8', 8192)])
def test_dynamic_range_beyond_f16(precision, var):
    """k_net_y and k_net_z keep fp32's range (a power-of-two image scale chosen from a weight bound:
    per board in k_net_y, per workgroup in k_net_z).  With trunk activations ~7e6 the logits match the
    REFERENCE's own fp32 eval forward (exp/policy.py Network on the build container's CPU,
    tests/golden/wide_net.npz by make_golden_r6.py; VERDICT r5 #2: not torch-ROCm) to 1e-5 of each
    row's largest logit (the fp32 error scale at these magnitudes), values (saturated tanh) to 1e-5,
    and the best legal move agrees wherever its margin exceeds that error scale."""
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen, pos_legal
    from oracle.net import state_dict_sha256
    from tests_positions import random_fens
    net = _wide_range_net()
    z = np.load(os.path.join(GOLDEN, 'wide_net.npz'))
    assert state_dict_sha256(net) == str(z['state_dict_sha256'])
    fens = [str(f) for f in z['fens']]
    assert fens == random_fens(129, seed=9)
    eng = Engine(n_games=64, sims=4)
    eng.set_precision(precision)
    eng.set_net_variant(var)
    eng.set_weights(net)
    pos = np.stack([pos_from_fen(f) for f in fens])
    logits, values = eng.evaluate(pos)
    p, v = z['logits'].astype(np.float64), z['values'].astype(np.float64)
    assert np.abs(p).max() > 1e5                          # the trunk really left f16's range
    scale = np.abs(p).max(axis=1, keepdims=True)
    # k_net_z's e4m3 cross terms carry ~2^-15 of each layer's output; through this net's 9
    # amplifying blocks the logits land within 5e-5 of the row scale (k_net_y: 1e-5)
    assert np.max(np.abs(logits - p) / scale) <= (1e-5 if precision == 'f16x3' else 1e-4)
    assert np.max(np.abs(values - v)) <= 1e-5
    for i in range(len(fens)):
        legal = pos_legal(pos[i])
        if len(set(legal)) > 1:
            ref = np.sort(p[i][legal])
            if ref[-1] - ref[-2] > 1e-4 * scale[i, 0]:
                assert legal[int(np.argmax(logits[i][legal]))] == legal[int(np.argmax(p[i][legal]))]


def _stress_net(name='stress'):
    """The round-3 stress checkpoint (tests/golden/stress/): trained in the C5 loop, trunk
    activations in the thousands.  'stress5': stress4 with its trunk in 2^7 larger units (k_net_y's
    exponents 1-4 on every board, values that vary; tests/golden/make_golden_r5.py)."""
    from safetensors.torch import load_file
    from minitchess_alphazero_amd.network import Network
    if name == 'stress6':   # rebuilt from stress4 and sha-checked (tools/make_stress6.py)
        from helpers import stress_network
        return stress_network('stress6')
    net = Network()
    net.load_state_dict(load_file(os.path.join(GOLDEN, name, f'{name}.safetensors')))
    return net.eval()


@pytest.mark.parametrize('net_kind', ['wide', 'stress', 'stress5', 'stress6'])
def test_board_results_independent_of_batch(net_kind):
    """a board's logits and value do not depend on the other boards of its batch or
    workgroup (the reference evaluates every leaf batch-1, exp/agent.py:67-69), also once the
    activations pass 2^14 and the stored-units exponent is nonzero.  The same positions in three
    batch compositions (another order, interleaved with other positions, other batch sizes taking
    other tail builds) give bitwise the same results per position."""
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from tests_positions import random_fens
    net = {'wide': _wide_range_net, 'stress': _stress_net, 'stress5': lambda: _stress_net('stress5'),
           'stress6': lambda: _stress_net('stress6')}[net_kind]()
    fens = random_fens(1300, seed=41)
    pos = np.stack([pos_from_fen(f) for f in fens])
    eng = Engine(n_games=4096, sims=4)
    eng.set_precision('f16x3')
    eng.set_weights(net)
    l0, v0 = eng.evaluate(pos)
    rng = np.random.default_rng(3)
    perm = rng.permutation(len(pos))
    l1, v1 = eng.evaluate(pos[perm])
    assert np.array_equal(l1.view(np.uint32), l0[perm].view(np.uint32))
    assert np.array_equal(v1.view(np.uint32), v0[perm].view(np.uint32))
    other = np.stack([pos_from_fen(f) for f in random_fens(1500, seed=43)])
    mix = np.concatenate([other[:700], pos[:500], other[700:], pos[500:]])
    l2, v2 = eng.evaluate(mix)
    sel = np.r_[700:1200, 2000:2800]
    assert np.array_equal(l2[sel].view(np.uint32), l0.view(np.uint32))
    assert np.array_equal(v2[sel].view(np.uint32), v0.view(np.uint32))
    for n in (37, 333, 1111):
        l3, v3 = eng.evaluate(pos[:n])
        assert np.array_equal(l3.view(np.uint32), l0[:n].view(np.uint32)), n
        assert np.array_equal(v3.view(np.uint32), v0[:n].view(np.uint32)), n
    eng.close()


@pytest.mark.parametrize('net_kind', ['wide', 'stress'])
def test_round3_kernel_was_batch_dependent(net_kind):
    """The case test_board_results_independent_of_batch guards against, shown on round 3's kernel
    (variant 3, one stored-units exponent per workgroup; diagnostic library, child process): on
    these nets the exponent leaves 0, and regrouping the same positions changes some boards' bits
    there, while round 4's per-board exponent (variant 0) changes none.  Records how many positions
    differ."""
    from conftest import REPO
    rc, out = _diag_child('batch_dependent', net_kind)
    msg = (f"{net_kind}: positions whose bits change with the batch order: round 3 {out['info'].get('round3')}, "
           f"round 4 {out['info'].get('round4')}")
    print(msg)
    os.makedirs(os.path.join(REPO, 'gpurun_out'), exist_ok=True)
    with open(os.path.join(REPO, 'gpurun_out', f'batch_dependence_{net_kind}.txt'), 'w') as fh:
        fh.write(msg + '\n')
    assert rc == 0 and out['ok'], out


def test_f16f8_refuses_the_memo_past_its_range():
    """VERDICT r4 #7 / ADVICE r4: k_net_z keeps one stored-units exponent per workgroup, so once a
    layer's bound passes 2^14 a board's result depends on the boards it shares a workgroup with,
    and a leaf memo (mtaz_set_memo >= 1) would hand such a result to other games.  On the wide-range
    net a play with f16f8 and the memo on fails with the range flag; the same play with the memo off
    runs, batch evaluation runs, and k_net_y (one exponent per board) plays with the memo on."""
    from minitchess_alphazero_amd import _lib
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.environment import pos_from_fen
    from tests_positions import random_fens
    net = _wide_range_net()
    eng = Engine(n_games=8, sims=8)
    eng.set_precision('f16f8')
    eng.set_weights(net)
    eng.set_memo(1)
    with pytest.raises(_lib.MtazError, match='f16f8-range-with-memo'):
        eng.play()
    eng.set_memo(0)
    st = eng.play()
    assert st['games'] == 8 and st['plies'] > 0
    eng.set_memo(2)
    pos = np.stack([pos_from_fen(f) for f in random_fens(37, seed=2)])
    logits, values = eng.evaluate(pos)
    assert np.isfinite(logits).all() and np.isfinite(values).all()
    eng.set_precision('f16x3')
    st = eng.play()
    assert st['games'] == 8 and st['plies'] > 0
    eng.close()
