#!/usr/bin/env python3
"""Make the STRESS5 checkpoint: stress4 (trained, value head alive) with its residual trunk carried in
2^k times larger units, an exact reparametrisation.

Why not trained directly: the C5 loop with the reference learner's update (exp/learner.py:72-94,
a fresh AdamW per update, batch 32, one pass) was run at the reference's own lr 0.2
(app/learner.py:65-69) and at 0.05, 0.02, 0.01 and 0.005, half the games from endgame starts
(profiles/r05/train_lr/): at every one of them the value head dies (its output is the same
number on every position: value_std 0) within 1-18 updates, and at lr 0.2 the trunk shrinks
(trunk |activation| 123 -> 2 over 40 updates, k_net_y's exponents 0 throughout).  The trunks of
the lr 0.05 / 0.01 runs do drive k_net_y's per-board exponent off 0 at times (up to 5-7), with a
dead value head; stress4 (lr 0.003) keeps a live value head with a trunk below the exponent range.

The reparametrisation: with c = 2^k, scale the stem BatchNorm's gamma and beta by c (the stem's
output becomes c x its old output, ReLU being positively homogeneous), and in every later trunk
ConvBlock the conv bias, the BatchNorm running mean and beta by c (an affine map of c x its old
input then gives c x its old output; the residual adds keep the factor); in the policy and value
heads' ConvBlocks scale the conv bias and running mean by c and gamma by 1/c, which maps c x the
old trunk output to exactly the old head input.  Every factor is a power of two, so in floating
point each operation's result is c x the old one bit for bit (no value reaches the subnormal or
overflow range): the reference's fp32 outputs are stress4's (checked below against stress4's
fixture, and by tests/golden/make_golden_r5.py with the reference's own Network), while the
bounds k_net_y computes per board and layer are c x larger, so its stored-units exponents leave 0
on most layers and positions (tools/net_range.py).

Usage: python tools/make_stress5.py [--k 6] [--out tests/golden/stress5/stress5.safetensors]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def rescale(sd, k, gain=None):
    """stress4's state_dict -> the reparametrised one (new tensors; exact powers of two).  With
    `gain` (tools/make_stress6.py) the factor is that float instead of 2^k: the same maps, no longer
    exact in floating point (each scaled tensor is rounded once), so the result is a new net."""
    from minitchess_alphazero_amd.network import Network
    c = float(2 ** k) if gain is None else float(gain)
    net = Network()
    net.load_state_dict(sd)
    with torch.no_grad():
        stem = net.resbody[0].layers
        stem[1].weight.mul_(c)
        stem[1].bias.mul_(c)
        blocks = []
        for res in list(net.resbody)[1:]:
            blocks += [res.convblock1.layers, res.convblock2.layers]
        for lay in blocks:
            lay[0].bias.mul_(c)
            lay[1].running_mean.mul_(c)
            lay[1].bias.mul_(c)
        for head in (net.pconv.layers, net.vconv.layers):
            head[0].bias.mul_(c)
            head[1].running_mean.mul_(c)
            head[1].weight.div_(c)
    return {n: t.detach().clone().contiguous() for n, t in net.state_dict().items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--k', type=int, default=6)
    ap.add_argument('--src', default=os.path.join(REPO, 'tests', 'golden', 'stress4', 'stress4.safetensors'))
    ap.add_argument('--out', default=os.path.join(REPO, 'tests', 'golden', 'stress5', 'stress5.safetensors'))
    args = ap.parse_args()
    from safetensors.torch import load_file, save_file
    from net_range import fens_profile, summarize
    from oracle.encoder import process_observation
    from oracle.net import Network as RefNet
    src = load_file(args.src)
    sd = rescale(src, args.k)
    # the oracle's restatement of the reference forward (exp/policy.py:71-80, eval, fp32) on stress4's
    # fixture positions: stress5's outputs must be stress4's bit for bit
    z = np.load(os.path.join(REPO, 'tests', 'golden', 'stress4_net.npz'))
    fens = [str(f) for f in z['fens']]
    a, b = RefNet(), RefNet()
    a.load_state_dict(src)
    b.load_state_dict(sd)
    a.eval(), b.eval()
    same = 0
    with torch.no_grad():
        for f in fens:
            pa, va = a(process_observation(f))
            pb, vb = b(process_observation(f))
            same += bool(torch.equal(pa, pb) and torch.equal(va, vb))
    prof = summarize(fens_profile(sd, fens))
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    save_file(sd, args.out)
    print(json.dumps({'k': args.k, 'out': args.out, 'positions': len(fens), 'outputs_bitwise_equal_to_stress4': same,
                      **{kk: v for kk, v in prof.items() if kk != 'per_layer'},
                      'layers_xs_max': [lay['xs_max'] for lay in prof['per_layer']]}))


if __name__ == '__main__':
    main()
