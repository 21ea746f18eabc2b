#!/usr/bin/env python3
"""k_net_y's per-board stored-units exponents, emulated on the CPU (measurement tool, not product).

k_net_y (csrc/mtaz_net16.hip, epilogue) keeps board b's activation image as x * 2^-xs[b] in f16
hi/lo.  Before a layer's outputs are stored it picks xo[b] from a rigorous bound on board b's
outputs (mtaz_net16.hip:657-671, the stem at :487-491):

    bound = (G_L * max_b(input) + B_L [+ max_b(block input) for conv B]) * (1 + 2^-10)
    xo    = ilogb(bound) - 14   if bound >= 2^14, else 0

G_L = max over output channels of the L1 norm of the BN-folded weights, B_L = max |folded bias|
(mtaz_host.cpp:1175-1201, NetWeights::yrange); the stem's input bound is max |embedding|.
max_b(.) is the measured maximum of the previous image over board b's squares.

This script recomputes those exponents from a float64 forward of the same network
(exp/policy.py:71-80 in eval mode), so that a checkpoint can be selected, and its fixture
documented, by whether it drives the kernel's nonzero-exponent path.
The float64 maxima differ from the kernel's stored f16 hi/lo maxima by ~2^-22 relative; a layer
whose bound sits that close to a power of two could differ by one, which the report shows as
`bound_log2` next to each exponent.

Usage: python tools/net_range.py CHECKPOINT.safetensors [FIXTURE.npz]
"""
import json
import math
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402

BN_EPS = 1e-5
MARGIN = 1.0009765625


def _gb(block):
    """(G, B) of a _ConvBN / ConvBlock: max_co L1(folded weight row), max |folded bias|."""
    conv, bn = block.layers[0], block.layers[1]
    w = conv.weight.detach().double()
    sc = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + BN_EPS)
    sh = (conv.bias.detach().double() - bn.running_mean.detach().double()) * sc + bn.bias.detach().double()
    g = (w.abs().flatten(1).sum(1) * sc.abs()).max().item()
    return g, sh.abs().max().item()


def _xo(bound):
    """The kernel's exponent for a bound (float64 array over boards)."""
    out = np.zeros(bound.shape, dtype=np.int64)
    big = bound >= 16384.0
    out[big] = np.floor(np.log2(bound[big])).astype(np.int64) - 14
    return out


def xs_profile(state_dict, tokens, clock, device='cpu'):
    """Per layer (stem, then the 18 residual convs in k_net_y's order L = 0..17): the exponent xo
    each board gets and the bound it came from.  tokens (B,2,6,5) int64, clock (B,1).
    device: where the float64 forward runs.
    Returns {'xs': int64 [19, B], 'bound': float64 [19, B], 'trunk_max': float}."""
    from minitchess_alphazero_amd.network import Network
    net = Network()
    net.load_state_dict(state_dict)
    net = net.double().eval().to(device)
    tokens = tokens.to(device)
    xs, bounds = [], []
    with torch.no_grad():
        emb = net.emb.weight.detach().double()
        x = net.emb(tokens).permute(0, 1, 4, 2, 3).reshape(-1, 8, 6, 5)
        mx = np.full(x.shape[0], emb.abs().max().item())
        stem = net.resbody[0]
        g, b = _gb(stem)
        bnd = (g * mx + b) * MARGIN
        xs.append(_xo(bnd)), bounds.append(bnd)
        x = stem(x)
        mx = x.flatten(1).abs().max(1).values.cpu().numpy()
        trunk = float(mx.max())
        for res in list(net.resbody)[1:]:
            blk = mx
            g, b = _gb(res.convblock1)
            bnd = (g * mx + b) * MARGIN
            xs.append(_xo(bnd)), bounds.append(bnd)
            a = res.convblock1(x)
            mx = a.flatten(1).abs().max(1).values.cpu().numpy()
            trunk = max(trunk, float(mx.max()))
            g, b = _gb(res.convblock2)
            bnd = (g * mx + b + blk) * MARGIN
            xs.append(_xo(bnd)), bounds.append(bnd)
            x = res.nonl(res.convblock2(a) + x)
            mx = x.flatten(1).abs().max(1).values.cpu().numpy()
            trunk = max(trunk, float(mx.max()))
    return {'xs': np.stack(xs), 'bound': np.stack(bounds), 'trunk_max': trunk}


def summarize(prof):
    """JSON-able per-layer summary: max exponent over boards, boards with a nonzero exponent,
    log2 of the largest bound."""
    xs, bnd = prof['xs'], prof['bound']
    names = ['stem'] + [f'conv{L}' for L in range(xs.shape[0] - 1)]
    layers = [{'layer': n, 'xs_max': int(xs[i].max()), 'boards_xs_pos': int((xs[i] > 0).sum()),
               'bound_log2_max': round(math.log2(max(float(bnd[i].max()), 1e-300)), 3)}
              for i, n in enumerate(names)]
    return {'boards': int(xs.shape[1]), 'xs_max': int(xs.max()), 'boards_any_xs_pos': int((xs > 0).any(0).sum()),
            'layers_xs_pos': int((xs > 0).any(1).sum()), 'trunk_max': prof['trunk_max'], 'per_layer': layers}


def fens_profile(state_dict, fens):
    from minitchess_alphazero_amd.environment import pos_encode, pos_from_fen
    toks, clks = [], []
    for f in fens:
        t, c = pos_encode(pos_from_fen(str(f)))
        toks.append(np.asarray(t).reshape(2, 6, 5))
        clks.append(c)
    tokens = torch.from_numpy(np.stack(toks).astype(np.int64))
    clock = torch.tensor(clks, dtype=torch.float64).reshape(-1, 1)
    return xs_profile(state_dict, tokens, clock)


def main():
    from safetensors.torch import load_file
    sd = load_file(sys.argv[1])
    if len(sys.argv) > 2:
        fens = np.load(sys.argv[2])['fens']
    else:
        from minitchess_alphazero_amd.environment import STARTING_FEN
        fens = [STARTING_FEN]
    print(json.dumps(summarize(fens_profile(sd, fens))))


if __name__ == '__main__':
    main()
