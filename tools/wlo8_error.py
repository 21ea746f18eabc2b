#!/usr/bin/env python3
"""CPU emulation for VERDICT r5 next #5: k_net_y's weight low parts stored as 8-bit significands.

k_net_y multiplies W = Wh + Wl (Wh = f16(W 2^e), Wl = f16(W 2^e - Wh), BN folded, per-layer power of
two e) with X = Xh + Xl as Wh Xh + Wh Xl + Wl Xh.  Storing Wl as an 8-bit signed significand of
Wh's exponent (Wl8 = round(Wl / 2^(E(Wh) - 18)) 2^(E(Wh) - 18), |integer| <= 127) would cut the weight
stream from 4 to 3 bytes per weight (the largest data-movement item, 9.1% of the kernel's time,
DESIGN.md section 3.1).  This script measures what it costs in accuracy before anything is built:
an fp64 forward of the reference network (exp/policy.py:71-80 restated, eval mode) on each net's
fixture positions with the convs' weights replaced by
  split16: Wh + Wl        (the product's weights; the activations' split and the Wl Xl term are
                           common to both forms and left exact here)
  wlo8:    Wh + Wl8       (the proposed form)
against the exact fp64 forward and against the reference's own fp32 outputs (the fixture), for
priors (softmax over the legal list) and values.  The product's measured error on top of that:
k_net_y 2.7e-6 on priors vs fp64 on the stress net.  The verdict's bar:
build only if wlo8 clears 1e-5 with a 3x margin on stress, stress5 and stress6.
Usage: python tools/wlo8_error.py [stress stress5 stress6 ...]   -> one JSON line per net
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests'))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def fold(block):
    conv, bn = block.layers[0], block.layers[1]
    s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    return conv.weight * s[:, None, None, None], bn.bias + (conv.bias - bn.running_mean) * s


def split(w, form):
    """w (float64) -> the weights the form multiplies with (float64)."""
    e = 14 - int(np.floor(np.log2(float(w.abs().max()))))
    ws = w * 2.0 ** e
    wh = ws.to(torch.float16).double()
    wl = (ws - wh).to(torch.float16).double()
    if form == 'wlo8':
        E = torch.floor(torch.log2(wh.abs().clamp_min(2.0 ** -14)))
        q = torch.clamp(torch.round((ws - wh) / 2.0 ** (E - 18)), -127, 127)
        wl = q * 2.0 ** (E - 18)
    return (wh + wl) * 2.0 ** -e


def forward(net, toks, clk, form):
    with torch.no_grad():
        x = net.emb(toks).permute(0, 1, 4, 2, 3).contiguous().view(-1, 8, 6, 5)

        def conv(block, x, relu):
            w, b = fold(block)
            if form != 'exact':
                w = split(w, form)
            y = torch.nn.functional.conv2d(x, w, b, padding=1)
            return torch.relu(y) if relu else y
        x = conv(net.resbody[0], x, True)
        for blk in list(net.resbody)[1:]:
            h = conv(blk.convblock1, x, True)
            x = torch.relu(conv(blk.convblock2, h, False) + x)
        p = net.plinear(torch.cat([net.pconv(x).view(-1, 60), clk], 1))
        v = net.vlinear(torch.cat([net.vconv(x).view(-1, 30), clk], 1))
        return p, v[:, 0]


def main():
    from helpers import stress_network
    from oracle.encoder import process_observation
    from oracle.net import Network
    from minitchess_alphazero_amd.environment import pos_from_fen, pos_legal
    torch.set_num_threads(8)
    for name in sys.argv[1:] or ['stress', 'stress5', 'stress6']:
        net = Network()
        net.load_state_dict(stress_network(name).state_dict())
        net = net.double().eval()
        z = np.load(os.path.join(REPO, 'tests', 'golden', f'{name}_net.npz'))
        fens = [str(f) for f in z['fens']]
        toks = torch.cat([process_observation(f)[0] for f in fens])
        clk = torch.cat([process_observation(f)[1] for f in fens]).double()
        legal = [pos_legal(pos_from_fen(f)) for f in fens]
        out = {'net': name, 'positions': len(fens)}
        p_ex, v_ex = forward(net, toks, clk, 'exact')

        def priors(p):
            return [torch.softmax(p[i][l], 0).numpy() if l else np.zeros(0) for i, l in enumerate(legal)]
        P_ex = priors(p_ex)
        ref_l = torch.from_numpy(z['logits'].astype(np.float64))
        P_ref = [torch.softmax(ref_l[i][l].float(), 0).double().numpy() if l else np.zeros(0) for i, l in enumerate(legal)]
        for form in ('split16', 'wlo8'):
            p, v = forward(net, toks, clk, form)
            P = priors(p)
            out[form] = {
                'priors_vs_fp64': max(float(np.abs(a - b).max()) for a, b in zip(P, P_ex) if len(a)),
                'values_vs_fp64': float((v - v_ex).abs().max()),
                'priors_vs_reference': max(float(np.abs(a - b).max()) for a, b in zip(P, P_ref) if len(a)),
                'values_vs_reference': float(np.abs(v.numpy() - z['values'].astype(np.float64)).max())}
        out['reference_priors_vs_fp64'] = max(float(np.abs(a - b).max()) for a, b in zip(P_ref, P_ex) if len(a))
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
