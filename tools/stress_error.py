#!/usr/bin/env python3
"""Error budget of the network on the stress checkpoint (CPU, build container).

Against an fp64 forward of the stress net (tests/golden/stress/stress.safetensors) on the fixture
positions (tests/golden/stress_net.npz), prints max |error| of the legal priors, values and logits
(relative to each row's largest |logit|) of:
  ref      the reference's own fp32 outputs (the fixture: exp/policy.py Network.forward, torch CPU)
  fp32f    fp32 with the BN folded into the convs (the GPU kernels' form)
  f16x3    Wh*Xh + Wh*Xl + Wl*Xh (k_net_y; per-layer weight scale, image unscaled below 2^14)
  f16x4    f16x3 + Wl*Xl
and the same measures between each of them and the reference (what tests/test_gpu_stress.py
gates).  Usage: python tools/stress_error.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
torch.set_num_threads(8)

from oracle.encoder import process_observation  # noqa: E402
from oracle.environment import MinitChessEpisode  # noqa: E402
from helpers import stress_network  # noqa: E402

Z = np.load(os.path.join(ROOT, 'tests', 'golden', 'stress_net.npz'))
FENS = [str(f) for f in Z['fens']]
REF_L, REF_V = Z['logits'].astype(np.float64), Z['values'].astype(np.float64)
LEGAL = [MinitChessEpisode(f).get_legal_moves() for f in FENS]
net = stress_network()
toks = torch.cat([process_observation(f)[0] for f in FENS])
clk = torch.cat([process_observation(f)[1] for f in FENS])


def fold(block, dt):
    conv, bn = block.layers[0], block.layers[1]
    s = bn.weight.to(dt) / torch.sqrt(bn.running_var.to(dt) + bn.eps)
    w = conv.weight.to(dt) * s[:, None, None, None]
    return w, bn.bias.to(dt) + (conv.bias.to(dt) - bn.running_mean.to(dt)) * s


def split_w(w):   # per-layer power of two putting the largest |w| just below 2^15, then hi/lo f16
    e = 14 - int(np.floor(np.log2(float(w.abs().max()))))
    ws = w * 2.0 ** e
    h = ws.to(torch.float16).double()
    lo = (ws - h).to(torch.float16).double()
    return h / 2.0 ** e, lo / 2.0 ** e


def split_x(x):   # the image: unscaled while activations stay below 2^14
    h = x.to(torch.float16).double()
    return h, (x - h).to(torch.float16).double()


def forward(mode):
    dt = torch.float32 if mode == 'fp32f' else torch.float64
    with torch.no_grad():
        x = net.emb.to(dt)(toks).permute(0, 1, 4, 2, 3).contiguous().view(-1, 8, 6, 5)
        net.emb.float()

        def conv(block, x, relu):
            w, b = fold(block, dt)
            c = lambda a, bb: torch.nn.functional.conv2d(a, bb, None, padding=1)  # noqa: E731
            if mode in ('exact', 'fp32f'):
                y = c(x, w)
            else:
                wh, wl = split_w(w)
                xh, xl = split_x(x)
                y = c(xh, wh) + c(xl, wh) + c(xh, wl)
                if mode == 'f16x4':
                    y = y + c(xl, wl)
            y = y + b[None, :, None, None]
            return torch.relu(y) if relu else y
        x = conv(net.resbody[0], x, True)
        for blk in list(net.resbody)[1:]:
            h = conv(blk.convblock1, x, True)
            x = torch.relu(conv(blk.convblock2, h, False) + x)
        m = net.to(dt)
        p = m.plinear(torch.cat([m.pconv(x).view(-1, 60), clk.to(dt)], 1))
        v = m.vlinear(torch.cat([m.vconv(x).view(-1, 30), clk.to(dt)], 1))
        net.float()
        return p.double().numpy(), v.double().numpy().reshape(-1)


def measure(l, v, l0, v0):
    dl = float(np.max(np.abs(l - l0) / np.maximum(1.0, np.abs(l0).max(axis=1, keepdims=True))))
    dv = float(np.max(np.abs(v - v0)))
    dp = 0.0
    for i, legal in enumerate(LEGAL):
        if legal:
            a = torch.from_numpy(l[i][legal].astype(np.float32)).softmax(0).double().numpy()
            b = torch.from_numpy(l0[i][legal].astype(np.float32)).softmax(0).double().numpy()
            dp = max(dp, float(np.max(np.abs(a - b))))
    return dl, dp, dv


def main():
    l0, v0 = forward('exact')
    rows = {'ref': (REF_L, REF_V)}
    for m in ('fp32f', 'f16x3', 'f16x4'):
        rows[m] = forward(m)
    for name, (l, v) in rows.items():
        e = measure(l, v, l0, v0)
        r = measure(l, v, REF_L, REF_V)
        print(f'{name:6s} vs fp64: logits {e[0]:.2e} priors {e[1]:.2e} values {e[2]:.2e}   '
              f'vs ref: logits {r[0]:.2e} priors {r[1]:.2e} values {r[2]:.2e}')


if __name__ == '__main__':
    main()
