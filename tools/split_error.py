#!/usr/bin/env python3
"""CPU emulation of the network under split-precision schemes (tools for choosing k_net_z).

fp64 forward of the seed-0 reference network (oracle.net) with each 3x3 conv computed as
  exact / w16 (weights rounded to f16) / x16 (activations rounded to f16) / f16x3 (Wh*Xh +
  Wh*Xl + Wl*Xh) / hl8 (Wh*Xl in e4m3) / cross8 (both cross terms in e4m3) / c8res8 (cross8 and
  the residual stored as Xh + e4m3(Xl), = k_net_z), against fp64, next to torch fp32 (the
  reference's own arithmetic).  Prints max |error| of values, priors (softmax over 554) and logits.
"""
import sys, numpy as np, torch
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, 'tests'))
from oracle.net import seed0_network
from oracle.encoder import process_observation
from tests_positions import random_fens
torch.set_num_threads(8)
def _load():
    # argv[1]: a state_dict (safetensors or torch.save) instead of the seed-0 weights
    if len(sys.argv) > 1:
        from oracle.net import Network
        if sys.argv[1].endswith('.safetensors'):
            from safetensors.torch import load_file
            sd = load_file(sys.argv[1])
        else:
            sd = torch.load(sys.argv[1], map_location='cpu', weights_only=True)
        n = Network()
        n.load_state_dict(sd)
        return n.eval()
    return seed0_network()
net = _load().double()
fens = random_fens(300, seed=3)
toks = torch.cat([process_observation(f)[0] for f in fens]); clk = torch.cat([process_observation(f)[1] for f in fens]).double()
def fold(block):
    conv, bn = block.layers[0], block.layers[1]
    s = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    return conv.weight * s[:,None,None,None], bn.bias + (conv.bias - bn.running_mean) * s
def r16(t):  # round to f16 with a per-tensor power-of-two scale keeping values normal
    if float(t.abs().max()) == 0:
        return t
    e = torch.floor(torch.log2(t.abs().max())).item()
    sc = 2.0 ** (14 - e)
    return (t*sc).to(torch.float16).double()/sc
def fwd(mode):
    with torch.no_grad():
        x = net.emb(toks).permute(0,1,4,2,3).contiguous().view(-1,8,6,5)
        def conv(block, x, relu):
            w,b = fold(block)
            if mode in ('w16','both'): w = r16(w)
            if mode in ('x16','both'): x = r16(x)
            y = torch.nn.functional.conv2d(x, w, b, padding=1)
            return torch.relu(y) if relu else y
        x = conv(net.resbody[0], x, True)
        for blk in list(net.resbody)[1:]:
            h = conv(blk.convblock1, x, True)
            x = torch.relu(conv(blk.convblock2, h, False) + x)
        p = net.plinear(torch.cat([net.pconv(x).view(-1,60), clk],1))
        v = net.vlinear(torch.cat([net.vconv(x).view(-1,30), clk],1))
        return p, v
p0,v0 = fwd('exact')
net32 = _load()
with torch.no_grad():
    p32, v32 = net32((toks, clk.float()))
def report(name, p, v):
    pr = torch.softmax(p,1); pr0 = torch.softmax(p0,1)
    print(f'{name:8s} value maxerr {float((v-v0).abs().max()):.3e}  prior maxerr {float((pr-pr0).abs().max()):.3e}  logit maxerr {float((p-p0).abs().max()):.3e}')
report('fp32ref', p32.double(), v32.double())
for m in ('w16','x16','both'):
    report(m, *fwd(m))

def r8(t):
    # e4m3 with a per-tensor power-of-two scale putting the max near 2^8 (max normal 448)
    if float(t.abs().max()) == 0:
        return t
    e = torch.floor(torch.log2(t.abs().max().clamp_min(1e-300))).item()
    sc = 2.0 ** (7 - e)
    return (t*sc).to(torch.float8_e4m3fn).double()/sc
def split16(t):
    if float(t.abs().max()) == 0:
        return t, t
    e = torch.floor(torch.log2(t.abs().max())).item(); sc = 2.0 ** (14 - e)
    h = (t*sc).to(torch.float16).double()
    l = ((t*sc) - h).to(torch.float16).double()
    return h/sc, l/sc
def fwd2(mode):
    with torch.no_grad():
        x = net.emb(toks).permute(0,1,4,2,3).contiguous().view(-1,8,6,5)
        def conv(block, x, relu):
            w,b = fold(block)
            wh, wl = split16(w); xh, xl = split16(x)
            c = lambda a, bb: torch.nn.functional.conv2d(a, bb, None, padding=1)
            if mode == 'f16x3': y = c(xh, wh) + c(xl, wh) + c(xh, wl)
            elif mode == 'cross8': y = c(xh, wh) + c(r8(xl), r8(wh)) + c(r8(xh), r8(wl))
            elif mode == 'hl8': y = c(xh, wh) + c(r8(xl), r8(wh)) + c(xh, wl)
            y = y + b[None,:,None,None]
            return torch.relu(y) if relu else y
        x = conv(net.resbody[0], x, True)
        for blk in list(net.resbody)[1:]:
            h = conv(blk.convblock1, x, True)
            x = torch.relu(conv(blk.convblock2, h, False) + x)
        p = net.plinear(torch.cat([net.pconv(x).view(-1,60), clk],1))
        v = net.vlinear(torch.cat([net.vconv(x).view(-1,30), clk],1))
        return p, v
for m in ('f16x3','hl8','cross8'):
    report(m, *fwd2(m))

def fwd3(res8):
    with torch.no_grad():
        x = net.emb(toks).permute(0,1,4,2,3).contiguous().view(-1,8,6,5)
        def conv(block, x, relu):
            w,b = fold(block)
            wh, wl = split16(w); xh, xl = split16(x)
            c = lambda a, bb: torch.nn.functional.conv2d(a, bb, None, padding=1)
            y = c(xh, wh) + c(r8(xl), r8(wh)) + c(r8(xh), r8(wl)) + b[None,:,None,None]
            return torch.relu(y) if relu else y
        def stored(x):   # the image as stored: Xh + e4m3(Xl)
            xh, xl = split16(x)
            return xh + r8(xl) if res8 else x
        x = conv(net.resbody[0], x, True)
        for blk in list(net.resbody)[1:]:
            h = conv(blk.convblock1, x, True)
            x = torch.relu(conv(blk.convblock2, h, False) + stored(x))
        p = net.plinear(torch.cat([net.pconv(x).view(-1,60), clk],1))
        v = net.vlinear(torch.cat([net.vconv(x).view(-1,30), clk],1))
        return p, v
report('c8exres', *fwd3(False))
report('c8res8', *fwd3(True))

# block-scaled (MX) forms: one power-of-two scale per 32 input channels of a row (activations: per
# board, square and 32-channel group; weights: per output channel, tap and 32-channel group), the
# scale operands v_mfma_scale_f32_16x16x128_f8f6f4 takes per lane
def rblk(t, fmt, channel_dim):
    x = t.movedim(channel_dim, -1)
    shp = x.shape
    g = x.reshape(*shp[:-1], shp[-1] // 32, 32)
    mx = g.abs().amax(-1, keepdim=True)
    top = {'e4m3': 7, 'e2m3': 2}[fmt]          # largest power of two of the format's range
    e = torch.floor(torch.log2(mx.clamp_min(1e-300)))
    sc = torch.where(mx > 0, 2.0 ** (top - e), torch.ones_like(mx))
    y = g * sc
    if fmt == 'e4m3':
        q = y.to(torch.float8_e4m3fn).double()
    else:   # e2m3: 1 sign, 2 exponent (bias 1), 3 mantissa bits: e4m3's grid below 2^-3, scaled by 2^6
        q = (y * 2.0 ** -6).to(torch.float8_e4m3fn).double() * 2.0 ** 6
    return (q / sc).reshape(shp).movedim(-1, channel_dim)
def fwd4(fmt, res):
    with torch.no_grad():
        x = net.emb(toks).permute(0,1,4,2,3).contiguous().view(-1,8,6,5)
        def conv(block, x, relu, first=False):
            w,b = fold(block)
            wh, wl = split16(w); xh, xl = split16(x)
            c = lambda a, bb: torch.nn.functional.conv2d(a, bb, None, padding=1)
            if first:
                y = c(xh, wh) + c(xl, wh) + c(xh, wl)
            else:
                y = c(xh, wh) + c(rblk(xl, fmt, 1), rblk(wh, fmt, 1)) + c(rblk(xh, fmt, 1), rblk(wl, fmt, 1))
            y = y + b[None,:,None,None]
            return torch.relu(y) if relu else y
        def stored(x):
            xh, xl = split16(x)
            return xh + rblk(xl, fmt, 1) if res else x
        x = conv(net.resbody[0], x, True, first=True)
        for blk in list(net.resbody)[1:]:
            h = conv(blk.convblock1, x, True)
            x = torch.relu(conv(blk.convblock2, h, False) + stored(x))
        p = net.plinear(torch.cat([net.pconv(x).view(-1,60), clk],1))
        v = net.vlinear(torch.cat([net.vconv(x).view(-1,30), clk],1))
        return p, v
report('mx8', *fwd4('e4m3', False))
report('mx8res', *fwd4('e4m3', True))
report('mx6res', *fwd4('e2m3', True))
def fwd5(fmt_lo, which):
    # one cross term in a block-scaled 8/6-bit format, the other in f16; residual at full precision
    with torch.no_grad():
        x = net.emb(toks).permute(0,1,4,2,3).contiguous().view(-1,8,6,5)
        def conv(block, x, relu, first=False):
            w,b = fold(block)
            wh, wl = split16(w); xh, xl = split16(x)
            c = lambda a, bb: torch.nn.functional.conv2d(a, bb, None, padding=1)
            if first:
                y = c(xh, wh) + c(xl, wh) + c(xh, wl)
            elif which == 'wl':   # Wl*Xh quantized, Wh*Xl in f16
                y = c(xh, wh) + c(xl, wh) + c(rblk(xh, fmt_lo, 1), rblk(wl, fmt_lo, 1))
            else:                 # Wh*Xl quantized, Wl*Xh in f16
                y = c(xh, wh) + c(rblk(xl, fmt_lo, 1), rblk(wh, fmt_lo, 1)) + c(xh, wl)
            y = y + b[None,:,None,None]
            return torch.relu(y) if relu else y
        x = conv(net.resbody[0], x, True, first=True)
        for blk in list(net.resbody)[1:]:
            h = conv(blk.convblock1, x, True)
            x = torch.relu(conv(blk.convblock2, h, False) + x)
        p = net.plinear(torch.cat([net.pconv(x).view(-1,60), clk],1))
        v = net.vlinear(torch.cat([net.vconv(x).view(-1,30), clk],1))
        return p, v
report('mxWl8', *fwd5('e4m3', 'wl'))
report('mxXl8', *fwd5('e4m3', 'xl'))
