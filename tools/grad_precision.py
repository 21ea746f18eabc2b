#!/usr/bin/env python3
"""Learner step gradients on the GPU vs the same step in float64 on the host (tools for the
learner's parity): prints the worst relative L2 gradient error per setting (conv biases that feed
a BatchNorm are skipped: their gradient is mathematically zero)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    import test_gpu_learner as T
    from minitchess_alphazero_amd.learner import ResidentBatches
    from minitchess_alphazero_amd.network import Network
    META = T.META

    def step(net, dev, dtype):
        pib, tok, clk, rew = ResidentBatches(META['batch'], dev).batch(list(range(32)))
        p, v = net((tok, clk.to(dtype)))
        loss = ((v - rew.to(dtype)) ** 2 - (pib.to(dtype) * p.log_softmax(-1)).sum(1)).mean()
        loss.backward()
        return {k: t.grad.double().cpu() for k, t in net.named_parameters()}

    torch.manual_seed(0)
    g64 = step(Network().train().double(), 'cpu', torch.float64)
    skip = {k for k in g64 if k.endswith('layers.0.bias')}
    settings = sys.argv[1].split(',') if len(sys.argv) > 1 and sys.argv[1] != '-v' else ['default', 'nocudnn', 'highest', 'nocudnn_highest']
    for s in settings:
        torch.backends.cudnn.enabled = 'nocudnn' not in s
        if 'highest' in s:
            torch.backends.cuda.matmul.allow_tf32 = False
            torch.backends.cudnn.allow_tf32 = False
            torch.set_float32_matmul_precision('highest')
        torch.manual_seed(0)
        g = step(Network().train().cuda(), 'cuda', torch.float32)
        rel = {k: float((g[k] - g64[k]).norm()) / float(g64[k].norm()) for k in g64 if k not in skip}
        top = sorted(rel.items(), key=lambda x: -x[1])[:4]
        print(s, os.environ.get('TORCH_BLAS_PREFER_HIPBLASLT', '-'), [(k, f'{v:.2e}') for k, v in top], flush=True)
        if '-v' in sys.argv:
            for k in g64:
                if k not in skip:
                    print(f'   {k:45s} {rel[k]:.2e}  |g| {float(g64[k].norm()):.3e}')


if __name__ == '__main__' and '--flips' not in sys.argv:
    main()


def relu_flips():
    """Pre-activation sign flips (BatchNorm outputs: > 0 on one side, <= 0 on the other) between the
    GPU step (MIOpen off) and the float64 host step."""
    import test_gpu_learner as T
    from minitchess_alphazero_amd.learner import ResidentBatches
    from minitchess_alphazero_amd.network import Network
    META = T.META
    outs = {}

    def run(net, dev, dtype, tag):
        hooks = []
        for name, m in net.named_modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                hooks.append(m.register_forward_hook(lambda mod, i, o, name=name: outs.setdefault(tag, {}).__setitem__(name, o.detach().double().cpu())))
        pib, tok, clk, rew = ResidentBatches(META['batch'], dev).batch(list(range(32)))
        net((tok, clk.to(dtype)))
        for h in hooks:
            h.remove()

    torch.manual_seed(0)
    run(Network().train().double(), 'cpu', torch.float64, 'ref')
    torch.backends.cudnn.enabled = False
    torch.manual_seed(0)
    run(Network().train().cuda(), 'cuda', torch.float32, 'gpu')
    tot = 0
    for k, r in outs['ref'].items():
        gg = outs['gpu'][k]
        flips = int(((r > 0) != (gg > 0)).sum())
        tot += flips
        if flips:
            d = (r - gg).abs()[(r > 0) != (gg > 0)]
            print(f'   {k}: {flips} flips, |pre-activation| at flips <= {float(r.abs()[(r > 0) != (gg > 0)].max()):.2e}')
    print('relu sign flips (GPU without MIOpen vs float64):', tot)


if __name__ == '__main__' and '--flips' in sys.argv:
    relu_flips()
