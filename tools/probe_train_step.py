#!/usr/bin/env python3
"""Probe: time one batch-32 training step (forward, loss, backward, AdamW) of the Network on
the GPU under conv backend settings (MIOpen find mode via cudnn.benchmark, channels-last),
eager and graph-captured.  Prints one JSON line per setting."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from minitchess_alphazero_amd.network import Network
    dev = torch.device('cuda')
    B = int(os.environ.get('B', 32))
    for bench_mode in (False, True):
        for cl in (False, True):
            torch.backends.cudnn.benchmark = bench_mode
            torch.manual_seed(0)
            net = Network().train().to(dev)
            if cl:
                net = net.to(memory_format=torch.channels_last)
            opt = torch.optim.AdamW(net.parameters(), lr=1e-4)
            tok = torch.randint(0, 7, (B, 2, 6, 5), device=dev)
            clk = torch.rand(B, 1, device=dev)
            pi = torch.softmax(torch.randn(B, 554, device=dev), -1)
            r = torch.randn(B, 1, device=dev)

            def step():
                p, v = net((tok, clk))
                loss = ((v - r) ** 2 - (pi * p.log_softmax(-1)).sum(1)).mean()
                opt.zero_grad(set_to_none=False)
                loss.backward()
                opt.step()
                return loss
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(50):
                step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 50 * 1e3
            print(json.dumps({'benchmark': bench_mode, 'channels_last': cl, 'batch': B, 'eager_ms': ms,
                              'tflops': 3 * 638245892 * B / (ms * 1e-3) / 1e12}), flush=True)


if __name__ == '__main__':
    main()
