#!/usr/bin/env python3
"""The STRESS6 checkpoint: stress4 (trained, value head alive) with its residual trunk carried in units
GAIN = 181 times larger, a NON-power-of-two gain.

stress5 (tools/make_stress5.py) scales the trunk by 2^7: every intermediate mantissa of the reference's
forward is stress4's bit for bit, so k_net_y's exponent plumbing was pinned only on stress4's
significands.  Here the same maps use 181 = 1.4140625 x 2^7: the stem BatchNorm's gamma and beta, every
later trunk ConvBlock's conv bias, running mean and beta are multiplied by 181, and the two heads'
ConvBlocks get their conv bias and running mean x 181 and their gamma / 181.  Each scaled tensor is
rounded once in fp32, so the net is a new one: its fp32 trunk values have new significands (not a
power-of-two copy of stress4's), its outputs stay close to stress4's (values alive), and k_net_y's
bounds grow by 181, putting its per-board exponents at 1..5 on every fixture position.

The checkpoint is NOT committed (42 MB): it is a deterministic function of the committed stress4
(element-wise fp32 multiplies and divides by one scalar on the CPU), rebuilt by `stress6_state_dict()`
and pinned by its sha256 in tests/golden/stress6.json, which tests/golden/make_golden_r6.py writes
together with the reference's own outputs and games on it.

Usage: python tools/make_stress6.py            (prints the exponent profile over stress4's fixture)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

GAIN = 181.0
SRC = os.path.join(REPO, 'tests', 'golden', 'stress4', 'stress4.safetensors')


def stress6_state_dict():
    """stress4 -> stress6 (new tensors, fp32, on the CPU)."""
    from safetensors.torch import load_file
    from make_stress5 import rescale
    return rescale(load_file(SRC), 0, gain=GAIN)


def main():
    import numpy as np
    from net_range import fens_profile, summarize
    from oracle.net import Network as RefNet, state_dict_sha256
    sd = stress6_state_dict()
    net = RefNet()
    net.load_state_dict(sd)
    fens = [str(f) for f in np.load(os.path.join(REPO, 'tests', 'golden', 'stress4_net.npz'))['fens']]
    prof = fens_profile(sd, fens)
    per_board_max = prof['xs'].max(0)
    print(json.dumps({'gain': GAIN, 'sha256': state_dict_sha256(net), 'positions': len(fens),
                      'min_over_boards_of_max_exponent': int(per_board_max.min()),
                      **{k: v for k, v in summarize(prof).items() if k != 'per_layer'},
                      'layers_xs_max': [lay['xs_max'] for lay in summarize(prof)['per_layer']]}))


if __name__ == '__main__':
    main()
