#!/usr/bin/env python3
"""Generate tests/golden/learner.{json,npz} by running the REFERENCE learner code.

Build container only (needs /root/reference, read-only).  Imports the reference's
exp/learner.py (with the stubs of make_golden.py; exp/learner.py:3-6 calls
logging.basicConfig(filename='log'), so the root logger is configured first, which makes
that call a no-op, and the import runs from a temporary directory), then records:

  * collate_fn (exp/learner.py:23-41) on a fixed batch of 32 dataset items taken from the
    reference's own self-play records in trees.json (InfoRecorder rows: observation,
    legal_moves, pi, reward), including rows whose legal list repeats a promotion code;
  * the training forward and loss of exp/learner.py:84-88 for the seed-0 Network in train
    mode: loss, policy logits, values, BatchNorm running statistics after the forward, the
    gradient norm of every parameter and the full gradients of the small tensors;
  * AvgSmoothLoss (exp/learner.py:44-59) on a fixed sequence.
Usage: python tests/golden/make_golden_learner.py
"""
import json
import logging
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from make_golden import import_reference  # noqa: E402

SMALL_GRADS = ['emb.weight', 'pconv.layers.0.weight', 'pconv.layers.0.bias', 'pconv.layers.1.weight',
               'pconv.layers.1.bias', 'plinear.bias', 'vconv.layers.0.weight', 'vconv.layers.1.weight',
               'vlinear.0.bias', 'vlinear.2.weight', 'vlinear.2.bias', 'resbody.0.layers.1.weight',
               'resbody.9.convblock2.layers.1.bias']


def learner_items():
    trees = json.load(open(os.path.join(HERE, 'trees.json')))
    items = [m for g in trees['synthetic'] for m in g['moves']]
    dup = [m for m in items if len(set(m['legal_moves'])) < len(m['legal_moves'])]
    rest = [m for m in items if m not in dup]
    batch = (dup[:6] + rest[::7])[:32]
    return [{'observation': m['observation'], 'legal_moves': m['legal_moves'], 'pi': m['pi'], 'reward': m['reward']}
            for m in batch], len(dup)


def main():
    logging.getLogger().addHandler(logging.NullHandler())   # exp/learner.py:3 basicConfig -> no-op
    renv, rpol, ragent, rcb = import_reference()
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.chdir(tmp)
        try:
            import exp.learner as rlearn
        finally:
            os.chdir(cwd)
    batch, ndup = learner_items()
    assert ndup > 0, 'fixture needs rows with repeated promotion codes'
    pib, channels, clock, reward = rlearn.collate_fn(batch)

    torch.manual_seed(0)
    net = rpol.Network()
    net.train()
    pb, vb = net((channels, clock))
    lp = pb.log_softmax(-1)
    loss = ((vb - reward) ** 2 - (pib * lp).sum(1)).mean()     # exp/learner.py:86-87
    loss.backward()
    named = dict(net.named_parameters())
    grad_norms = {k: float(p.grad.double().norm()) for k, p in named.items()}
    small = {k: named[k].grad.numpy().astype(np.float32) for k in SMALL_GRADS}
    running = {k: v.numpy().astype(np.float32) for k, v in net.state_dict().items()
               if k.endswith('running_mean') or k.endswith('running_var')}

    m = rlearn.AvgSmoothLoss().reset()
    smooth = []
    for x in [3.0, 2.5, 2.75, 1.0, 0.5, 4.0, 2.0]:
        m.accumulate(x)
        smooth.append(m.value)

    arrays = {'pib': pib.numpy(), 'channels': channels.numpy().astype(np.int8), 'clock': clock.numpy(),
              'reward': reward.numpy(), 'logits': pb.detach().numpy(), 'values': vb.detach().numpy()}
    arrays.update({'grad/' + k: v for k, v in small.items()})
    arrays.update({'running/' + k: v for k, v in running.items()})
    np.savez_compressed(os.path.join(HERE, 'learner.npz'), **arrays)
    meta = {'batch': batch, 'rows_with_repeated_codes': min(ndup, 6), 'loss': float(loss.item()),
            'grad_norms': grad_norms, 'small_grads': SMALL_GRADS, 'avg_smooth_inputs': [3.0, 2.5, 2.75, 1.0, 0.5, 4.0, 2.0],
            'avg_smooth_values': smooth, 'seed': 0}
    with open(os.path.join(HERE, 'learner.json'), 'w') as fh:
        json.dump(meta, fh, separators=(',', ':'))
    print('loss', meta['loss'], 'rows', len(batch), 'dup rows', meta['rows_with_repeated_codes'])


if __name__ == '__main__':
    main()
