"""CPU restatement of the reference learner (TEST INFRASTRUCTURE, see oracle/__init__.py).

exp/learner.py:23-91 and exp/dataset.py:6-20.  Pinned by tests/golden/learner.{json,npz},
which tests/golden/make_golden_learner.py recorded by running the reference's own
collate_fn / loss / backward in the build container.

  collate_fn          :23-41   dense pi[554] (pi[legal_moves] = pi; a repeated code keeps the
                               value of its last occurrence), tokens (B,2,6,5), clock (B,1),
                               reward (B,1)
  AvgSmoothLoss       :44-59   debiased exponential moving average, beta 0.98
  loss                :84-87   mean((v - r)^2 - sum(pi * log_softmax(p)))
  update              :70-91   fresh AdamW(**optim_params) per call, DataLoader(batch_size,
                               shuffle=True), model.train(), `epochs` passes
  Dataset             dataset.py:6-20   deque(maxlen) of rows, extend on push
"""
from collections import deque

import numpy as np
import torch

from .encoder import process_observation

NUM_ACTIONS = 554


def collate_fn(batch):
    pib, chans, clocks, rewards = [], [], [], []
    for item in batch:
        pi = torch.zeros(NUM_ACTIONS, dtype=torch.float32)
        vals = torch.tensor(item['pi'], dtype=torch.float32)
        for j, code in enumerate(item['legal_moves']):       # later duplicates overwrite earlier ones
            pi[code] = vals[j]
        pib.append(pi)
        t, c = process_observation(item['observation'])
        chans.append(t)
        clocks.append(float(c.item()))
        rewards.append(float(item['reward']))
    return (torch.vstack(pib), torch.cat(chans, dim=0), torch.tensor(clocks, dtype=torch.float32).reshape(-1, 1),
            torch.tensor(rewards, dtype=torch.float32).reshape(-1, 1))


class AvgSmoothLoss:
    def __init__(self, beta=0.98):
        self.beta = beta
        self.count, self.val = 0, 0.0

    def reset(self):
        self.count, self.val = 0, 0.0
        return self

    def accumulate(self, x):
        self.count += 1
        self.val = x + self.beta * (self.val - x)

    @property
    def value(self):
        return self.val / (1 - self.beta ** self.count)


def loss_fn(model, pib, chans, clock, reward):
    p, v = model((chans, clock))
    return ((v - reward) ** 2 - (pib * p.log_softmax(-1)).sum(1)).mean()


class Dataset(torch.utils.data.Dataset):
    def __init__(self, max_length):
        self.rows = deque(maxlen=max_length)

    def push(self, rows):
        self.rows.extend(rows)

    def __len__(self):
        return len(self.rows)

    def __getitem__(self, i):
        return self.rows[i]


def update(model, dataset, batch_size, epochs, optim_params, device='cpu'):
    """One learner update; returns the smoothed loss after each batch."""
    opt = torch.optim.AdamW(model.parameters(), **optim_params)
    loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=True, collate_fn=collate_fn)
    model.train().to(device)
    metric = AvgSmoothLoss().reset()
    trace = []
    for _ in range(epochs):
        for pib, chans, clock, reward in loader:
            loss = loss_fn(model, pib.to(device), chans.to(device), clock.to(device), reward.to(device))
            opt.zero_grad()
            loss.backward()
            metric.accumulate(float(loss.detach().cpu().item()))
            opt.step()
            trace.append(metric.value)
    return np.array(trace)
