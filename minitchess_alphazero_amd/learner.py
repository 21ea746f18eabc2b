"""Learner: drop-in for exp/learner.py, exp/dataset.py and LearnPuppet (app/base.py:137-205).

SURVEY 8f rank 1.  Training is the reference's update on PyTorch-ROCm autograd (SURVEY 8f:
"PyTorch-ROCm autograd is acceptable here"): the same loss (exp/learner.py:86-87), a fresh
AdamW(**optim_params) per update (:71-72), a shuffled pass over the dataset in batches of
`batch_size` (:73-76), `epochs` passes, train-mode BatchNorm.

What differs is how batches are built.  The reference collates every batch on the host from
FEN strings (:23-41).  Here the whole dataset is encoded once per update: the positions
are parsed by libmtaz, the tokens and clocks come from the HIP batch encoder
(mtaz_encode_batch, the kernel that feeds self-play), and the dense pi targets are built
with numpy.  These tensors stay resident on the GPU.  Each batch is an index gather in
the order the reference's DataLoader would draw: the same RandomSampler on torch's global
RNG, so a seeded update visits the rows in the same order.  `collate_fn` is kept with the
reference's signature and output for callers that use a DataLoader themselves.

MQTT / HTTP transport (app/learner.py) is out of scope (wire formats are rank 3);
LearnPuppet keeps the state machine, the dataset and the versioned weights.
"""
import copy
import ctypes
import logging
from collections import deque
from datetime import datetime

import numpy as np
import torch

from . import _lib
from .environment import pos_encode, pos_from_fen
from .network import NUM_ACTIONS, Network
from .puppet import MasterOfPuppetsStatus

log = logging.getLogger(__name__)


# ---- dataset (exp/dataset.py:6-20) --------------------------------------------------------------
class SimpleAlphaZeroDataset(torch.utils.data.Dataset):
    """Replay memory of self-play rows {'observation', 'legal_moves', 'pi', 'reward'}: a
    deque of max_length rows; push() extends it (oldest rows fall out)."""

    def __init__(self, max_length):
        self._memory = deque(maxlen=max_length)

    def get_memory(self):
        return list(self._memory)

    def push(self, data):
        self._memory.extend(data)

    def __len__(self):
        return len(self._memory)

    def __getitem__(self, i):
        return self._memory[i]


# ---- batch construction ---------------------------------------------------------------------------
def dense_pi(rows):
    """pi targets [n, 554] float32: pi[legal_moves] = pi (float32), a code that repeats in
    the legal list (promotions) keeps its last value (exp/learner.py:29-30)."""
    out = np.zeros((len(rows), NUM_ACTIONS), np.float32)
    for i, r in enumerate(rows):
        out[i, np.asarray(r['legal_moves'], np.int64)] = np.asarray(r['pi'], np.float64).astype(np.float32)
    return out


def collate_fn(batch):
    """exp/learner.py:23-41: (pi [B,554] f32, tokens [B,2,6,5] i64, clock [B,1] f32, reward [B,1] f32)."""
    toks, clocks = [], []
    for r in batch:
        t, c = pos_encode(pos_from_fen(r['observation']))
        toks.append(t)
        clocks.append(c)
    return (torch.from_numpy(dense_pi(batch)), torch.from_numpy(np.stack(toks)).reshape(-1, 2, 6, 5),
            torch.tensor(np.asarray(clocks, np.float32)).reshape(-1, 1),
            torch.tensor(np.asarray([float(r['reward']) for r in batch], np.float32)).reshape(-1, 1))


def encode_positions(pos, device):
    """Packed positions [n, 5] u32 -> tokens [n,2,6,5] int64 and clock [n,1] f32 on `device`,
    by the HIP batch encoder (exp/policy.py:96-105 for the whole batch in one launch)."""
    dev = torch.device(device)
    d_pos = torch.from_numpy(np.ascontiguousarray(pos, np.uint32).view(np.int32)).to(dev)
    n = d_pos.shape[0]
    tok = torch.empty((n, 60), dtype=torch.uint8, device=dev)
    clk = torch.empty((n,), dtype=torch.float32, device=dev)
    torch.cuda.synchronize(dev)
    _lib.check(_lib.lib().mtaz_encode_batch(dev.index or 0, d_pos.data_ptr(), n, tok.data_ptr(), clk.data_ptr(), None))
    torch.cuda.synchronize(dev)
    return tok.long().reshape(n, 2, 6, 5), clk.reshape(n, 1)


class ResidentBatches:
    """A dataset encoded once and kept on the device; batches are index gathers."""

    def __init__(self, rows, device):
        self.device = torch.device(device)
        if isinstance(rows, EpisodeRecords):
            pos, pi, reward = rows.pos, rows.pi_dense(), rows.reward
        else:
            pos = np.stack([pos_from_fen(r['observation']) for r in rows]) if rows else np.zeros((0, 5), np.uint32)
            pi = dense_pi(rows)
            reward = np.asarray([float(r['reward']) for r in rows], np.float32)
        if self.device.type == 'cuda':
            self.tokens, self.clock = encode_positions(pos, self.device)
        else:   # host encoder (CPU tests; the product learner runs on the GPU)
            enc = [pos_encode(p) for p in pos]
            self.tokens = torch.from_numpy(np.stack([t for t, _ in enc])).reshape(-1, 2, 6, 5)
            self.clock = torch.tensor(np.asarray([c for _, c in enc], np.float32)).reshape(-1, 1)
        self.pi = torch.from_numpy(pi).to(self.device)
        self.reward = torch.from_numpy(np.ascontiguousarray(reward, np.float32)).reshape(-1, 1).to(self.device)

    def __len__(self):
        return self.pi.shape[0]

    def gather(self, i):
        """Rows at the device index tensor i (capturable in a HIP graph)."""
        return self.pi[i], self.tokens[i], self.clock[i], self.reward[i]

    def batch(self, idx):
        return self.gather(torch.as_tensor(idx, dtype=torch.long, device=self.device))


class ReplayBuffer:
    """SimpleAlphaZeroDataset (exp/dataset.py:6-20) resident in HBM.

    A ring of encoded rows: tokens [cap, 60] u8, clock [cap] f32, dense pi [cap, 554] f32,
    reward [cap] f32 (2,284 B per row, so the reference's max_length of 1e6 rows is 2.3 GB).
    push_records() uploads the packed records (EpisodeRecords: 20 B of position + 6 B per legal
    entry per row) and one HIP launch (mtaz_replay_put) encodes them into the slots after the
    newest row; past max_length the oldest rows are overwritten, the deque(maxlen) semantics.
    Row i (0 = oldest, as deque indexing) lives in slot (head + i) % cap.  Batches are index
    gathers on the device, so an update never re-encodes or re-uploads its dataset.  The
    ring grows geometrically up to max_length (no up-front 2.3 GB allocation)."""

    ROW_BYTES = 60 + 4 + 4 * NUM_ACTIONS + 4

    def __init__(self, max_length, device, initial=1 << 16):
        self.max_length = int(max_length)
        self.device = torch.device(device)
        if self.device.type != 'cuda':
            raise RuntimeError('ReplayBuffer lives in GPU memory (HIP ingest kernel); use '
                               'SimpleAlphaZeroDataset / ResidentBatches on the host')
        self.cap = 0
        self.head = 0
        self.size = 0
        self._alloc(min(self.max_length, initial))

    def _alloc(self, cap):
        dev = self.device
        new = (torch.zeros((cap, 60), dtype=torch.uint8, device=dev), torch.zeros(cap, dtype=torch.float32, device=dev),
               torch.zeros((cap, NUM_ACTIONS), dtype=torch.float32, device=dev),
               torch.zeros(cap, dtype=torch.float32, device=dev))
        if self.size:
            order = (torch.arange(self.size, device=dev) + self.head) % self.cap
            for dst, src in zip(new, (self._tokens, self._clock, self._pi, self._reward)):
                dst[:self.size] = src[order]
        self._tokens, self._clock, self._pi, self._reward = new
        self.cap, self.head = cap, 0

    def __len__(self):
        return self.size

    def clear(self):
        """A fresh, empty dataset (LearnPuppet._init_dataset) keeping the allocation."""
        self.head = self.size = 0

    def push_records(self, rec):
        """Append packed rows (EpisodeRecords, host arrays) in order."""
        dev = self.device
        n = len(rec)
        if n == 0:
            return
        k = torch.from_numpy(rec.k.astype(np.int32)).to(dev)
        self.push_device(torch.from_numpy(rec.pos.view(np.int32)).to(dev), k,
                         torch.from_numpy(rec.codes.view(np.int16)).to(dev),
                         torch.from_numpy(rec.visits.view(np.int32)).to(dev),
                         torch.from_numpy(rec.reward).to(dev))

    def push_device(self, pos, k, codes, visits, reward):
        """Append rows already on the device: pos [n,5] i32 (u32 bits), k [n] i32, codes [E]
        i16 (u16 bits), visits [E] i32 (u32 bits), reward [n] f32."""
        n = int(k.shape[0])
        if n == 0:
            return
        e0 = torch.cumsum(k.to(torch.int64), 0) - k.to(torch.int64)
        if n > self.max_length:                        # only the newest max_length rows survive
            s = n - self.max_length
            pos, k, e0, reward, n = pos[s:], k[s:], e0[s:], reward[s:], self.max_length
        if self.size + n > self.cap and self.cap < self.max_length:
            self._alloc(min(self.max_length, max(2 * self.cap, self.size + n)))
        tail = (self.head + self.size) % self.cap
        args = [c.contiguous() for c in (pos, k, e0, codes, visits, reward)]
        _lib.check(_lib.lib().mtaz_replay_put(
            self.device.index or 0, n, *[a.data_ptr() for a in args], self.cap, tail,
            self._tokens.data_ptr(), self._clock.data_ptr(), self._pi.data_ptr(), self._reward.data_ptr(),
            ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)))
        over = max(0, self.size + n - self.cap)
        self.size = min(self.cap, self.size + n)
        self.head = (self.head + over) % self.cap

    def push_rows(self, rows):
        """Append dict rows (InfoRecorder format, the MQTT learner's push_data) in order: tokens and
        clock by the HIP encoder, pi by dense_pi (exp/learner.py:29-30), written to the slots after
        the newest row like push_records, so both push paths share one ring in arrival order."""
        n = len(rows)
        if n == 0:
            return
        if n > self.max_length:
            rows, n = rows[n - self.max_length:], self.max_length
        dev = self.device
        pos = np.stack([pos_from_fen(r['observation']) for r in rows])
        tok, clk = encode_positions(pos, dev)
        pi = torch.from_numpy(dense_pi(rows)).to(dev)
        rew = torch.tensor([float(r['reward']) for r in rows], dtype=torch.float32, device=dev)
        if self.size + n > self.cap and self.cap < self.max_length:
            self._alloc(min(self.max_length, max(2 * self.cap, self.size + n)))
        slots = (torch.arange(n, device=dev) + self.head + self.size) % self.cap
        self._tokens[slots] = tok.reshape(n, 60).to(torch.uint8)
        self._clock[slots] = clk.reshape(n)
        self._pi[slots] = pi
        self._reward[slots] = rew
        over = max(0, self.size + n - self.cap)
        self.size = min(self.cap, self.size + n)
        self.head = (self.head + over) % self.cap

    def gather(self, i):
        """Rows i (device index tensor, 0 = oldest) -> (pi, tokens [.,2,6,5] i64, clock [.,1],
        reward [.,1]); capturable in a HIP graph (head is fixed for an update)."""
        j = (i + self.head) % self.cap if self.head else i
        return (self._pi[j], self._tokens[j].long().reshape(-1, 2, 6, 5), self._clock[j].reshape(-1, 1),
                self._reward[j].reshape(-1, 1))

    def batch(self, idx):
        return self.gather(torch.as_tensor(idx, dtype=torch.long, device=self.device))


class EpisodeRecords:
    """Self-play rows as packed arrays in Engine.records() layout: pos [N,5] u32, k [N] legal
    list lengths, codes / visits concatenated over rows, reward [N].  pi = visits / sum(visits)
    per row (float64, as Engine.episodes / exp/policy.py:120 compute it).  The loop moves these
    arrays between ranks instead of FEN-keyed dicts."""

    def __init__(self, pos, k, codes, visits, reward):
        self.pos = np.ascontiguousarray(pos, np.uint32).reshape(-1, 5)
        self.k = np.ascontiguousarray(k, np.int32)
        self.codes = np.ascontiguousarray(codes, np.uint16)
        self.visits = np.ascontiguousarray(visits, np.uint32)
        self.reward = np.ascontiguousarray(reward, np.float32)

    @classmethod
    def from_engine(cls, rec):
        return cls(rec['pos'], rec['k'], rec['codes'], rec['visits'], rec['reward'])

    @classmethod
    def concat(cls, parts):
        parts = [p for p in parts if len(p)]
        if not parts:
            return cls(np.zeros((0, 5), np.uint32), [], [], [], [])
        return cls(np.concatenate([p.pos for p in parts]), np.concatenate([p.k for p in parts]),
                   np.concatenate([p.codes for p in parts]), np.concatenate([p.visits for p in parts]),
                   np.concatenate([p.reward for p in parts]))

    def __len__(self):
        return int(self.k.shape[0])

    def slice(self, a, b):
        """Rows [a, b)."""
        e0, e1 = int(self.k[:a].sum()), int(self.k[:b].sum())
        return EpisodeRecords(self.pos[a:b], self.k[a:b], self.codes[e0:e1], self.visits[e0:e1], self.reward[a:b])

    def tail(self, n):
        """The last n rows (deque(maxlen) semantics of exp/dataset.py:8)."""
        if n >= len(self):
            return self
        return self.slice(len(self) - n, len(self))

    def pi_dense(self):
        """[N, 554] float32 targets, the same values and duplicate rule as dense_pi(rows)."""
        n = len(self)
        out = np.zeros((n, NUM_ACTIONS), np.float32)
        if n == 0:
            return out
        row = np.repeat(np.arange(n), self.k)
        starts = np.concatenate([[0], np.cumsum(self.k)[:-1]])
        sums = np.add.reduceat(self.visits.astype(np.float64), starts)
        vals = (self.visits.astype(np.float64) / sums[row]).astype(np.float32)
        out[row, self.codes.astype(np.int64)] = vals   # repeated (row, code): the last occurrence is kept
        return out

    def to_rows(self):
        """dict rows (exp/callbacks.py:40-47 InfoRecorder format, without 'action')."""
        from .environment import pos_to_fen
        rows, e = [], 0
        for i in range(len(self)):
            k = int(self.k[i])
            N = self.visits[e:e + k].astype(np.float64)
            rows.append({'observation': pos_to_fen(self.pos[i]), 'legal_moves': [int(c) for c in self.codes[e:e + k]],
                         'pi': (N / N.sum()).tolist(), 'reward': float(self.reward[i])})
            e += k
        return rows


def sampler_order(n):
    """The row order a DataLoader(shuffle=True) draws for an n-row dataset, consuming torch's
    global generator as the reference's DataLoader does: the iterator first draws its worker
    base seed, then RandomSampler draws the seed of its own generator for randperm
    (tests/test_learner_cpu.py checks the order against a real DataLoader)."""
    torch.empty((), dtype=torch.int64).random_()
    return list(iter(torch.utils.data.RandomSampler(range(n))))


# ---- loss / metric (exp/learner.py:44-59, :84-88) --------------------------------------------------
class AvgSmoothLoss:
    def __init__(self, beta=0.98):
        self.beta = beta
        self.count, self.val = 0, 0.0

    def reset(self):
        self.count, self.val = 0, 0.0
        return self

    def accumulate(self, new_val):
        self.count += 1
        self.val = new_val + self.beta * (self.val - new_val)

    @property
    def value(self):
        return self.val / (1 - self.beta ** self.count)


def alphazero_loss(model, pib, tokens, clock, reward):
    """mean((v - r)^2 - sum(pi * log_softmax(p)))  (exp/learner.py:86-87)"""
    p, v = model((tokens, clock))
    return ((v - reward) ** 2 - (pib * p.log_softmax(-1)).sum(1)).mean()


# ---- learner (exp/learner.py:62-91) ------------------------------------------------------------------
class SimpleAlphaZeroLearner:
    def __init__(self, env, num_simulations, network, batch_size, epochs, optim_params, device=None):
        self._env = env
        self._num_simulations = num_simulations
        self._network = network
        self._batch_size = batch_size
        self._epochs = epochs
        self._optim_params = dict(optim_params)
        self._device = torch.device(device) if device is not None else \
            torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() else torch.device('cpu')
        self.last_losses = []

    def update(self, dataset):
        """One learner update over `dataset` (rows, SimpleAlphaZeroDataset or EpisodeRecords).
        Returns the smoothed loss; per-batch values in self.last_losses.

        On a GPU the full-size batch step (gather, forward, loss, backward, AdamW) is captured
        once per update in a HIP graph and replayed per batch: at the reference's batch of 32
        the step is launch-bound.  The graph is captured after warm-up steps, and the weights,
        BatchNorm buffers and optimizer state are then restored to their pre-warm-up values,
        so the replayed steps are the reference's steps; AdamW runs with capturable=True (its
        step count on the device).  A partial last batch runs eagerly."""
        model = self._network.train().to(self._device)
        if isinstance(dataset, ReplayBuffer):
            data = dataset
        else:
            rows = dataset if isinstance(dataset, EpisodeRecords) else \
                dataset.get_memory() if hasattr(dataset, 'get_memory') else list(dataset)
            data = ResidentBatches(rows, self._device)
        use_graph = self.graphs and self._device.type == 'cuda' and len(data) >= self._batch_size
        optimizer = torch.optim.AdamW(model.parameters(), **self._optim_params,
                                      **({'capturable': True} if use_graph else {}))
        step = self._graph_step(model, optimizer, data) if use_graph else None
        metric = AvgSmoothLoss().reset()
        losses = []
        for epoch in range(self._epochs):
            order = sampler_order(len(data))
            pending = []
            for s in range(0, len(order), self._batch_size):
                idx = order[s:s + self._batch_size]
                if step is not None and len(idx) == self._batch_size:
                    pending.append(step(idx))
                    continue
                pib, tok, clk, rew = data.batch(idx)
                loss = alphazero_loss(model, pib, tok, clk, rew)
                optimizer.zero_grad()
                loss.backward()
                pending.append(loss.detach().clone())
                optimizer.step()
            for lt in torch.stack(pending).tolist() if pending else []:   # one sync per epoch
                metric.accumulate(lt)
                losses.append(lt)
            log.info('Epoch %d: %.2f', epoch, metric.value if metric.count else float('nan'))
        self.last_losses = losses
        return metric.value if metric.count else float('nan')

    graphs = True

    def _graph_step(self, model, optimizer, data):
        """Capture one full-batch training step; returns step(idx) -> loss tensor (a copy)."""
        dev = self._device
        static_idx = torch.zeros(self._batch_size, dtype=torch.long, device=dev)
        static_loss = torch.zeros((), dtype=torch.float32, device=dev)
        saved = {k: v.detach().clone() for k, v in model.state_dict().items()}

        def body():
            pib, tok, clk, rew = data.gather(static_idx)
            loss = alphazero_loss(model, pib, tok, clk, rew)
            optimizer.zero_grad(set_to_none=False)
            loss.backward()
            optimizer.step()
            static_loss.copy_(loss.detach())

        static_idx.copy_(torch.arange(self._batch_size, device=dev) % len(data))
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(3):
                body()
        torch.cuda.current_stream(dev).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            body()
        # undo the warm-up and capture steps: weights, BN buffers, AdamW moments and step count
        with torch.no_grad():
            for k, v in model.state_dict().items():
                v.copy_(saved[k])
            for st in optimizer.state.values():
                for t in st.values():
                    if torch.is_tensor(t):
                        t.zero_()
            for p in model.parameters():
                if p.grad is not None:
                    p.grad.zero_()

        def step(idx):
            static_idx.copy_(torch.as_tensor(idx, dtype=torch.long).to(dev, non_blocking=True))
            graph.replay()
            return static_loss.clone()
        return step


# ---- LearnPuppet (app/base.py:137-205, transport excluded) --------------------------------------------
class LearnPuppet:
    def __init__(self, userid, batch_size, epochs, optim_params, device=None, max_length=1_000_000):
        self._userid = userid
        self._max_length = max_length
        self._replay = None
        self._dataset = None
        self._init_dataset()
        self._network = Network()
        self._learner = SimpleAlphaZeroLearner(None, 36, self._network, batch_size, epochs, optim_params, device)
        self._episode_counter = 0
        self._weights_version = None
        self._weights = None
        self.weights = self._network.state_dict()
        self._status = MasterOfPuppetsStatus.SIMULATE

    def _init_dataset(self):
        self._dataset = SimpleAlphaZeroDataset(max_length=self._max_length)
        self._records = EpisodeRecords.concat([])
        # host learner only: ('rows', list of dicts) / ('records', EpisodeRecords) in push order, for
        # an update over both push paths (a GPU learner puts both into the HBM ring in push order)
        self._arrivals = []
        if getattr(self, '_replay', None) is not None:
            self._replay.clear()

    @property
    def episode_counter(self):
        return self._episode_counter

    @property
    def weights_version(self):
        return self._weights_version

    @property
    def weights(self):
        return self._weights

    @weights.setter
    def weights(self, value):
        self._weights = {k: v.detach().cpu().clone() for k, v in value.items()}
        self._weights_version = datetime.now().strftime('%Y%m%d%H%M%S')

    @property
    def status(self):
        return self._status.name

    def train(self):
        self._status = MasterOfPuppetsStatus.TRAIN

    def simulate(self):
        self._status = MasterOfPuppetsStatus.SIMULATE

    def _ring(self):
        if self._learner._device.type != 'cuda':
            return None
        if self._replay is None:
            self._replay = ReplayBuffer(self._max_length, self._learner._device)
        return self._replay

    def push_data(self, data):
        """One episode's rows (app/learner.py:54 -> app/base.py:182-185)."""
        if MasterOfPuppetsStatus[self.status] == MasterOfPuppetsStatus.SIMULATE:
            self._episode_counter += 1
            self._dataset.push(data)
            ring = self._ring()
            if ring is not None:
                ring.push_rows(list(data))
            else:
                self._arrivals.append(('rows', data))

    def push_records(self, records, episodes):
        """push_data for packed rows (EpisodeRecords) of `episodes` episodes.  On a GPU learner
        the rows go straight into the HBM replay ring (ReplayBuffer), encoded on arrival."""
        if MasterOfPuppetsStatus[self.status] == MasterOfPuppetsStatus.SIMULATE:
            self._episode_counter += episodes
            ring = self._ring()
            if ring is not None:
                ring.push_records(records)
            else:
                self._arrivals.append(('records', records))
                self._records = EpisodeRecords.concat([self._records, records]).tail(self._max_length)

    def update(self, encode=True):
        """app/base.py:188-195: load the current weights, train on the dataset, publish the new
        weights as a new version, start a fresh dataset.  Returns get_weights_dict() plus
        'loss'; encode=False puts the state_dict itself under 'weights' (for callers that move
        the tensors over torch.distributed instead of HTTP, minitchess_alphazero_amd.loop)."""
        self._network.load_state_dict(self.weights)
        kinds = {k for k, _ in self._arrivals}
        if kinds == {'rows', 'records'}:
            # both push paths were used: train on every row in arrival order, as the reference's
            # one dataset holds everything pushed since the last update (exp/dataset.py:12-13)
            data = SimpleAlphaZeroDataset(max_length=self._max_length)
            for kind, payload in self._arrivals:
                data.push(payload if kind == 'rows' else payload.to_rows())
        elif self._replay is not None and len(self._replay):
            data = self._replay
        else:
            data = self._records if len(self._records) else self._dataset
        loss = self._learner.update(data)
        self.weights = self._network.state_dict()
        self._init_dataset()
        out = self.get_weights_dict() if encode else {'weights': copy.copy(self.weights),
                                                      'version': self.weights_version}
        out['loss'] = loss
        return out

    def get_weights_dict(self):
        """app/base.py:201-203: {'weights': jsonpickle.encode(state_dict), 'version'}, the
        document the learner posts to rlweb (minitchess_alphazero_amd.wire)."""
        from .wire import get_weights_dict
        return get_weights_dict(self.weights, self.weights_version)
