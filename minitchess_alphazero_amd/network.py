"""Policy/value network parameters: drop-in for exp/policy.py's Network as a weight container.

PyTorch holds the parameters only (device memory + the state_dict format the
reference's learner/rlweb exchange, app/base.py:126-129, :171-174).  Parameter
creation order and state_dict keys equal the reference's (exp/policy.py:53-69),
so `torch.manual_seed(0); Network()` yields the reference's random-init weights
and `load_state_dict` accepts reference checkpoints.  Inference runs in the HIP
kernels (csrc/mtaz_device.hip) through Engine.set_weights / Engine.evaluate;
there is no torch forward on the product path.
"""
import torch
from torch import nn

NUM_ACTIONS = 554
EMBEDDING_DIM = 4
MAX_NUM_MOVES_ALLOWED = 30


def _conv_bn(cin, cout, k, relu=True):
    m = nn.Module()
    mods = [nn.Conv2d(cin, cout, kernel_size=k, stride=1, padding=k // 2), nn.BatchNorm2d(cout)]
    if relu:
        mods.append(nn.ReLU())
    m.layers = nn.Sequential(*mods)
    return m


class _Residual(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.convblock1 = _conv_bn(ch, ch, 3)
        self.convblock2 = _conv_bn(ch, ch, 3, relu=False)
        self.nonl = nn.ReLU()


class Network(nn.Module):
    def __init__(self, num_actions=NUM_ACTIONS):
        super().__init__()
        self.emb = nn.Embedding(7, EMBEDDING_DIM)
        self.resbody = nn.Sequential(_conv_bn(2 * EMBEDDING_DIM, 256, 3), *[_Residual(256) for _ in range(9)])
        self.pconv = _conv_bn(256, 2, 1)
        self.plinear = nn.Linear(2 * 6 * 5 + 1, num_actions)
        self.vconv = _conv_bn(256, 1, 1)
        self.vlinear = nn.Sequential(nn.Linear(6 * 5 + 1, 256), nn.ReLU(), nn.Linear(256, 1), nn.Tanh())

    def forward(self, *a, **k):
        raise NotImplementedError('inference runs in the HIP engine: use Engine.evaluate / Engine.play')

    @classmethod
    def process_observation(cls, observation):
        """exp/policy.py:96-105 (same tensors), computed by the libmtaz encoder."""
        from .environment import pos_encode, pos_from_fen
        tokens, clock = pos_encode(pos_from_fen(observation))
        return torch.from_numpy(tokens).reshape(1, 2, 6, 5), torch.tensor([[clock]], dtype=torch.float32)


def weight_tensors(network_or_state_dict):
    """The 133 float32 tensors the C ABI expects (state_dict order, num_batches_tracked skipped)."""
    sd = network_or_state_dict.state_dict() if hasattr(network_or_state_dict, 'state_dict') else network_or_state_dict
    out = [v for k, v in sd.items() if not k.endswith('num_batches_tracked')]
    if len(out) != 133:
        raise ValueError(f'expected 133 tensors, got {len(out)}')
    return out
