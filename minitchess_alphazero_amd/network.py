"""Policy/value network: drop-in for exp/policy.py's Network.

Parameter creation order and state_dict keys equal the reference's
(exp/policy.py:53-69), so `torch.manual_seed(0); Network()` yields the reference's
random-init weights and `load_state_dict` accepts reference checkpoints.

Self-play inference does not use this module's forward: it runs in the HIP kernels (k_net_y by
default, csrc/mtaz_net16.hip, precision 'f16x3'; k_net_z, csrc/mtaz_net8.hip, precision 'f16f8',
is an option outside the 1e-5 contract on trained nets) through Engine.set_weights /
Engine.evaluate.  The torch
forward below is the TRAINING path of the learner (exp/learner.py:84-88; autograd on
PyTorch-ROCm): train-mode BatchNorm uses batch statistics, which the folded
inference kernels cannot express.
"""
import torch
from torch import nn

NUM_ACTIONS = 554
EMBEDDING_DIM = 4
MAX_NUM_MOVES_ALLOWED = 30


class _ConvBN(nn.Module):
    """exp/policy.py:15-38 ConvBlock: Conv2d(k, pad k//2) -> BatchNorm2d [-> ReLU]."""

    def __init__(self, cin, cout, k, relu=True):
        super().__init__()
        mods = [nn.Conv2d(cin, cout, kernel_size=k, stride=1, padding=k // 2), nn.BatchNorm2d(cout)]
        if relu:
            mods.append(nn.ReLU())
        self.layers = nn.Sequential(*mods)

    def forward(self, x):
        return self.layers(x)


def _conv_bn(cin, cout, k, relu=True):
    return _ConvBN(cin, cout, k, relu)


class _Residual(nn.Module):
    """exp/policy.py:41-50: relu(convblock2(convblock1(x)) + x)."""

    def __init__(self, ch):
        super().__init__()
        self.convblock1 = _conv_bn(ch, ch, 3)
        self.convblock2 = _conv_bn(ch, ch, 3, relu=False)
        self.nonl = nn.ReLU()

    def forward(self, x):
        return self.nonl(self.convblock2(self.convblock1(x)) + x)


class Network(nn.Module):
    def __init__(self, num_actions=NUM_ACTIONS):
        super().__init__()
        self.emb = nn.Embedding(7, EMBEDDING_DIM)
        self.resbody = nn.Sequential(_conv_bn(2 * EMBEDDING_DIM, 256, 3), *[_Residual(256) for _ in range(9)])
        self.pconv = _conv_bn(256, 2, 1)
        self.plinear = nn.Linear(2 * 6 * 5 + 1, num_actions)
        self.vconv = _conv_bn(256, 1, 1)
        self.vlinear = nn.Sequential(nn.Linear(6 * 5 + 1, 256), nn.ReLU(), nn.Linear(256, 1), nn.Tanh())

    def forward(self, input_data):
        """Training forward (exp/policy.py:71-80): tokens (B,2,6,5) int64, clock (B,1) ->
        (logits (B,554), value (B,1))."""
        tokens, clock = input_data
        x = self.emb(tokens).permute(0, 1, 4, 2, 3).reshape(-1, 2 * EMBEDDING_DIM, 6, 5)
        x = self.resbody(x)
        logits = self.plinear(torch.cat([self.pconv(x).flatten(1), clock], dim=1))
        value = self.vlinear(torch.cat([self.vconv(x).flatten(1), clock], dim=1))
        return logits, value

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
