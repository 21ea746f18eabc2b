"""CPU torch restatement of the reference ResNet (TEST INFRASTRUCTURE, see oracle/__init__.py).

exp/policy.py:15-80.  Parameter creation order and state_dict keys match the
reference so that `torch.manual_seed(0); Network()` reproduces its random-init
weights bit-for-bit (sha256 pinned in tests/golden/net.json):

  emb                      Embedding(7, 4)                                  :56
  resbody.0                ConvBlock(8 -> 256, 3x3, pad 1) conv, BN, ReLU    :58
  resbody.1..9             ResidualBlock: ConvBlock, ConvBlock(no ReLU), +x, ReLU   :41-50, :59-60
  pconv / plinear          ConvBlock(256 -> 2, 1x1), Linear(61 -> 554)      :62-63
  vconv / vlinear          ConvBlock(256 -> 1, 1x1), Linear(31,256) ReLU Linear(256,1) Tanh   :65-69

Forward (:71-80): emb -> permute(0,1,4,2,3) -> view(B, 8, 6, 5) -> trunk ->
policy logits from [flatten(pconv), clock]; value from [flatten(vconv), clock].
"""
import torch
from torch import nn

NUM_ACTIONS = 554
EMBEDDING_DIM = 4


def conv_block(cin, cout, k, relu=True):
    # module attribute `layers` = Sequential(conv, bn[, relu]) gives keys layers.0.*, layers.1.*
    blk = nn.Module()
    mods = [nn.Conv2d(cin, cout, kernel_size=k, stride=1, padding=k // 2), nn.BatchNorm2d(cout)]
    if relu:
        mods.append(nn.ReLU())
    blk.layers = nn.Sequential(*mods)
    blk.forward = blk.layers.forward
    return blk


class Residual(nn.Module):
    def __init__(self, ch):
        super().__init__()
        self.convblock1 = conv_block(ch, ch, 3)
        self.convblock2 = conv_block(ch, ch, 3, relu=False)

    def forward(self, x):
        return torch.relu(self.convblock2(self.convblock1(x)) + x)


class Network(nn.Module):
    def __init__(self, num_actions=NUM_ACTIONS, channels=256, blocks=9):
        super().__init__()
        self.emb = nn.Embedding(7, EMBEDDING_DIM)
        self.resbody = nn.Sequential(conv_block(2 * EMBEDDING_DIM, channels, 3),
                                     *[Residual(channels) for _ in range(blocks)])
        self.pconv = conv_block(channels, 2, 1)
        self.plinear = nn.Linear(2 * 30 + 1, num_actions)
        self.vconv = conv_block(channels, 1, 1)
        self.vlinear = nn.Sequential(nn.Linear(30 + 1, 256), nn.ReLU(), nn.Linear(256, 1), nn.Tanh())

    def forward(self, input_data):
        tokens, clock = input_data
        x = self.emb(tokens).permute(0, 1, 4, 2, 3).contiguous().view(-1, 2 * EMBEDDING_DIM, 6, 5)
        x = self.resbody(x)
        p = self.plinear(torch.cat([self.pconv(x).view(-1, 60), clock], dim=1))
        v = self.vlinear(torch.cat([self.vconv(x).view(-1, 30), clock], dim=1))
        return p, v


def seed0_network():
    """The bench / fixture weights: torch.manual_seed(0); Network()."""
    torch.manual_seed(0)
    return Network().eval()


def state_dict_sha256(net):
    import hashlib
    h = hashlib.sha256()
    for k, v in net.state_dict().items():
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()
