"""FEN -> network input (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates exp/policy.py:82-105:
  * side view: white keeps the board FEN, black reverses it and swaps case (:85)
  * digits expanded, '/' dropped -> 30 characters (:89-91)
  * plane 0 = pieces of the side to move, plane 1 = the opponent's, each coded
    by '0prbnqk' (:7, :92-94)
  * clock = (fullmove + 0.5*[black]) / 30 as float32 (:101-104)
"""
import numpy as np

CODES = {v: k for k, v in enumerate('0prbnqk')}
MAX_NUM_MOVES_ALLOWED = 30


def side_view(bfen, color):
    assert color in ('w', 'b')
    return bfen if color == 'w' else bfen[::-1].swapcase()


def tokenize(bfen, color):
    s = side_view(bfen, color).replace('/', '')
    flat = []
    for ch in s:
        if ch.isdigit():
            flat.extend('0' * int(ch))
        else:
            flat.append(ch)
    own = [CODES[ch.lower()] if ch.isupper() else 0 for ch in flat]
    opp = [CODES[ch] if ch.islower() else 0 for ch in flat]
    return own + opp


def encode(fen):
    """-> (tokens int64[60], clock float32)."""
    bfen, color, _half, full = fen.split()
    tokens = np.asarray(tokenize(bfen, color), dtype=np.int64)
    clock = float(full) + (0.5 if color == 'b' else 0.0)
    return tokens, np.float32(clock / MAX_NUM_MOVES_ALLOWED)


def process_observation(fen):
    """Same tensors the reference feeds its Network: (LongTensor(1,2,6,5), FloatTensor(1,1))."""
    import torch
    tokens, clock = encode(fen)
    return torch.from_numpy(tokens).reshape(1, 2, 6, 5), torch.tensor([[clock]], dtype=torch.float32)
