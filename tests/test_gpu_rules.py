"""GPU: batched legal-list / mask / outcome / encoder kernels vs the oracle (bit-exact)."""
import ctypes

import numpy as np
import pytest

from conftest import LONG_LIST_FENS, load_golden

pytestmark = pytest.mark.gpu


def _positions(n, seed=5):
    from oracle import rules
    rs = np.random.RandomState(seed)
    out = []
    while len(out) < n:
        b = rules.Board(rules.STARTING_FEN)
        for _ in range(rs.randint(0, 80)):
            m = b.legal_moves
            if not m:
                break
            b.push(m[rs.randint(len(m))])
            out.append(b.fen())
            if b.result() != '*':
                break
    return out[:n] + [f['fen'] for f in load_golden('encoder')] + LONG_LIST_FENS


def test_legal_batch_kernel_matches_oracle():
    import torch
    from minitchess_alphazero_amd import _lib
    from minitchess_alphazero_amd.environment import pos_from_fen
    from oracle.environment import MinitChessEpisode
    from oracle import rules
    fens = _positions(3000)
    pos = np.stack([pos_from_fen(f) for f in fens])
    n = len(fens)
    dev = torch.device('cuda', 0)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    d_codes = torch.zeros((n, _lib.KMAX), dtype=torch.int16, device=dev)
    d_counts = torch.zeros(n, dtype=torch.int32, device=dev)
    d_masks = torch.zeros((n, 18), dtype=torch.int32, device=dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    L = _lib.lib()
    _lib.check(L.mtaz_legal_batch(0, d_pos.data_ptr(), n, _lib.RF_DEFAULT, 30, d_codes.data_ptr(), d_counts.data_ptr(),
                                  d_masks.data_ptr(), d_out.data_ptr(), None))
    codes = d_codes.cpu().numpy().view(np.uint16)
    counts = d_counts.cpu().numpy()
    masks = d_masks.cpu().numpy().view(np.uint32)
    outs = d_out.cpu().numpy()
    for i, f in enumerate(fens):
        ep = MinitChessEpisode(f)
        legal = ep.get_legal_moves()
        assert counts[i] == len(legal), f
        assert codes[i, :counts[i]].tolist() == legal, f
        m = np.zeros(18, np.uint32)
        for c in legal:
            m[c >> 5] |= np.uint32(1 << (c & 31))
        assert np.array_equal(masks[i], m), f
        b = rules.Board(f)         # no history: exactly the MCTS-episode view
        res = b.result()
        exp = 0 if res == '*' else (1 if res in ('1-0', '0-1') else 2)
        assert outs[i] == exp, f


def test_encode_batch_kernel_matches_reference():
    import torch
    from minitchess_alphazero_amd import _lib
    from minitchess_alphazero_amd.environment import pos_from_fen
    rows = load_golden('encoder')
    pos = np.stack([pos_from_fen(r['fen']) for r in rows])
    n = len(rows)
    dev = torch.device('cuda', 0)
    d_pos = torch.from_numpy(pos.view(np.int32)).to(dev)
    d_tok = torch.zeros((n, 60), dtype=torch.uint8, device=dev)
    d_clk = torch.zeros(n, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    _lib.check(_lib.lib().mtaz_encode_batch(0, d_pos.data_ptr(), n, d_tok.data_ptr(), d_clk.data_ptr(), None))
    tok = d_tok.cpu().numpy()
    clk = d_clk.cpu().numpy()
    for i, r in enumerate(rows):
        assert tok[i].tolist() == r['tokens'], r['fen']
        assert float(clk[i]) == r['clock']
