"""Random MinitChess positions for tests (oracle rules random walks)."""
import numpy as np


def random_fens(n, seed=0, max_plies=80):
    from oracle import rules
    rs = np.random.RandomState(seed)
    out = []
    while len(out) < n:
        b = rules.Board(rules.STARTING_FEN)
        for _ in range(rs.randint(0, max_plies)):
            m = b.legal_moves
            if not m or b.result() != '*':
                break
            b.push(m[rs.randint(len(m))])
            out.append(b.fen())
    return out[:n]
