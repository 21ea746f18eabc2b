"""MinitChess rules restatement with the python-chess API surface the reference uses.

TEST INFRASTRUCTURE (see oracle/__init__.py).

The reference delegates all rules to the un-vendored python-chess "minitchess"
fork (README.md:13-17, Dockerfile:14-15).  This module restates the rules the
build assumes (RULES.md) behind exactly the API the reference consumes:

  chess.Board(fen), .fen(), .result(), .legal_moves, .push(move), .turn
      exp/environment.py:25,36,39,48,76
  chess.Move.from_uci(uci), Move(from_square=, to_square=).uci(), equality
      exp/environment.py:72-76, exp/generate_moves_list.py:45,55

so that tests/golden/make_golden.py can inject it as the `chess` module when
importing the reference's exp/*.py.  The HIP rules (csrc/rules.h) must agree
with this module bit-for-bit (tests/test_rules_*.py).

Board geometry: 5 files x 6 ranks, square = 5*rank + file,
name = 'abcde'[file] + str(rank + 1).  FEN has 4 fields: board turn half full.
"""

FILES = 'abcde'
NFILES, NRANKS, NSQ = 5, 6, 30
WHITE, BLACK = True, False
PAWN, KNIGHT, BISHOP, ROOK, QUEEN, KING = 1, 2, 3, 4, 5, 6
PIECE_SYMBOLS = [None, 'p', 'n', 'b', 'r', 'q', 'k']
SYMBOL_TO_TYPE = {s: i for i, s in enumerate(PIECE_SYMBOLS) if s}

STARTING_FEN = '2nbk/2ppp/5/5/PPP2/KBN2 w 0 1'   # exp/environment.py:6

# Rule switches (RULES.md).  Defaults are the build's assumption about the fork.
RULES = {
    'double_step': False,    # no pawn double step (the 4-field FEN has no ep field)
    'promo_all': True,       # python-chess generates q, r, b, n promotions
    'insufficient': True,    # python-chess is_insufficient_material draw
    'fivefold': True,        # python-chess fivefold repetition (game history only)
    'seventyfive': True,     # python-chess 75-move rule
    'move_cap': 30,          # draw once fullmove_number > cap (exp/policy.py:11-12)
}

PROMOTIONS_ALL = (QUEEN, ROOK, BISHOP, KNIGHT)


def square_name(sq):
    return FILES[sq % NFILES] + str(sq // NFILES + 1)


def parse_square(name):
    f = FILES.index(name[0])
    r = int(name[1]) - 1
    if not (0 <= r < NRANKS):
        raise ValueError(name)
    return r * NFILES + f


def _sq(f, r):
    return r * NFILES + f if (0 <= f < NFILES and 0 <= r < NRANKS) else None


def _build_tables():
    knight, king, rays = [], [], []
    pawn_att = {WHITE: [], BLACK: []}          # squares a pawn of colour c on sq attacks
    pawn_attackers = {WHITE: [], BLACK: []}    # squares from which a pawn of c attacks sq
    kd = [(1, 2), (1, -2), (-1, 2), (-1, -2), (2, 1), (2, -1), (-2, 1), (-2, -1)]
    gd = [(dx, dy) for dx in (-1, 0, 1) for dy in (-1, 0, 1) if dx or dy]
    dirs = [(0, 1), (0, -1), (1, 0), (-1, 0), (1, 1), (1, -1), (-1, 1), (-1, -1)]
    for sq in range(NSQ):
        f, r = sq % NFILES, sq // NFILES
        knight.append(tuple(s for s in (_sq(f + dx, r + dy) for dx, dy in kd) if s is not None))
        king.append(tuple(s for s in (_sq(f + dx, r + dy) for dx, dy in gd) if s is not None))
        rr = []
        for dx, dy in dirs:
            ray, k = [], 1
            while _sq(f + k * dx, r + k * dy) is not None:
                ray.append(_sq(f + k * dx, r + k * dy))
                k += 1
            rr.append(tuple(ray))
        rays.append(tuple(rr))
        for c, dy in ((WHITE, 1), (BLACK, -1)):
            pawn_att[c].append(tuple(s for s in (_sq(f - 1, r + dy), _sq(f + 1, r + dy)) if s is not None))
            pawn_attackers[c].append(tuple(s for s in (_sq(f - 1, r - dy), _sq(f + 1, r - dy)) if s is not None))
    return knight, king, rays, pawn_att, pawn_attackers


KNIGHT_T, KING_T, RAYS, PAWN_ATT, PAWN_ATTACKERS = _build_tables()
ORTHO, DIAG = (0, 1, 2, 3), (4, 5, 6, 7)
DARK = [((sq % NFILES) + (sq // NFILES)) % 2 == 0 for sq in range(NSQ)]   # a1 dark


class Move:
    """python-chess Move subset (from_square, to_square, promotion, uci)."""
    __slots__ = ('from_square', 'to_square', 'promotion')

    def __init__(self, from_square, to_square, promotion=None):
        self.from_square = from_square
        self.to_square = to_square
        self.promotion = promotion

    def uci(self):
        s = square_name(self.from_square) + square_name(self.to_square)
        return s + PIECE_SYMBOLS[self.promotion] if self.promotion else s

    @classmethod
    def from_uci(cls, uci):
        if len(uci) == 4:
            return cls(parse_square(uci[0:2]), parse_square(uci[2:4]))
        if len(uci) == 5:
            return cls(parse_square(uci[0:2]), parse_square(uci[2:4]), SYMBOL_TO_TYPE[uci[4]])
        raise ValueError(f'invalid uci: {uci!r}')

    def __eq__(self, other):
        return (isinstance(other, Move) and self.from_square == other.from_square
                and self.to_square == other.to_square and self.promotion == other.promotion)

    def __hash__(self):
        return hash((self.from_square, self.to_square, self.promotion))

    def __repr__(self):
        return f'Move.from_uci({self.uci()!r})'

    def __str__(self):
        return self.uci()


def is_attacked(bd, sq, by_white):
    """True if square sq is attacked by the side `by_white` on mailbox bd."""
    s = 1 if by_white else -1
    n, k, p, b, r, q = 2 * s, 6 * s, 1 * s, 3 * s, 4 * s, 5 * s
    for t in KNIGHT_T[sq]:
        if bd[t] == n:
            return True
    for t in KING_T[sq]:
        if bd[t] == k:
            return True
    for t in PAWN_ATTACKERS[by_white][sq]:
        if bd[t] == p:
            return True
    rays = RAYS[sq]
    for d in ORTHO:
        for t in rays[d]:
            v = bd[t]
            if v:
                if v == r or v == q:
                    return True
                break
    for d in DIAG:
        for t in rays[d]:
            v = bd[t]
            if v:
                if v == b or v == q:
                    return True
                break
    return False


def pseudo_targets(bd, sq, white, double_step=None):
    """Pseudo-legal destination squares of the piece on sq (side to move `white`)."""
    if double_step is None:
        double_step = RULES['double_step']
    v = bd[sq]
    t = v if white else -v
    out = []
    if t == PAWN:
        dy = 5 if white else -5
        fwd = sq + dy
        if 0 <= fwd < NSQ and bd[fwd] == 0:
            out.append(fwd)
            start_rank = 1 if white else NRANKS - 2
            if double_step and sq // NFILES == start_rank and bd[fwd + dy] == 0:
                out.append(fwd + dy)
        for c in PAWN_ATT[white][sq]:
            w = bd[c]
            if w and ((w < 0) if white else (w > 0)):
                out.append(c)
    elif t == KNIGHT or t == KING:
        for c in (KNIGHT_T[sq] if t == KNIGHT else KING_T[sq]):
            w = bd[c]
            if not w or ((w < 0) if white else (w > 0)):
                out.append(c)
    else:
        dirs = ORTHO if t == ROOK else DIAG if t == BISHOP else ORTHO + DIAG
        rays = RAYS[sq]
        for d in dirs:
            for c in rays[d]:
                w = bd[c]
                if not w:
                    out.append(c)
                else:
                    if (w < 0) if white else (w > 0):
                        out.append(c)
                    break
    return out


def king_square(bd, white):
    k = KING if white else -KING
    for i in range(NSQ):
        if bd[i] == k:
            return i
    return None


def apply_move(bd, frm, to, promotion, white):
    """Return the new mailbox after a move (no legality checks)."""
    nb = list(bd)
    v = nb[frm]
    nb[frm] = 0
    if promotion:
        v = promotion if white else -promotion
    nb[to] = v
    return nb


class Board:
    """python-chess Board subset for MinitChess (see module docstring)."""

    def __init__(self, fen=STARTING_FEN):
        self.move_stack = []
        self._keys = []      # transposition key of the position before each pushed move
        self._zeroing = []   # whether that move was zeroing (capture / pawn move)
        self._legal = None
        self.set_fen(fen)

    # ---- FEN ---------------------------------------------------------------------
    def set_fen(self, fen):
        parts = fen.split()
        if len(parts) != 4:
            raise ValueError(f'expected 4-field MinitChess FEN: {fen!r}')
        rows = parts[0].split('/')
        if len(rows) != NRANKS:
            raise ValueError(f'expected {NRANKS} ranks: {fen!r}')
        bd = [0] * NSQ
        for i, row in enumerate(rows):
            r = NRANKS - 1 - i
            f = 0
            for ch in row:
                if ch.isdigit():
                    f += int(ch)
                else:
                    t = SYMBOL_TO_TYPE[ch.lower()]
                    if f >= NFILES:
                        raise ValueError(fen)
                    bd[r * NFILES + f] = t if ch.isupper() else -t
                    f += 1
            if f != NFILES:
                raise ValueError(f'bad rank {row!r} in {fen!r}')
        if parts[1] not in ('w', 'b'):
            raise ValueError(fen)
        self.board = bd
        self.turn = parts[1] == 'w'
        self.halfmove_clock = int(parts[2])
        self.fullmove_number = int(parts[3])
        self.move_stack, self._keys, self._zeroing, self._legal = [], [], [], None

    def board_fen(self):
        out = []
        bd = self.board
        for r in range(NRANKS - 1, -1, -1):
            row, e = '', 0
            for f in range(NFILES):
                v = bd[r * NFILES + f]
                if v == 0:
                    e += 1
                else:
                    if e:
                        row += str(e)
                        e = 0
                    s = PIECE_SYMBOLS[abs(v)]
                    row += s.upper() if v > 0 else s
            if e:
                row += str(e)
            out.append(row)
        return '/'.join(out)

    def fen(self):
        return f"{self.board_fen()} {'w' if self.turn else 'b'} {self.halfmove_clock} {self.fullmove_number}"

    def copy(self):
        b = Board.__new__(Board)
        b.board = list(self.board)
        b.turn, b.halfmove_clock, b.fullmove_number = self.turn, self.halfmove_clock, self.fullmove_number
        b.move_stack, b._keys, b._zeroing = list(self.move_stack), list(self._keys), list(self._zeroing)
        b._legal = self._legal
        return b

    def piece_type_at(self, sq):
        v = self.board[sq]
        return abs(v) if v else None

    # ---- move generation -----------------------------------------------------------
    def _gen_legal(self):
        bd, white = self.board, self.turn
        promo = PROMOTIONS_ALL if RULES['promo_all'] else (QUEEN,)
        last_rank = NRANKS - 1 if white else 0
        ksq = king_square(bd, white)
        out = []
        for sq in range(NSQ):
            v = bd[sq]
            if not v or (v > 0) != white:
                continue
            is_pawn = abs(v) == PAWN
            for to in pseudo_targets(bd, sq, white):
                nb = apply_move(bd, sq, to, None, white)
                k = to if abs(v) == KING else ksq
                if k is not None and is_attacked(nb, k, not white):
                    continue
                if is_pawn and to // NFILES == last_rank:
                    for p in promo:
                        out.append(Move(sq, to, p))
                else:
                    out.append(Move(sq, to))
        return out

    @property
    def legal_moves(self):
        if self._legal is None:
            self._legal = self._gen_legal()
        return self._legal

    def is_check(self):
        k = king_square(self.board, self.turn)
        return k is not None and is_attacked(self.board, k, not self.turn)

    def is_checkmate(self):
        return self.is_check() and not self.legal_moves

    def is_stalemate(self):
        return not self.is_check() and not self.legal_moves

    def is_zeroing(self, move):
        v = self.board[move.from_square]
        w = self.board[move.to_square]
        return abs(v) == PAWN or (w != 0 and (w > 0) != self.turn)

    def _key(self):
        return (tuple(self.board), self.turn)

    def push(self, move):
        self._keys.append(self._key())
        self._zeroing.append(self.is_zeroing(move))
        self.move_stack.append(move)
        if self._zeroing[-1]:
            self.halfmove_clock = 0
        else:
            self.halfmove_clock += 1
        if not self.turn:
            self.fullmove_number += 1
        self.board = apply_move(self.board, move.from_square, move.to_square, move.promotion, self.turn)
        self.turn = not self.turn
        self._legal = None

    # ---- game end ----------------------------------------------------------------------
    def has_insufficient_material(self, white):
        """python-chess Board.has_insufficient_material on the 5x6 board."""
        bd = self.board
        own = [abs(v) for v in bd if v and (v > 0) == white]
        if any(t in (PAWN, ROOK, QUEEN) for t in own):
            return False
        opp = [abs(v) for v in bd if v and (v > 0) != white]
        if KNIGHT in own:
            return len(own) <= 2 and not any(t not in (KING, QUEEN) for t in opp)
        if BISHOP in own:
            bishops = [sq for sq in range(NSQ) if abs(bd[sq]) == BISHOP]
            same_colour = all(DARK[sq] for sq in bishops) or not any(DARK[sq] for sq in bishops)
            any_pawn = any(abs(v) == PAWN for v in bd)
            any_knight = any(abs(v) == KNIGHT for v in bd)
            return same_colour and not any_pawn and not any_knight
        return True

    def is_insufficient_material(self):
        return self.has_insufficient_material(True) and self.has_insufficient_material(False)

    def is_fivefold_repetition(self):
        """python-chess is_repetition(5): positions since the last irreversible move."""
        cur = self._key()
        count = 1
        for i in range(len(self._keys) - 1, -1, -1):
            if self._zeroing[i]:
                break
            if self._keys[i] == cur:
                count += 1
                if count >= 5:
                    return True
        return False

    def is_seventyfive_moves(self):
        return self.halfmove_clock >= 150 and bool(self.legal_moves)

    def result(self):
        if self.is_checkmate():
            return '0-1' if self.turn else '1-0'
        if RULES['seventyfive'] and self.is_seventyfive_moves():
            return '1/2-1/2'
        if RULES['fivefold'] and self.is_fivefold_repetition():
            return '1/2-1/2'
        if RULES['insufficient'] and self.is_insufficient_material():
            return '1/2-1/2'
        if not self.legal_moves:
            return '1/2-1/2'
        cap = RULES['move_cap']
        if cap and self.fullmove_number > cap:
            return '1/2-1/2'
        return '*'

    def is_game_over(self):
        return self.result() != '*'

    def __repr__(self):
        return f'Board({self.fen()!r})'
