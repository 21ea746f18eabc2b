"""MinitChess environment restatement over oracle.rules (TEST INFRASTRUCTURE, see oracle/__init__.py).

Behaviour of exp/environment.py:1-91 that the tests pin:
  * observation = 4-field FEN; result '1-0'/'0-1' -> reward 1.0, '1/2-1/2' -> 0.0,
    done; an ongoing position leaves the previous reward untouched (:39-45, the `self_reward`
    typo means _reward is only ever None or a terminal reward)
  * legal moves = codes of m.uci()[:4], sorted, duplicates kept (:48-50)
  * step: terminal -> TerminatedEpisodeStepException; decode the code, try the uci4 move,
    then the queen promotion, else IlegalMoveException (:68-82)
  * both exceptions derive from BaseException (:8-13)
"""
from collections import namedtuple

from . import rules
from .codec import moves_dict

STARTING_FEN = rules.STARTING_FEN

EpisodeStatus = namedtuple('EpisodeStatus', ['observation', 'reward', 'done'])


def _side_tables():
    md = moves_dict()
    enc = {True: md['w'], False: md['b']}
    dec = {side: {code: uci for uci, code in table.items()} for side, table in enc.items()}
    return enc, dec


MOVES_DICT, MOVES_DICT_INV = _side_tables()
NUM_ACTIONS = len(MOVES_DICT[True])


class TerminatedEpisodeStepException(BaseException):
    pass


class IlegalMoveException(BaseException):
    pass


_RESULT_REWARD = {'1-0': 1.0, '0-1': 1.0, '1/2-1/2': 0.0}


class MinitChessEpisode:
    def __init__(self, fen, board=None):
        self._board = rules.Board(fen) if board is None else board
        self._reward = None
        self._done = None
        self._refresh()

    def _refresh(self):
        b = self._board
        self._observation = b.fen()
        outcome = b.result()
        if outcome in _RESULT_REWARD:
            self._reward, self._done = _RESULT_REWARD[outcome], True
        else:
            self._done = False
        self._moves = list(b.legal_moves)
        table = MOVES_DICT[b.turn]
        self._codes = sorted(table[m.uci()[:4]] for m in self._moves)

    def get_observation(self):
        return self._observation

    def get_reward(self):
        return self._reward

    def is_done(self):
        return self._done

    def get_legal_moves(self):
        return self._codes

    @property
    def turn(self):
        return self._board.turn

    @property
    def board(self):
        return self._board

    def step(self, action, return_status=True):
        if self._done:
            raise TerminatedEpisodeStepException
        uci4 = MOVES_DICT_INV[self.turn][action]
        for candidate in (uci4, uci4 + 'q'):
            mv = rules.Move.from_uci(candidate)
            if mv in self._moves:
                break
        else:
            raise IlegalMoveException
        self._board.push(mv)
        self._refresh()
        return self.get_status() if return_status else None

    def get_status(self):
        return EpisodeStatus(self._observation, self._reward, self._done)


class MinitChessEnvironment:
    def new_episode(self, fen=None):
        ep = MinitChessEpisode(fen or STARTING_FEN)
        return ep, ep.get_observation()
