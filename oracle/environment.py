"""MinitChess environment / episode restatement (TEST INFRASTRUCTURE, see oracle/__init__.py).

Restates exp/environment.py:1-91 over oracle.rules (the fork stand-in):
  * _update_attributes: FEN observation, result -> (reward, done), legal move
    codes SORTED with duplicates kept (:34-50)
  * step: uci4 decode, retry with +'q' (queen promotion), else IlegalMove (:68-82)
  * exceptions derive from BaseException (:8-13)
"""
from collections import namedtuple

from . import rules
from .codec import moves_dict

STARTING_FEN = rules.STARTING_FEN

EpisodeStatus = namedtuple('EpisodeStatus', ['observation', 'reward', 'done'])

_MD = moves_dict()
MOVES_DICT = {True: _MD['w'], False: _MD['b']}                                     # :16-18
MOVES_DICT_INV = {side: {v: k for k, v in MOVES_DICT[side].items()} for side in (True, False)}  # :19
NUM_ACTIONS = len(MOVES_DICT[True])


class TerminatedEpisodeStepException(BaseException):
    pass


class IlegalMoveException(BaseException):
    pass


class MinitChessEpisode:
    def __init__(self, fen, board=None):
        self._board = board if board is not None else rules.Board(fen)
        self._reward = None
        self._done = None
        self._update_attributes()

    def _update_attributes(self):                                                  # :34-50
        self._observation = self._board.fen()
        res = self._board.result()
        if res in ('1-0', '0-1'):
            self._reward, self._done = 1., True
        elif res == '1/2-1/2':
            self._reward, self._done = 0., True
        else:
            self._done = False          # NB the reference never resets _reward here (:45 typo)
        self._legal_moves_uci = list(self._board.legal_moves)
        side = MOVES_DICT[self.turn]
        self._legal_moves = sorted(side[m.uci()[:4]] for m in self._legal_moves_uci)

    def get_observation(self):
        return self._observation

    def get_reward(self):
        return self._reward

    def is_done(self):
        return self._done

    def get_legal_moves(self):
        return self._legal_moves

    @property
    def turn(self):
        return self._board.turn

    @property
    def board(self):
        return self._board

    def step(self, action, return_status=True):                                   # :68-82
        if self.is_done():
            raise TerminatedEpisodeStepException
        uci = MOVES_DICT_INV[self.turn][action]
        move = rules.Move.from_uci(uci)
        if move not in self._legal_moves_uci:
            move = rules.Move.from_uci(uci + 'q')
        if move not in self._legal_moves_uci:
            raise IlegalMoveException
        self._board.push(move)
        self._update_attributes()
        if return_status:
            return self.get_status()

    def get_status(self):
        return EpisodeStatus(self._observation, self._reward, self._done)


class MinitChessEnvironment:
    def new_episode(self, fen=None):                                               # :88-91
        episode = MinitChessEpisode(fen or STARTING_FEN)
        return episode, episode.get_observation()
