"""MinitChess environment: drop-in for the reference's exp/environment.py.

Same public surface (exp/environment.py:1-91): STARTING_FEN, MOVES_DICT,
MOVES_DICT_INV, NUM_ACTIONS, TerminatedEpisodeStepException and
IlegalMoveException (BaseException subclasses, :8-13), MinitChessEpisode
(get_observation / get_reward / is_done / get_legal_moves / turn / step /
get_status) and MinitChessEnvironment.new_episode(fen=None).

The rules run in libmtaz (csrc/rules.h, the same code the GPU kernels use)
instead of the python-chess fork; positions are packed 5 x uint32 keys.
"""
import ctypes
import json
from collections import namedtuple

import numpy as np

from . import _lib

STARTING_FEN = '2nbk/2ppp/5/5/PPP2/KBN2 w 0 1'        # exp/environment.py:6
MOVE_CAP = 30                                         # exp/policy.py:11-12 (RULES.md)
RULES_FLAGS = _lib.RF_DEFAULT

EpisodeStatus = namedtuple('EpisodeStatus', ['observation', 'reward', 'done'])


class TerminatedEpisodeStepException(BaseException):
    pass


class IlegalMoveException(BaseException):
    pass


with open(_lib.CODEC_PATH) as _fh:
    _MD = json.load(_fh)
MOVES_DICT = {True: _MD['w'], False: _MD['b']}                                                   # :16-18
MOVES_DICT_INV = {side: {v: k for k, v in MOVES_DICT[side].items()} for side in (True, False)}   # :19
NUM_ACTIONS = len(MOVES_DICT[True])                                                              # :20


# ---- packed-position helpers (C ABI, host side) ------------------------------------------------
def pos_from_fen(fen):
    out = np.zeros(5, np.uint32)
    _lib.check(_lib.lib().mtaz_pos_from_fen(fen.encode(), _lib.ptr(out, ctypes.c_uint32)))
    return out


def pos_to_fen(pos):
    pos = np.ascontiguousarray(pos, np.uint32)
    buf = ctypes.create_string_buffer(64)
    _lib.check(_lib.lib().mtaz_pos_to_fen(_lib.ptr(pos, ctypes.c_uint32), buf, 64))
    return buf.value.decode()


def pos_legal(pos, flags=None):
    pos = np.ascontiguousarray(pos, np.uint32)
    out = np.zeros(_lib.KMAX, np.uint16)
    k = _lib.check(_lib.lib().mtaz_pos_legal(_lib.ptr(pos, ctypes.c_uint32), RULES_FLAGS if flags is None else flags,
                                             _lib.ptr(out, ctypes.c_uint16), _lib.KMAX))
    return [int(x) for x in out[:k]]


def pos_outcome(pos, reps=1, flags=None, move_cap=None):
    pos = np.ascontiguousarray(pos, np.uint32)
    return _lib.check(_lib.lib().mtaz_pos_outcome(_lib.ptr(pos, ctypes.c_uint32), RULES_FLAGS if flags is None else flags,
                                                  MOVE_CAP if move_cap is None else move_cap, reps))


def pos_step(pos, code, flags=None):
    pos = np.ascontiguousarray(pos, np.uint32)
    out = np.zeros(5, np.uint32)
    _lib.check(_lib.lib().mtaz_pos_step(_lib.ptr(pos, ctypes.c_uint32), int(code), RULES_FLAGS if flags is None else flags,
                                        _lib.ptr(out, ctypes.c_uint32)))
    return out


def pos_encode(pos):
    pos = np.ascontiguousarray(pos, np.uint32)
    tok = np.zeros(60, np.uint8)
    clk = ctypes.c_float()
    _lib.check(_lib.lib().mtaz_pos_encode(_lib.ptr(pos, ctypes.c_uint32), _lib.ptr(tok, ctypes.c_uint8), ctypes.byref(clk)))
    return tok.astype(np.int64), np.float32(clk.value)


def pos_turn(pos):
    return bool(int(pos[4]) & 1)


def pos_half(pos):
    return (int(pos[4]) >> 8) & 0xff


def pos_full(pos):
    return int(pos[4]) >> 16


class MinitChessEpisode:
    """exp/environment.py:22-85 over the libmtaz rules (history kept for repetition)."""

    def __init__(self, fen):
        self._pos = pos_from_fen(fen)
        self._history = []          # (board+turn key, halfmove-after) of earlier positions
        self._reward = None
        self._done = None
        self._update_attributes()

    def _reps(self):
        key = self._pos[:4].tobytes() + bytes([int(self._pos[4]) & 1])
        h = pos_half(self._pos)
        n = 1
        for k in self._history[len(self._history) - h:] if h else []:
            if k == key:
                n += 1
        return n

    def _update_attributes(self):                                             # :34-50
        self._observation = pos_to_fen(self._pos)
        oc = pos_outcome(self._pos, self._reps())
        if oc == 1:
            self._reward, self._done = 1., True
        elif oc == 2:
            self._reward, self._done = 0., True
        else:
            self._done = False
        self._legal_moves = pos_legal(self._pos)

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
        return pos_turn(self._pos)

    @property
    def position(self):
        return self._pos.copy()

    def step(self, action, return_status=True):                               # :68-82
        if self.is_done():
            raise TerminatedEpisodeStepException
        nxt = pos_step(self._pos, int(action))          # raises IlegalMoveException
        self._history.append(self._pos[:4].tobytes() + bytes([int(self._pos[4]) & 1]))
        self._pos = nxt
        self._update_attributes()
        if return_status:
            return self.get_status()

    def get_status(self):
        return EpisodeStatus(self.get_observation(), self.get_reward(), self.is_done())


class MinitChessEnvironment:
    def new_episode(self, fen=None):                                           # :88-91
        episode = MinitChessEpisode(fen or STARTING_FEN)
        return episode, episode.get_observation()
