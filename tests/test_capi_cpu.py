"""C-ABI library checks that need no GPU: it loads, exports every symbol declared in
include/mtaz.h, and its HOST-side functions (rules, FEN, encoder, numpy-legacy RNG)
agree with the oracle / numpy.  No device compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO, load_golden

from minitchess_alphazero_amd import _lib
from minitchess_alphazero_amd import environment as env


def _declared_symbols():
    src = open(os.path.join(REPO, 'include', 'mtaz.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(mtaz_[a-z_0-9]+)\s*\(', src)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = _declared_symbols()
    assert len(syms) >= 40
    for s in syms:
        assert hasattr(L, s), s
        assert s in _lib.SIGNATURES, f'{s} missing from the ctypes signature table'
    assert L.mtaz_abi_version() == 2


def test_library_carries_the_tree_fingerprint():
    """The loaded library was built from these sources (build.py source_hash is compiled into
    mtaz_version); a library from other sources is refused."""
    from minitchess_alphazero_amd import build
    ver = _lib.lib().mtaz_version().decode()
    assert ver.endswith('mtaz-src-sha256=' + build.source_hash())
    assert build.embedded_hash(_lib.LIB_PATH) == build.source_hash()
    with pytest.raises(_lib.MtazLibraryError):
        _lib.check_fingerprint(ver[:-64] + '0' * 64)


def test_codec_file_matches_reference_hash():
    import hashlib
    g = load_golden('codec')
    assert hashlib.sha256(open(_lib.CODEC_PATH, 'rb').read()).hexdigest() == g['sha256']


def test_host_rules_match_oracle_env_fixtures():
    g = load_golden('env')
    for row in g['positions']:
        ep = env.MinitChessEpisode(row['fen'])
        assert ep.get_observation() == row['fen']
        assert ep.get_legal_moves() == row['legal'], row['fen']
        assert ep.is_done() == row['done'] and ep.get_reward() == row['reward'] and ep.turn == row['turn']
    for row in g['steps']:
        ep = env.MinitChessEpisode(row['fen'])
        st = ep.step(row['code'])
        assert (st.observation, st.reward, st.done) == (row['next'], row['reward'], row['done'])


def test_host_encoder_matches_reference():
    for row in load_golden('encoder'):
        tok, clk = env.pos_encode(env.pos_from_fen(row['fen']))
        assert tok.tolist() == row['tokens'] and float(clk) == row['clock'], row['fen']


def test_host_rules_random_games_vs_oracle():
    """Random walks with repetition / promotions: host libmtaz episode == oracle episode."""
    from oracle import environment as oenv
    rs = np.random.RandomState(7)
    for game in range(40):
        a = env.MinitChessEpisode(env.STARTING_FEN)
        b = oenv.MinitChessEpisode(oenv.STARTING_FEN)
        while True:
            assert a.get_observation() == b.get_observation()
            assert a.get_legal_moves() == b.get_legal_moves()
            assert (a.is_done(), a.get_reward()) == (b.is_done(), b.get_reward())
            if a.is_done():
                break
            lm = a.get_legal_moves()
            # bias towards shuffling moves so repetition draws occur
            code = lm[rs.randint(len(lm))] if rs.rand() < 0.7 else lm[0]
            a.step(code)
            b.step(code)


def test_exceptions_are_base_exceptions():
    ep = env.MinitChessEpisode(env.STARTING_FEN)
    with pytest.raises(env.IlegalMoveException):
        ep.step(0)
    assert not issubclass(env.IlegalMoveException, Exception)
    done = env.MinitChessEpisode('k4/1QK2/5/5/5/5 b 1 5')
    assert done.is_done() and done.get_reward() == 1.0
    with pytest.raises(env.TerminatedEpisodeStepException):
        done.step(0)


def test_host_rng_matches_numpy_legacy():
    L = _lib.lib()
    st = ctypes.create_string_buffer(L.mtaz_rng_state_size())
    for row in load_golden('rng'):
        L.mtaz_rng_seed(st, row['seed'])
        for op in row['ops']:
            if op['op'] == 'dirichlet':
                out = np.zeros(op['k'], np.float64)
                L.mtaz_rng_dirichlet(st, 0.6, op['k'], _lib.ptr(out, ctypes.c_double))
                assert out.tolist() == op['out']
            elif op['op'] == 'choice_p':
                p = np.asarray(op['p'], np.float64)
                assert 100 + L.mtaz_rng_choice_p(st, _lib.ptr(p, ctypes.c_double), len(p)) == op['out']
            else:
                assert L.mtaz_rng_randint(st, op['m']) == op['out']


def test_host_rng_long_streams_vs_numpy():
    L = _lib.lib()
    st = ctypes.create_string_buffer(L.mtaz_rng_state_size())
    for seed in (0, 1, 12345, 2**32 - 1):
        rs = np.random.RandomState(seed)
        L.mtaz_rng_seed(st, seed)
        for j in range(400):
            k = 1 + j % 23
            ref = rs.dirichlet([0.6] * k)
            out = np.zeros(k, np.float64)
            L.mtaz_rng_dirichlet(st, 0.6, k, _lib.ptr(out, ctypes.c_double))
            assert np.array_equal(out, ref), (seed, j)
            m = 1 + j % 7
            assert L.mtaz_rng_randint(st, m) == rs.choice(np.arange(m))
        for alpha in (0.3, 1.0, 2.5):
            ref = rs.dirichlet([alpha] * 5)
            out = np.zeros(5, np.float64)
            L.mtaz_rng_dirichlet(st, alpha, 5, _lib.ptr(out, ctypes.c_double))
            assert np.array_equal(out, ref), (seed, alpha)


def test_arena_winner_rule_cpu():
    """WinnerRecorder (exp/callbacks.py:19-22): the agent that made the last move of a decisive
    game wins; agent 0 moves first; draws are not counted."""
    import numpy as np
    from minitchess_alphazero_amd.arena import gate, winners
    rec = {'plies': np.array([1, 2, 7, 10, 5]), 'outcome': np.array([1, 1, 1, 2, 1])}
    assert winners(rec) == {False: 3, True: 1}
    assert gate(0.56) and not gate(0.55)
