"""CPU oracle for the MinitChess AlphaZero self-play hot path.

TEST INFRASTRUCTURE ONLY.  Nothing in the shipped package
(`minitchess_alphazero_amd/`) imports this directory.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may use it, and
only as the checker / the reported CPU baseline, never as the measured path.

Contents (each function cites the reference file:line it restates):
  rules.py   - python-chess-compatible MinitChess rules (the reference's rules
               live in the un-vendored python-chess "minitchess" fork; the
               rule CONTENT is a build decision documented in RULES.md, so the
               rules themselves are "parity unpinned"; how they are consumed
               is pinned by exp/environment.py:34-82).
  codec.py   - the 554-code action space (exp/generate_moves_list.py:5-57),
               pinned byte-for-byte against exp/moves_dict.json.
  encoder.py - FEN -> tokens/clock (exp/policy.py:82-105), pinned by golden
               vectors produced by importing the reference.
  net.py     - the ResNet (exp/policy.py:15-80), same parameter creation
               order, so torch.manual_seed(0) reproduces the reference weights.
  mcts.py    - MCTS / agent / referee / policy (exp/agent.py, exp/policy.py:
               107-125), with numpy-1 / numpy-2 casting modes.
  selfplay.py- the app/puppet episode loop + InfoRecorder records
               (app/base.py:108-124, exp/callbacks.py:31-62).

Parity pinning: tests/golden/make_golden.py imports the reference's own
exp/*.py (with stub erlyx modules and oracle.rules as `chess`) in the build
container and commits its outputs as fixtures; tests check this oracle
against those fixtures.
"""
