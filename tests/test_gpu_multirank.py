"""GPU: the multi-GPU sharding contract at the engine level, world size 2.

Two ranks started the way bench.py --gpus N starts them (minitchess_alphazero_amd.launch), both on
cuda:0 of the one-GPU test box, gloo for the exchange: each plays its shard of global game ids
(Engine(seed_base = shard(rank, 2, G)[0])); the gathered episodes must equal ONE engine playing all
2G games, and reduce_run must give the max of the ranks' times and the sum of their counters."""
import json
import os
import sys

import pytest

from conftest import REPO
from helpers import compare_records

pytestmark = pytest.mark.gpu


def test_two_ranks_equal_one_engine(tmp_path):
    import torch
    from minitchess_alphazero_amd.engine import Engine
    from minitchess_alphazero_amd.launch import spawn_ranks
    from minitchess_alphazero_amd.network import Network
    G, sims = 6, 8
    out = str(tmp_path / 'ranks.json')
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    rc = spawn_ranks(2, [sys.executable, os.path.join(REPO, 'tests', 'rank_worker_engine.py'), out, str(G), str(sims)],
                     env=env)
    assert rc == 0
    res = json.load(open(out))
    one = Engine(n_games=2 * G, sims=sims, seed_base=0)
    torch.manual_seed(0)
    one.set_weights(Network())
    st = one.play()
    ref = one.episodes()
    assert len(res['episodes']) == 2 * G
    for g in range(2 * G):
        assert compare_records(res['episodes'][g], ref[g])[2] is None, g
        assert [r['reward'] for r in res['episodes'][g]] == [r['reward'] for r in ref[g]]
    assert res['seconds'] == 2.0
    for k in ('games', 'plies', 'sims', 'nn_evals', 'terminal_sims', 'decisive'):
        assert res['totals'][k] == st[k], k
