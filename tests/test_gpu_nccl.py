"""GPU: the nccl (RCCL) code paths of bench.py and loop.py at world size 1, the only world the
one-GPU box allows: init_process_group('nccl', device_id=...), reduce_run on CUDA tensors, the
flat weight broadcast and records gather of the C5 loop (multi-GPU runs are the driver's)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_nccl_paths_at_world_one():
    from minitchess_alphazero_amd.launch import free_port
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0', LOCAL_WORLD_SIZE='1',
               MASTER_ADDR='127.0.0.1', MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, os.path.join(REPO, 'tests', 'rank_worker_nccl.py')], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out['backend'] == 'nccl' and out['world'] == 1
    assert out['reduce'] == [1.25, {'games': 3.0, 'sims': 7.0}]
    assert out['broadcast_equal'] is True
    assert out['loop_rows'] and out['loop_rows'] > 8
