"""GPU: the driver's form `python bench.py --gpus N` end to end, N = 2 and 8 on the one-GPU box.

bench.py starts its own ranks (minitchess_alphazero_amd.launch), both placed on cuda:0 with
--device 0 and gloo for the final reduction (RCCL needs one GPU per rank).  The JSON line must
report n_gpus 2, both ranks' games in the whole-job value, and the usual roofline fields."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n', [2, 8])
def test_bench_gpus_n_launches_its_ranks(n):
    """N = 8 is BASELINE config 4's rank count (32,768 games on 8 GPUs) in miniature: eight ranks of
    32 games on the one GPU, each pinned to its share of the box's cores.  At N = 8 the line must also
    carry the CPU baseline (rank 0 runs it after the timed region while the other ranks wait; VERDICT
    r5 #7) and the 36-sims step's parity stamp (rank 0's games 0-3 = the reference's 36-sim games)."""
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    cmd = [sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', str(n), '--device', '0', '--dist-backend', 'gloo',
           '--games', '32', '--sims', '8', '--steps', '1', '--warmup', '0']
    if n != 8:
        cmd.append('--no-cpu-baseline')
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d['n_gpus'] == n and d['scaling'] == 'weak'
    assert d['config']['games_per_gpu'] == 32
    # whole-job value: every rank's games over the max of the ranks' times
    assert abs(d['value'] - 32 * n / (d['ms_per_step'] / 1e3)) <= 1e-6 * d['value']
    assert d['roofline']['avg_launch_ms'] > 0 and d['roofline_tree']['avg_launch_ms'] > 0
    if n == 8:
        cb = d['cpu_baseline']
        assert cb['value'] > 0 and cb['cores'] >= 1 and 'rank 0 after the timed region' in cb['sample']
        assert d['vs_cpu_baseline'] == d['value'] / cb['value']
        par = d['at_repo_default_sims']['parity']
        assert par['ok'] and par['identical_plies'] == par['plies'] > 0, par
        assert d['rng_device'] is True
