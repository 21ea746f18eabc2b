"""CPU: the N-rank launcher behind `python bench.py --gpus N` (minitchess_alphazero_amd.launch)."""
import os
import subprocess
import sys

from conftest import REPO

from minitchess_alphazero_amd.launch import spawn_ranks

GLOO_RANK = r'''
import os, sys, torch, torch.distributed as dist
dist.init_process_group('gloo')
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
assert t.item() == sum(range(1, dist.get_world_size() + 1)), t
assert os.environ['LOCAL_RANK'] == os.environ['RANK']
if dist.get_rank() == 0:
    open(sys.argv[1], 'w').write(os.environ['WORLD_SIZE'])
dist.destroy_process_group()
'''


def test_spawn_ranks_runs_a_gloo_world(tmp_path):
    out = tmp_path / 'w.txt'
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    env.pop('WORLD_SIZE', None)
    assert spawn_ranks(3, [sys.executable, '-c', GLOO_RANK, str(out)], env=env) == 0
    assert out.read_text() == '3'


def test_spawn_ranks_reports_a_failed_rank_and_stops_the_others():
    code = 'import os, sys, time\nif os.environ["RANK"] == "1": sys.exit(3)\ntime.sleep(120)'
    import time
    t0 = time.time()
    assert spawn_ranks(3, [sys.executable, '-c', code]) == 3
    assert time.time() - t0 < 60


def test_bench_rejects_a_world_size_that_differs_from_gpus():
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '2'], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert '--gpus 2' in r.stderr


def test_rank_host_share_splits_cores_and_threads():
    """Ranks on a node get disjoint core ranges covering the mask, and thread budgets that together
    stay within the usable CPUs (the smaller of the mask and the cgroup quota)."""
    from minitchess_alphazero_amd.launch import rank_host_share
    cores = list(range(16))
    slices = [rank_host_share(r, 8, cores=cores, quota=None) for r in range(8)]
    assert [s[1] for s in slices] == [2] * 8
    got = [c for s in slices for c in s[0]]
    assert got == cores
    # a 192-CPU mask under a 16-CPU quota: 24 cores each, 2 threads each
    big = [rank_host_share(r, 8, cores=list(range(192)), quota=16.0) for r in range(8)]
    assert all(len(c) == 24 and t == 2 for c, t in big)
    assert len({x for c, _ in big for x in c}) == 192
    # more ranks than cores: no pinning, one thread each
    assert rank_host_share(3, 8, cores=[0, 1, 2, 3], quota=None) == (None, 1)
    assert rank_host_share(0, 1, cores=cores, quota=None) == (cores, 16)
