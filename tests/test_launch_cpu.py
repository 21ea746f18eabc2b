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


def test_rank_host_share_follows_the_gpus_numa_nodes():
    """a rank is pinned to cores of its GPU's NUMA node, split among the ranks whose
    GPUs share that node; without usable topology the mask is split by rank index as before."""
    from minitchess_alphazero_amd.launch import rank_host_share
    cores = list(range(128))
    node_cpus = {0: list(range(0, 64)), 1: list(range(64, 128))}
    gpu_numa = [0, 0, 0, 0, 1, 1, 1, 1]
    got = [rank_host_share(r, 8, cores=cores, quota=16.0, gpu_numa=gpu_numa, node_cpus=node_cpus) for r in range(8)]
    assert got[0] == (list(range(0, 16)), 2)
    assert got[5] == (list(range(80, 96)), 2)
    assert all(set(c) <= set(node_cpus[gpu_numa[r]]) for r, (c, _) in enumerate(got))
    assert len({x for c, _ in got for x in c}) == 128
    # interleaved GPUs: ranks 0, 2, 4, 6 on node 1
    alt = [1, 0] * 4
    got = [rank_host_share(r, 8, cores=cores, quota=None, gpu_numa=alt, node_cpus=node_cpus)[0] for r in range(8)]
    assert got[0] == list(range(64, 80)) and got[1] == list(range(0, 16)) and got[6] == list(range(112, 128))
    # the mask holds only node 0's cores: node-1 ranks find none there and fall back to the index split
    half = list(range(64))
    assert rank_host_share(5, 8, cores=half, quota=None, gpu_numa=gpu_numa, node_cpus=node_cpus) == (list(range(40, 48)), 8)
    # unknown topology (-1, or no data): the index split
    assert rank_host_share(5, 8, cores=cores, gpu_numa=[-1] * 8, node_cpus=node_cpus, quota=None)[0] == list(range(80, 96))
    assert rank_host_share(2, 8, cores=cores, gpu_numa=[], node_cpus={}, quota=None)[0] == list(range(32, 48))


def test_topology_readers_parse_sysfs(tmp_path):
    from minitchess_alphazero_amd.launch import _cpulist, gpu_numa_nodes, numa_cpus
    assert _cpulist('0-3,8,10-11\n') == [0, 1, 2, 3, 8, 10, 11]
    node = tmp_path / 'node'
    for n, cl in ((0, '0-7'), (1, '8-15')):
        (node / f'node{n}').mkdir(parents=True)
        (node / f'node{n}' / 'cpulist').write_text(cl + '\n')
    assert numa_cpus(str(node)) == {0: list(range(8)), 1: list(range(8, 16))}
    kfd, pci = tmp_path / 'kfd', tmp_path / 'pci'
    # node 0: a CPU; nodes 1, 2: GPUs at 0000:c1:00.0 (NUMA 1) and 0000:05:00.0 (NUMA 0)
    for n, props in ((0, 'simd_count 0\n'), (1, f'simd_count 1216\nlocation_id {0xc1 << 8}\ndomain 0\n'),
                     (2, f'simd_count 1216\nlocation_id {0x05 << 8}\ndomain 0\n')):
        (kfd / str(n)).mkdir(parents=True)
        (kfd / str(n) / 'properties').write_text(props)
    for bdf, numa in (('0000:c1:00.0', 1), ('0000:05:00.0', 0)):
        (pci / bdf).mkdir(parents=True)
        (pci / bdf / 'numa_node').write_text(f'{numa}\n')
    os.environ.pop('ROCR_VISIBLE_DEVICES', None)
    os.environ.pop('HIP_VISIBLE_DEVICES', None)
    assert gpu_numa_nodes(str(kfd), str(pci)) == [1, 0]
    os.environ['HIP_VISIBLE_DEVICES'] = '1'
    try:
        assert gpu_numa_nodes(str(kfd), str(pci)) == [0]
    finally:
        del os.environ['HIP_VISIBLE_DEVICES']


def test_drm_fallback_orders_gpus_by_pci_address(tmp_path):
    """Without a KFD topology the AMD GPUs behind /sys/class/drm/card* count, in PCI address order."""
    from minitchess_alphazero_amd.launch import _drm_numa_nodes
    drm, pci = tmp_path / 'drm', tmp_path / 'pci'
    devs = {'0000:c1:00.0': ('0x1002', '0x120000', 1), '0000:05:00.0': ('0x1002', '0x038000', 0),
            '0000:07:00.0': ('0x8086', '0x030000', 0)}
    for bdf, (vendor, cls, numa) in devs.items():
        d = pci / bdf
        d.mkdir(parents=True)
        (d / 'vendor').write_text(vendor + '\n')
        (d / 'class').write_text(cls + '\n')
        (d / 'numa_node').write_text(f'{numa}\n')
    for i, bdf in enumerate(['0000:c1:00.0', '0000:05:00.0', '0000:07:00.0']):
        (drm / f'card{i}').mkdir(parents=True)
        os.symlink(pci / bdf, drm / f'card{i}' / 'device')
    (drm / 'renderD128').mkdir()
    assert _drm_numa_nodes(str(drm)) == [0, 1]
