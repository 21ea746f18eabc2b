"""One process per GPU without an external launcher.

`python bench.py --gpus N` (the driver's form) must run N ranks even when nothing like
torch.distributed.run started it.  spawn_ranks() starts N children of the same command line with
the launcher's environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT) and waits for
them.  The parent never initialises HIP: it must be called before anything in the calling process
touches the GPU (no torch.cuda call, no engine), and it starts the children as new processes
(subprocess), never by replacing itself.  This module imports no torch.
"""
import os
import socket
import subprocess
import sys
import time


def free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv, env=None, poll_s=0.2):
    """Run `argv` as ranks 0..n-1 (children inherit stdout/stderr) and return the exit code: 0 if
    every rank exits 0, else the first non-zero code seen.  When a rank fails, the others are
    terminated (then killed after 30 s) so that no rank waits forever in a collective."""
    if n < 1:
        raise ValueError(f'need at least one rank, got {n}')
    base = dict(os.environ if env is None else env)
    base.setdefault('MASTER_ADDR', '127.0.0.1')
    base['MASTER_PORT'] = str(free_port())
    base['WORLD_SIZE'] = str(n)
    base['LOCAL_WORLD_SIZE'] = str(n)
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen(list(argv), env=e))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(poll_s)
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
                deadline = time.time() + 30
                for q in live:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
    return rc


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 quota (None: unlimited or unknown)."""
    try:
        q, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        return None if q == 'max' else float(q) / float(period)
    except (OSError, ValueError):
        return None


def _cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]"""
    out = []
    for part in text.strip().split(','):
        if part:
            lo, _, hi = part.partition('-')
            out += range(int(lo), int(hi or lo) + 1)
    return out


def numa_cpus(root='/sys/devices/system/node'):
    """NUMA node -> its CPUs ({} when the kernel exposes no NUMA topology)."""
    out = {}
    try:
        for name in os.listdir(root):
            if name.startswith('node') and name[4:].isdigit():
                with open(os.path.join(root, name, 'cpulist')) as f:
                    out[int(name[4:])] = _cpulist(f.read())
    except OSError:
        return {}
    return out


def _drm_numa_nodes(drm='/sys/class/drm'):
    """Fallback without a KFD topology: the AMD display / accelerator PCI functions behind
    /sys/class/drm/card*, in PCI address order (the order HIP enumerates them by default), with
    their numa_node."""
    found = {}
    try:
        for name in os.listdir(drm):
            if not (name.startswith('card') and name[4:].isdigit()):
                continue
            dev = os.path.realpath(os.path.join(drm, name, 'device'))
            try:
                with open(os.path.join(dev, 'vendor')) as f:
                    vendor = f.read().strip()
                with open(os.path.join(dev, 'class')) as f:
                    cls = f.read().strip()
                with open(os.path.join(dev, 'numa_node')) as f:
                    numa = int(f.read())
            except (OSError, ValueError):
                continue
            if vendor == '0x1002' and (cls.startswith('0x03') or cls.startswith('0x12')):
                found[os.path.basename(dev)] = numa
    except OSError:
        return []
    return [found[b] for b in sorted(found)]


def gpu_numa_nodes(kfd='/sys/class/kfd/kfd/topology/nodes', pci='/sys/bus/pci/devices'):
    """HIP device index -> the NUMA node of its PCI function (-1 unknown), [] when unavailable.  The
    KFD topology lists the GPU nodes (simd_count > 0) in the order of the HSA agents HIP enumerates;
    each node's location_id is its PCI bus << 8 | devfn.  Without a KFD topology, the AMD GPUs
    behind /sys/class/drm in PCI address order.  ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES
    of plain indices select and reorder them as the runtime does."""
    gpus = []
    if not os.path.isdir(kfd):
        gpus = _drm_numa_nodes()
    try:
        for n in sorted((x for x in os.listdir(kfd) if x.isdigit()), key=int) if not gpus else []:
            props = {}
            with open(os.path.join(kfd, n, 'properties')) as f:
                for line in f:
                    kv = line.split()
                    if len(kv) == 2:
                        props[kv[0]] = kv[1]
            if int(props.get('simd_count', 0)) == 0:
                continue
            loc, dom = int(props.get('location_id', 0)), int(props.get('domain', 0))
            bdf = f'{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7:x}'
            try:
                with open(os.path.join(pci, bdf, 'numa_node')) as f:
                    gpus.append(int(f.read()))
            except (OSError, ValueError):
                gpus.append(-1)
    except OSError:
        return []
    for var in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES'):
        sel = os.environ.get(var)
        if sel:
            try:
                gpus = [gpus[int(i)] for i in sel.split(',')]
            except (ValueError, IndexError):
                return []
    return gpus


def rank_host_share(local_rank, local_world, cores=None, quota=None, gpu_numa=None, node_cpus=None):
    """This rank's slice of the host: its usable CPUs (the smaller of the mask and the cgroup quota)
    split into equal thread budgets, so N ranks of host work (torch, the engine's host threads) do
    not oversubscribe the cores the node grants, and a disjoint range of the affinity mask to pin to.
    With the NUMA topology known (gpu_numa[d] = NUMA node of HIP device d, the rank's device being
    its local rank; node_cpus[node] = that node's CPUs), the range comes from the mask's cores on its
    GPU's NUMA node, split among the ranks whose GPUs sit on that node; otherwise
    the whole mask is split by rank index.  -> (cores, threads); cores is None when there are fewer
    cores than ranks to share them (no pinning then)."""
    if cores is None:
        cores = sorted(os.sched_getaffinity(0))
    if quota is None:
        quota = cgroup_cpu_quota()
    usable = len(cores) if quota is None else max(1, min(len(cores), int(quota)))
    threads = max(1, usable // max(1, local_world))
    if gpu_numa and node_cpus and len(gpu_numa) >= local_world and gpu_numa[local_rank] in node_cpus:
        node = gpu_numa[local_rank]
        local = sorted(set(cores) & set(node_cpus[node]))
        peers = [r for r in range(local_world) if gpu_numa[r] == node]
        per = len(local) // len(peers)
        if per >= 1:
            i = peers.index(local_rank)
            return local[i * per:(i + 1) * per], threads
    per = len(cores) // max(1, local_world)
    mine = cores[local_rank * per:(local_rank + 1) * per] if per >= 1 else None
    return mine, threads


def pin_rank(local_rank, local_world):
    """Apply rank_host_share to this process (before it starts threads), with the node's NUMA
    topology when the kernel exposes it; returns the thread budget."""
    mine, threads = rank_host_share(local_rank, local_world, gpu_numa=gpu_numa_nodes(), node_cpus=numa_cpus())
    if mine and local_world > 1:
        os.sched_setaffinity(0, mine)
    return threads


def main_or_spawn(n_requested, script):
    """For a script started as `python script ... --gpus N`: returns the world size this process
    belongs to, after checking it against N, or (with no launcher and N > 1) runs N ranks of the
    same command line and exits with their code."""
    world_env = os.environ.get('WORLD_SIZE')
    if world_env is None and n_requested > 1:
        sys.exit(spawn_ranks(n_requested, [sys.executable, os.path.abspath(script)] + sys.argv[1:]))
    world = int(world_env or 1)
    if world != n_requested:
        sys.stderr.write(f'{os.path.basename(script)}: --gpus {n_requested} but the launcher started '
                         f'{world} rank(s) (WORLD_SIZE)\n')
        sys.exit(2)
    return world
