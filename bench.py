#!/usr/bin/env python3
"""Self-play throughput benchmark (BASELINE.json metric, config 2 / config 4).

A "step" = one complete self-play batch: every one of the G game slots on every
GPU plays a full episode from STARTING_FEN at `sims` MCTS simulations per move
(network, tree search, Dirichlet noise, action sampling all inside the timed
region).  value = games finished by all ranks / max-over-ranks wall time.

Launch: python bench.py [--gpus N --steps K --warmup W]
        N>1 under torch.distributed.run (one process per GPU, RANK/LOCAL_RANK/
        WORLD_SIZE from the env).  Games shard by global id: rank r plays seeds
        r*G .. r*G+G-1, no collective on the data path.
"""
import argparse
import json
import os
import sys
import time

T_START = time.time()                # the budget clock (--time-budget) starts with the process
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = 'self-play games/sec + MCTS sims/sec at 1/2/4/8 MI355X (fixed sims/move)'
FP32_MATRIX_PEAK_TFLOPS = 157.3      # MI355X_MICROARCH.md chip table (f32-input MFMA = f32 vector rate)
F16_MATRIX_PEAK_TFLOPS = 2500.0      # dense f16/bf16 MFMA (MI355X_MICROARCH.md; sparsity figures excluded)
HBM_PEAK_GBS = 8000.0                # MI355X_MICROARCH.md HBM peak
# the arithmetic of each network build and the nets its 1e-5 claim is tested on
PRECISION_NOTE = {
    1: ('f16x3: fp16 hi/lo split of weights and activations, three f16 MFMA passes (Wh*Xh + Wh*Xl + Wl*Xh), '
        'fp32 accumulate (k_net_y: off-board taps skipped, bitwise unchanged); priors and values within 1e-5 of '
        'the reference fp32 forward on the seed-0, C3, stress and stress4 nets (tests/test_gpu_search_parity.py, '
        'tests/test_gpu_stress.py)'),
    2: ('f16+e4m3: fp16 hi/lo split, Wh*Xh in f16, the cross terms in block-scaled e4m3, fp32 accumulate; priors '
        'and values within 1e-5 of the reference on the seed-0 and C3 nets, NOT on the stress net '
        '(tests/test_gpu_stress.py)'),
    0: 'fp32: fp32 MFMA trunk (k_conv3x3)',
}
TREE_BYTES_PER_SIM = 700             # SURVEY 8d algorithmic bytes per simulation of the tree walk


def elapsed():
    """Seconds since this process started (the driver's own clock starts a little earlier)."""
    return time.time() - T_START


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout)."""
    print(f'[bench] {msg}', file=sys.stderr, flush=True)


def _cpu_game(job):
    """One seeded game of the oracle's restatement of the app/puppet CPU path (batch-1 torch-CPU
    fp32 per leaf, FEN-keyed dict tables, Python rules) on `threads` torch threads."""
    sims, seed, threads = job[:3]
    if len(job) > 3 and job[3] is not None:
        os.sched_setaffinity(0, {job[3]})   # one core of its own (the 1-thread legs)
    import torch
    torch.set_num_threads(threads)
    from oracle.mcts import TorchNetEvaluator
    from oracle.net import seed0_network
    from oracle import selfplay
    ev = TorchNetEvaluator(seed0_network())
    st = {}
    selfplay.play_games(ev, 1, sims, seed_base=seed, stats=st)
    return {'seconds': st['seconds'], 'plies': st['plies'], 'nn_evals': st['nn_evals']}


def host_cores():
    """The host cores this process may use: os.cpu_count() (the whole machine), the affinity mask
    and the cgroup CPU quota (the GPU box grants a share of a larger host).  'usable' = the
    smaller of the last two: the thread count of the all-core CPU baseline."""
    n_os = os.cpu_count() or 1
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(n_os))
    quota = None
    try:
        q, period = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    usable = len(aff) if quota is None else max(1, min(len(aff), int(quota)))
    span = f'{aff[0]}-{aff[-1]}' if aff and aff[-1] - aff[0] + 1 == len(aff) else ','.join(map(str, aff))
    from minitchess_alphazero_amd.launch import gpu_numa_nodes, numa_cpus
    return {'os_cpu_count': n_os, 'affinity_count': len(aff), 'affinity': span, 'cgroup_quota_cpus': quota,
            'usable': usable, 'gpu_numa_nodes': gpu_numa_nodes(),
            'numa_nodes': {str(k): len(v) for k, v in sorted(numa_cpus().items())}}


def one_thread_jobs(gpu_sims, extra_sims=()):
    """The 1-thread legs of the full plan: every (sims, seed) game, one single-threaded process each."""
    seeds = [0, 1, 2]
    sims_list = sorted({32, gpu_sims, *extra_sims})
    return [(sm, sd, 1) for sm in sims_list for sd in seeds], sims_list, seeds


def start_one_thread_legs(gpu_sims, extra_sims=(), reserve=2):
    """Start the 1-thread legs asynchronously, BEFORE this process touches the GPU, so
    that they run during engine setup and the untimed warm-up steps and are collected before the
    timed region starts.  Each game runs in its own spawned process (never exec'ed over this one),
    pinned to its own core of this process's affinity mask, skipping the first `reserve` cores (the
    GPU rank's main thread and host threads).  Returns (pool, async result, meta)."""
    import multiprocessing as mp
    jobs, sims_list, seeds = one_thread_jobs(gpu_sims, extra_sims)
    cores = sorted(os.sched_getaffinity(0))
    free = cores[reserve:] if len(cores) > reserve + len(jobs) else cores
    jobs = [j + (free[i % len(free)] if len(free) >= len(jobs) else None,) for i, j in enumerate(jobs)]
    pool = mp.get_context('spawn').Pool(len(jobs))
    res = pool.map_async(_cpu_game, jobs, chunksize=1)
    meta = {'sims_list': sims_list, 'seeds': seeds, 'cores': [j[3] for j in jobs], 't_start': elapsed()}
    log(f'cpu baseline 1-thread legs started: {len(jobs)} games on cores {meta["cores"]}')
    return pool, res, meta


def cpu_baseline(plan, all_threads, gpu_sims, extra_sims=(), deadline=None, budget=None, one_thread=None):
    """seeded games (np.random.seed(g), random-init weights) at C1's 32 sims,
    the repo's default 36 (app/base.py:25) and the GPU's sims per move, each on all cores (games one
    after another, torch.set_num_threads = all_threads) and on 1 thread (all single-thread games at
    once, one process each: every game still runs alone on one core).  Children are separate
    processes (spawned, never exec'ed over this one) and touch no GPU; nothing else runs meanwhile.
    value = games/s at the GPU's sims on all cores.

    The legs run in priority order, each only when its estimate (scaled from the first leg's
    seconds per game) ends before `deadline` (s since process start): the GPU's sims on all cores
    (the value), the other sims on all cores, then the 1-thread legs (all at once).  Skipped legs
    are named in budget['skipped'], never silently dropped."""
    import multiprocessing as mp
    # all-core legs: 2 seeded games each at the GPU's sims, the repo default 36 and C1's 32 (VERDICT r5
    # #6: all three inside the driver's budget); the 1-thread legs (run during the warm-up) keep 3
    seeds = [0, 1] if plan == 'full' else [0]
    others = sorted({32, *extra_sims} - {gpu_sims}, reverse=True) if plan == 'full' else sorted(set(extra_sims) - {gpu_sims})
    sims_list = sorted({gpu_sims, *others})
    ctx = mp.get_context('spawn')
    runs = {}
    skipped = budget['skipped'] if budget is not None else []

    def record(sims, label, thr, games, sds=None):
        secs = [g['seconds'] for g in games]
        log(f'cpu baseline {sims} sims, {thr} thread(s): {[round(x, 1) for x in secs]} s per game')
        runs[f'{sims}sims/{label}'] = {
            'threads': thr, 'seeds': sds or seeds, 'seconds_per_game': [round(x, 3) for x in secs],
            'games_per_s': len(secs) / sum(secs), 'plies': [g['plies'] for g in games],
            'nn_evals': [g['nn_evals'] for g in games],
            'sims_per_s': sum(g['plies'] for g in games) * sims / sum(secs)}

    def fits(label, est):
        if deadline is None or elapsed() + est <= deadline:
            return True
        skipped.append({'leg': f'cpu baseline {label}', 'estimate_s': round(est, 1)})
        log(f'BUDGET: skipping cpu baseline {label} (~{est:.0f} s; {elapsed():.0f} s used of {deadline:.0f} s)')
        return False

    def all_cores(sims):
        with ctx.Pool(1) as pool:
            record(sims, 'all', all_threads, pool.map(_cpu_game, [(sims, sd, all_threads) for sd in seeds], chunksize=1))

    # the value leg: the GPU's sims on all cores (its own estimate: ~0.35 s per sim per game on 16
    # cores, measured rounds 1-3)
    if not fits(f'{gpu_sims} sims all cores', len(seeds) * 0.35 * gpu_sims * 16 / max(1, all_threads) + 5):
        return None
    all_cores(gpu_sims)
    per_sim = sum(runs[f'{gpu_sims}sims/all']['seconds_per_game']) / len(seeds) / gpu_sims   # s per game per sim
    for sims in others:
        if fits(f'{sims} sims all cores', len(seeds) * per_sim * sims * 1.25 + 5):
            all_cores(sims)
    if plan == 'full' and one_thread is not None:
        # measured during the warm-up steps (start_one_thread_legs)
        for sm in one_thread['sims_list']:
            record(sm, '1thread', 1, one_thread['games'][sm], one_thread['seeds'])
    elif plan == 'full':
        # 1 thread: every (sims, seed) game at once, one single-threaded process each (each game alone
        # on its core; measured at ~2.4x the all-core seconds per game)
        if fits('1-thread legs', per_sim * max(sims_list) * 2.6 * 1.2 + 8):
            seeds1 = [0, 1, 2]
            jobs = [(sm, sd, 1) for sm in sims_list for sd in seeds1]
            with ctx.Pool(len(jobs)) as pool:
                out = pool.map(_cpu_game, jobs, chunksize=1)
            for i, sm in enumerate(sims_list):
                record(sm, '1thread', 1, out[i * len(seeds1):(i + 1) * len(seeds1)], seeds1)
    head = runs[f'{gpu_sims}sims/all']
    sample = (f'{len(seeds)} seeded games (np.random.seed 0..{len(seeds) - 1}) from STARTING_FEN at '
              f'{gpu_sims} sims/move on {all_threads} threads: the oracle restatement of app/puppet '
              f'(batch-1 torch CPU fp32, dict tables, Python rules); value = games / total seconds')
    if one_thread is not None:
        sample += (f'.  The 1-thread runs ({", ".join(map(str, one_thread["sims_list"]))} sims x seeds '
                   f'{one_thread["seeds"]}, one process per game pinned to cores {one_thread["cores"]}) ran '
                   f'during the untimed engine setup and warm-up steps ({one_thread["overlap"]}), concurrently '
                   f'with each other and with the GPU rank (whose host threads were limited to '
                   f'{one_thread["gpu_host_threads"]} meanwhile), never during the timed region')
    return {'value': head['games_per_s'], 'unit': 'games/s', 'cores': all_threads, 'kind': 'port',
            'sample': sample, 'sims_per_s': head['sims_per_s'], 'runs': runs}


# the reference's own self-play games a benched engine's games 0.. must reproduce (seeds 0..n-1 =
# np.random.seed(g) games, seed-0 net or the C3 checkpoint): sims -> (fixture, key, weights)
PARITY_FIXTURES = {
    (64, None): ('trees_r2.json', 'net_seed0_64'),     # tests/golden/make_golden_r2.py
    (36, None): ('trees_r6.json', 'net_seed0_36'),     # tests/golden/make_golden_r6.py
    (32, None): ('trees.json', 'net_seed0'),           # tests/golden/make_golden.py
    (256, 'c3'): ('c3.json', 'c3_256'),                # BASELINE config 3 (make_golden_r2.py)
}


def parity_stamp(engine, sims, weights_kind, seed_base):
    """After a timed play (untimed): the engine's games 0.. against the reference's games of the same
    seeds, ply for ply (observation, legal list, pi, action, reward); a plain JSON compare.  None
    when no fixture covers this workload."""
    fx = PARITY_FIXTURES.get((sims, weights_kind))
    if fx is None or seed_base != 0:
        return None
    games = json.load(open(os.path.join(HERE, 'tests', 'golden', fx[0])))[fx[1]]
    if engine.G < len(games):
        return None
    got = engine.episodes(len(games))
    ident = plies = 0
    first = None
    for g, ref in enumerate(games):
        assert ref['seed'] == g
        plies += max(len(ref['moves']), len(got[g]))
        for i, (a, b) in enumerate(zip(got[g], ref['moves'])):
            if (a['observation'] == b['observation'] and a['legal_moves'] == b['legal_moves'] and a['pi'] == b['pi']
                    and a['action'] == b['action'] and a['reward'] == b['reward']):
                ident += 1
            elif first is None:
                first = {'game': g, 'ply': i}
    return {'fixture': f'tests/golden/{fx[0]}:{fx[1]}', 'games': [g['seed'] for g in games], 'identical_plies': ident,
            'plies': plies, 'first_mismatch': first, 'ok': ident == plies}


def kernel_roofline(tot, prec):
    """Roofline of the dominant kernel from the engine's HIP events (one record per network launch).
      f16x3 (default): k_net_y, the fused network with all three split products on f16 MFMA (16x16x32);
      f16f8: k_net_z, the same network with the fp16 split's two cross terms on the block-scaled
        e4m3 MFMA (16x16x128);
        both: ONE network launch per simulation wave = the whole network on the wave's leaves (the
        full-round kernel and its three tail kernels, k_net_*<NVB = 4> then <1..3>, between the two
        events); algorithmic FLOP per launch = leaves x 638,245,892, peak = the dense
        f16 MFMA rate;
      fp32: k_conv3x3, 18 launches per wave; FLOP per launch = leaves x 2*30*256*2304."""
    from minitchess_alphazero_amd.engine import FLOP_PER_CONV_BOARD, FLOP_PER_EVAL
    if prec in (1, 2):
        launches = tot['waves']
        flop_per_launch = FLOP_PER_EVAL * tot['trunk_boards'] / tot['waves'] if launches else float('nan')
        kernel, peak = ('k_net_y (fused network, fp16x3 on MFMA 16x16x32 f16, class tiles: 57 of 72 tile-taps '
                        'run)'), F16_MATRIX_PEAK_TFLOPS
        if prec == 2:
            kernel = ('k_net_z (fused network: Wh*Xh on MFMA 16x16x32 f16, cross terms on the block-scaled '
                      'e4m3 MFMA 16x16x128)')
    else:
        launches = 18 * tot['waves']
        flop_per_launch = FLOP_PER_CONV_BOARD * tot['trunk_boards'] / tot['waves'] if launches else float('nan')
        kernel, peak = 'k_conv3x3 (fp32 MFMA 32x32x2)', FP32_MATRIX_PEAK_TFLOPS
    # issued MFMA work in dense-f16 equivalents: f16x3 runs 3 passes on 57 of the 72 tile-taps of each
    # conv (the skipped ones multiply zeros; the stem and heads, 0.2% of the FLOP, run every tap)
    passes_eq = {1: 3.0 * 57 / 72, 2: 2.0}.get(prec, 1.0)
    ms = tot['trunk_ms'] / launches if launches else float('nan')
    achieved = flop_per_launch / (ms * 1e-3) / 1e12
    return {'bound': 'mfma', 'kernel': kernel, 'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s',
            'frac': achieved / peak, 'avg_launch_ms': ms, 'flop_per_launch': flop_per_launch,
            'mfma_passes': {1: 'f16 x3 on 57 of 72 tile-taps', 2: 'f16 x1 + e4m3 x2'}.get(prec, 'f32 x1'),
            # the MFMA work the split actually issues, in dense-f16 equivalents (an e4m3 MFMA of the
            # block-scaled form runs at twice the f16 rate: 3 passes for f16x3, 1 + 2/2 for
            # f16+e4m3), over the same dense f16 peak: the MFMA pipes' utilisation
            'issued_achieved': achieved * passes_eq, 'issued_frac': achieved * passes_eq / peak,
            'issued_note': ('pass factor of the main launch (f16x3: 3 x 57/72 tile-taps) applied to every board: '
                            'the 1- and 2-board tail instances run all 72 tile-taps and the 3-board one 49 of 54, '
                            'so issued_* slightly understate the issued MFMA work (ADVICE r4)') if prec == 1 else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=1)
    ap.add_argument('--warmup', type=int, default=0)
    ap.add_argument('--games', type=int, default=4096, help='parallel games per GPU (BASELINE config 2: 4096)')
    ap.add_argument('--sims', type=int, default=64, help='MCTS simulations per move (config 2: 64)')
    ap.add_argument('--precision', default='f16x3', choices=['f16x3', 'f16f8', 'fp32'],
                    help='network build: f16x3 = k_net_y (default; within 1e-5 of fp32 on every tested net), '
                         'f16f8 = k_net_z (faster; within 1e-5 on the seed-0 and C3 nets only), fp32')
    ap.add_argument('--groups', type=int, default=1, help='game groups on separate HIP streams (mtaz_set_pipeline)')
    ap.add_argument('--net-variant', type=int, default=0, help='parity-tested network build (Engine.set_net_variant)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-threads', type=int, default=0)
    ap.add_argument('--cpu-plan', default='full', choices=['full', 'quick'],
                    help='full: BASELINE.md section 4 (3 seeded games x {32, --sims} sims x {all cores, 1 thread}); '
                         'quick: 1 game at --sims on all cores')
    ap.add_argument('--secondary', action='store_true',
                    help='one more timed step with the other fused network (k_net_z when the main line runs '
                         'k_net_y): an A/B outside the 1e-5 contract on the stress net, off by default')
    ap.add_argument('--no-secondary', action='store_true', help=argparse.SUPPRESS)   # (the default now)
    ap.add_argument('--host-threads', type=int, default=0,
                    help="host threads of the engine's per-move work (Dirichlet draws, action choice); 0 = this "
                         "rank's share of the usable cores (launch.rank_host_share), at most 16")
    ap.add_argument('--time-budget', type=float, default=float(os.environ.get('MTAZ_BENCH_BUDGET_S', 500)),
                    help='wall-clock budget in s from process start (the driver kills the run at 600 s): the '
                         'timed steps must fit (else exit 3 with a message before timing); the optional legs '
                         '(36-sims step, CPU baseline runs) are skipped, and named in the JSON, when they '
                         'would not')
    ap.add_argument('--default-sims', type=int, default=36,
                    help="one more timed step at the repo's default sims per move (app/base.py:25: 36; 0 = skip), "
                         'reported with its CPU baseline as at_repo_default_sims')
    ap.add_argument('--memo', type=int, default=2, choices=[0, 1, 2],
                    help='leaf memo: 2 = per game + batch (default), 1 = per game, 0 = evaluate every leaf '
                         '(results identical in every mode)')
    ap.add_argument('--traffic-json', default=os.path.join(HERE, 'profiles', 'conv_traffic.json'))
    ap.add_argument('--weights', default='', help='state_dict file (safetensors or torch.save) instead of random '
                                                  'init (BASELINE config 3: tests/golden/c3/c3.safetensors)')
    ap.add_argument('--dist-backend', default='nccl', choices=['nccl', 'gloo'],
                    help='N>1 end-of-run reductions: nccl (RCCL, one GPU per rank) or gloo (host; with '
                         '--device, a rehearsal of the N-rank path on one GPU)')
    ap.add_argument('--device', type=int, default=None, help='GPU of this rank (default LOCAL_RANK)')
    ap.add_argument('--rank-share', type=int, default=0,
                    help='run this one process at the host share one of N ranks on the node gets '
                         '(launch.rank_host_share: usable CPUs / N): before anything touches the GPU, pin '
                         'to that many cores of the affinity mask and use that many host threads '
                         '(VERDICT r4 #2: the 8-rank host share measured on a 1-GPU box)')
    ap.add_argument('--sync-mode', type=int, default=-1, choices=[-1, 0, 1],
                    help='how the engine waits for its stream: 0 = hipStreamSynchronize, 1 = blocking-sync '
                         'event (Engine.set_sync_mode); -1 (default) = 1 when this rank has a share of a '
                         'multi-rank node (N > 1 or --rank-share), else 0 (profiles/r05/hostshare: +2.1%% '
                         'at the 2-CPU share, neutral at 16)')
    ap.add_argument('--defer', type=int, default=2, choices=[0, 1, 2],
                    help='deferred tails (Engine.set_defer): 2 (default, round 6) = a wave evaluates its whole '
                         'rounds of 4 boards x CUs and the rest of its leaves wait for the next wave; 1 = only a '
                         'remainder a tail launch would take waits (round 5); 0 = every leaf every wave (round 4). '
                         'Results are identical (profiles/r06/sched2)')
    ap.add_argument('--one-thread-during-warmup', type=int, default=1, choices=[0, 1],
                    help='1 (default): run the CPU baseline 1-thread legs during engine setup and the '
                         'untimed warm-up steps (collected before the timed region); 0: after the timed '
                         'steps, budget permitting')
    args = ap.parse_args()

    # N ranks: under torch.distributed.run WORLD_SIZE must equal --gpus; without a launcher this
    # process starts the N ranks itself (before anything here touches the GPU) and exits with their code
    from minitchess_alphazero_amd.launch import main_or_spawn
    if os.environ.get('WORLD_SIZE') is None and args.gpus > 1:
        from minitchess_alphazero_amd.build import build
        build(verbose=False)                  # once for all ranks (hipcc only, no GPU call)
    world = main_or_spawn(args.gpus, __file__)

    rank = int(os.environ.get('RANK', 0))
    local = int(os.environ.get('LOCAL_RANK', 0))
    node_mask = sorted(os.sched_getaffinity(0))   # before this rank pins itself to its slice
    # this rank's disjoint slice of the host cores and its host-thread budget (launch.rank_host_share)
    from minitchess_alphazero_amd.launch import pin_rank, rank_host_share
    rank_share = None
    if args.rank_share > 1:
        # one rank's share of an N-rank node, emulated in this single process before any thread or GPU
        # context exists: `threads` CPUs (usable // N) as the affinity mask and the thread budget
        cores_all = sorted(os.sched_getaffinity(0))
        _, thr = rank_host_share(0, args.rank_share)
        os.sched_setaffinity(0, cores_all[:thr])
        host_threads = thr
        rank_share = {'ranks': args.rank_share, 'cores': cores_all[:thr], 'threads': thr}
        log(f'rank share of {args.rank_share}: affinity {cores_all[:thr]}, {thr} host threads')
    else:
        host_threads = pin_rank(local, int(os.environ.get('LOCAL_WORLD_SIZE', world)))
    # the CPU baseline's 1-thread legs run during setup and warm-up (rank 0 of a 1-GPU run), started
    # before this process touches the GPU
    legs = None
    legs_mask = None
    if (world == 1 and not args.no_cpu_baseline and args.cpu_plan == 'full' and args.one_thread_during_warmup
            and rank_share is None):
        extra = (args.default_sims,) if args.default_sims and args.default_sims != args.sims else ()
        legs = start_one_thread_legs(args.sims, extra)
        # while the legs run, this process (its main thread, the HIP runtime's threads and the engine's
        # host threads, all started after this point) stays on the reserved cores the legs skip, so
        # that it does not slow the legs it is compared with
        legs_mask = sorted(os.sched_getaffinity(0))
        leg_cores = legs[2]['cores']
        reserved = [c for c in legs_mask if c not in set(leg_cores)][:2] if None not in leg_cores else []
        if reserved:
            os.sched_setaffinity(0, reserved)
            legs[2]['gpu_process_cores'] = reserved
    import numpy as np
    import torch
    torch.set_num_threads(host_threads)
    dist = None
    device = local if args.device is None else args.device
    red_device = torch.device('cuda', device)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(device)
        if args.dist_backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', device))
        else:
            dist.init_process_group('gloo')
            red_device = torch.device('cpu')

    from minitchess_alphazero_amd.build import build
    if rank == 0 or world == 1:
        build(verbose=False)
    if dist is not None:
        dist.barrier()
    from minitchess_alphazero_amd.engine import Engine, FLOP_PER_EVAL, start_position
    from minitchess_alphazero_amd.network import Network

    from minitchess_alphazero_amd.sharding import reduce_run, shard
    G, sims = args.games, args.sims
    seed_base, _ = shard(rank, world, G)
    eng = Engine(n_games=G, sims=sims, device=device, seed_base=seed_base)
    weights_sha = None
    weights_kind = None if not args.weights else 'other'   # None: the seed-0 random init
    if args.weights:
        import hashlib
        if args.weights.endswith('.safetensors'):
            from safetensors.torch import load_file
            sd = load_file(args.weights)
        else:
            sd = torch.load(args.weights, map_location='cpu', weights_only=True)
        net_for_engine = Network()
        net_for_engine.load_state_dict(sd)
        h = hashlib.sha256()                      # over the state_dict in module order (tests/golden/c3.json)
        for k, v in net_for_engine.state_dict().items():
            h.update(k.encode())
            h.update(v.detach().cpu().contiguous().numpy().tobytes())
        weights_sha = h.hexdigest()
        try:
            if weights_sha == json.load(open(os.path.join(HERE, 'tests', 'golden', 'c3.json')))['state_dict_sha256']:
                weights_kind = 'c3'
        except (OSError, KeyError, ValueError):
            pass
    else:
        torch.manual_seed(0)                      # random-init weights of the reference architecture
        net_for_engine = Network()
    eng_threads = args.host_threads or min(16, host_threads)
    eng.set_weights(net_for_engine)
    eng.set_memo(args.memo)
    eng.set_host_threads(eng_threads)
    eng.set_precision(args.precision)
    eng.set_net_variant(args.net_variant)
    eng.set_timing(True)
    eng.set_pipeline(args.groups)
    sync_mode = args.sync_mode if args.sync_mode >= 0 else int(world > 1 or rank_share is not None)
    eng.set_sync_mode(sync_mode)
    eng.set_defer(args.defer)
    eng.evaluate(np.stack([start_position()] * 8))    # load code objects before timing
    LEG_HOST_THREADS = 2
    if legs is not None:
        eng.set_host_threads(min(eng_threads, LEG_HOST_THREADS))   # leave the cores to the 1-thread legs

    def agree_max(x):
        """The max of x over ranks (budget decisions must be the same on every rank)."""
        if dist is None:
            return float(x)
        t = torch.tensor([float(x)], dtype=torch.float64, device=red_device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    warm_s = []
    for i in range(args.warmup):
        t0 = time.perf_counter()
        eng.play()
        warm_s.append(time.perf_counter() - t0)
        log(f'warmup {i + 1}/{args.warmup}: {warm_s[-1]:.2f} s')
    budget = {'limit_s': args.time_budget, 'skipped': []}
    one_thread = None
    if legs is not None:
        pool, res, meta = legs
        t_wait = elapsed()
        out = res.get()
        pool.close()
        pool.join()
        os.sched_setaffinity(0, legs_mask)   # (threads started from here on get the whole mask)
        eng.set_host_threads(eng_threads)
        waited = elapsed() - t_wait
        per = len(meta['seeds'])
        one_thread = {**meta, 'games': {sm: out[i * per:(i + 1) * per] for i, sm in enumerate(meta['sims_list'])},
                      'gpu_host_threads': LEG_HOST_THREADS, 'gpu_process_cores': meta.get('gpu_process_cores'),
                      'overlap': (f'{args.warmup} warm-up step(s); started at {meta["t_start"]:.1f} s, the timed '
                                  f'region waited {waited:.1f} s more for them')}
        budget['one_thread_legs_wait_s'] = round(waited, 1)
        log(f'cpu baseline 1-thread legs done (waited {waited:.1f} s after the warm-up)')
    if warm_s:
        # the timed steps are the contract: if they cannot fit the budget, say so and stop before
        # timing rather than being killed without a line
        step_est = agree_max(sum(warm_s[1:] or warm_s) / len(warm_s[1:] or warm_s))
        need = elapsed() + args.steps * step_est
        budget['main_projected_end_s'] = round(need, 1)
        if need > args.time_budget:
            log(f'BUDGET: {args.steps} steps of ~{step_est:.1f} s would end at {need:.0f} s, past the '
                f'{args.time_budget:.0f} s budget (--time-budget); stopping before the timed region')
            if dist is not None:
                dist.destroy_process_group()
            sys.exit(3)

    def sync():
        torch.cuda.synchronize(device)
        if dist is not None:
            dist.barrier()

    KEYS = ('sims', 'nn_evals', 'memo_hits', 'memo_batch_hits', 'plies', 'trunk_ms', 'trunk_boards', 'waves', 'terminal_sims',
            'decisive', 'host_rng_ms', 'sync_ms', 'select_ms', 'compact_ms', 'choice_ms', 'gap_ms', 'extra_waves', 'moves',
            'rng_dev_ms', 'rng_device')

    import resource

    def cpu_s():
        r = resource.getrusage(resource.RUSAGE_SELF)
        return r.ru_utime + r.ru_stime

    def timed(engine, steps, label):
        """`steps` full self-play batches between barrier + synchronize; max wall over ranks and
        summed counters (sharding.reduce_run).  tot['host_cpu_ms']: this process's CPU time (every
        thread, user + system) over the region, summed over ranks."""
        tot = {k: 0.0 for k in KEYS}
        sync()
        c0 = cpu_s()
        t0 = time.perf_counter()
        for i in range(steps):
            st = engine.play()
            for k in tot:
                tot[k] += st[k]
            if rank == 0:
                log(f'{label} step {i + 1}/{steps}: {st["wall_ms"] / 1e3:.2f} s')
        sync()
        dt = time.perf_counter() - t0
        tot['host_cpu_ms'] = (cpu_s() - c0) * 1e3
        dt, tot = reduce_run(dt, tot, dist, red_device)
        return dt, tot, int(st.get('net_precision', 0))

    def counters(tot, dt, games):
        ref_evals = tot['nn_evals'] + tot['memo_hits']
        return {'sims_per_s': tot['sims'] / dt, 'plies_per_game': tot['plies'] / games,
                # network evaluations: computed on the GPU, supplied by the per-game leaf memo, and their
                # sum = the reference's evaluations (one per non-terminal expansion, exp/agent.py:64-71)
                'nn_evals_per_game': tot['nn_evals'] / games, 'memo_hits_per_game': tot['memo_hits'] / games,
                'nn_evals_reference_per_game': ref_evals / games,
                'memo_hit_frac': tot['memo_hits'] / ref_evals if ref_evals else 0.0,
                'memo_batch_hit_frac': tot['memo_batch_hits'] / ref_evals if ref_evals else 0.0,
                'nn_evals_per_s': tot['nn_evals'] / dt, 'nn_evals_reference_per_s': ref_evals / dt,
                'terminal_sims_per_game': tot['terminal_sims'] / games, 'decisive_games': int(tot['decisive']),
                'nn_tflops_algorithmic': tot['nn_evals'] * FLOP_PER_EVAL / dt / 1e12,
                # simulation waves (one network launch each) and, with deferred tails, the waves that
                # ended moves for the games whose leaves had waited
                'waves': int(tot['waves']), 'extra_waves': int(tot['extra_waves'])}

    dt, tot, prec = timed(eng, args.steps, 'main')
    games = G * args.steps * world
    step_s = dt / args.steps
    # untimed: the last timed play's games 0.. against the reference's games of the same seeds
    parity = parity_stamp(eng, sims, weights_kind, seed_base) if rank == 0 else None
    if parity is not None:
        log(f'parity vs {parity["fixture"]}: {parity["identical_plies"]}/{parity["plies"]} plies identical')

    def fits(label, est_s):
        """True when an optional leg of ~est_s seconds ends inside the budget (same answer on every
        rank); otherwise it is named in the JSON line's budget.skipped."""
        ok = agree_max(elapsed() + est_s) <= args.time_budget
        if not ok:
            budget['skipped'].append({'leg': label, 'estimate_s': round(est_s, 1)})
            log(f'BUDGET: skipping {label} (~{est_s:.0f} s; {elapsed():.0f} s of {args.time_budget:.0f} s used)')
        return ok

    # the north_star's measurement point: the repo's default sims per move (app/base.py:25), same
    # games, seeds, weights and precision as the main line
    at_default = None
    if args.default_sims and args.default_sims != sims and fits(f'{args.default_sims}-sims step',
                                                                 step_s * args.default_sims / sims * 1.15 + 5):
        eng36 = Engine(n_games=G, sims=args.default_sims, device=device, seed_base=seed_base)
        eng36.set_weights(net_for_engine)
        eng36.set_precision(args.precision)
        eng36.set_net_variant(args.net_variant)
        eng36.set_timing(True)
        eng36.set_pipeline(args.groups)
        eng36.set_memo(args.memo)
        eng36.set_host_threads(eng_threads)
        eng36.set_sync_mode(sync_mode)
        eng36.set_defer(args.defer)
        eng36.evaluate(np.stack([start_position()] * 8))
        # a second step when it and the CPU legs still to come end inside the budget by cpu_baseline's
        # own estimates (the value leg at 0.35 s per sim per game on 16 cores, the others 1.25x that),
        # so that the step never costs a CPU leg (the 36-sims point for at least 2
        # steps if the budget allows; at the driver's --steps 20 it does not: profiles/r05/final2)
        cpu_rest = 0.0
        if world == 1 and not args.no_cpu_baseline:
            # the all-core legs still to come (cpu_baseline: 2 seeds each at the GPU's sims, 36 and 32 in
            # the full plan): 0.32 s per sim per game on 16 cores (round 6: 0.317 at 64, 36 and 32 sims),
            # plus the legs' process starts
            n_seeds = 2 if args.cpu_plan == 'full' else 1
            others = (args.default_sims + 32) if args.cpu_plan == 'full' else args.default_sims
            cpu_rest = n_seeds * 0.32 * (sims + others) * 16 / max(1, host_cores()['usable']) + 10
        step36 = step_s * args.default_sims / sims * 1.15
        n36 = 3
        while n36 > 1 and agree_max(elapsed() + n36 * step36 + 5 + cpu_rest) > args.time_budget:
            n36 -= 1
        if n36 < 3:
            budget['skipped'].append({'leg': f'{args.default_sims}-sims steps {n36 + 1}..3', 'estimate_s': round(step36, 1)})
        dt3, tot3, prec3 = timed(eng36, n36, f'{args.default_sims} sims')
        at_default = {'sims_per_move': args.default_sims, 'value': G * world * n36 / dt3, 'unit': 'games/s', 'steps': n36,
                      'ms_per_step': dt3 * 1e3 / n36, 'roofline': kernel_roofline(tot3, prec3),
                      **counters(tot3, dt3, G * world * n36)}
        if rank == 0:
            at_default['parity'] = parity_stamp(eng36, args.default_sims, weights_kind, seed_base)
        eng36.close()

    # secondary line (opt-in, --secondary): one more timed step on the other fused network (k_net_z,
    # f16f8, when the main line runs k_net_y), same engine, seeds and workload.  k_net_z's tested scope
    # is narrower: within 1e-5 on the seed-0 and C3 nets, not on the stress net
    secondary = None
    other = {'f16x3': 'f16f8', 'f16f8': 'f16x3'}.get(args.precision)
    if args.secondary and other and fits(f'secondary ({other})', step_s + 5):
        eng.set_precision(other)
        eng.evaluate(np.stack([start_position()] * 8))    # load the other build's code objects
        dt2, tot2, prec2 = timed(eng, 1, f'secondary ({other})')
        eng.set_precision(args.precision)
        secondary = {'precision': PRECISION_NOTE[prec2], 'value': G * world / dt2, 'unit': 'games/s', 'steps': 1,
                     'ms_per_step': dt2 * 1e3, 'roofline': kernel_roofline(tot2, prec2), **counters(tot2, dt2, G * world)}
    # N > 1: rank 0 runs the CPU baseline after the timed region on the node's usable
    # cores while the other ranks wait idle at a barrier
    cb_multi = None
    if world > 1 and not args.no_cpu_baseline:
        if rank == 0:
            mask = sorted(os.sched_getaffinity(0))
            os.sched_setaffinity(0, node_mask)   # the spawned games get the node's cores, not rank 0's slice
            try:
                hc = host_cores()
                extra = (args.default_sims,) if args.default_sims and args.default_sims != sims else ()
                cb_multi = cpu_baseline('quick', args.cpu_threads or hc['usable'], sims, extra,
                                        deadline=args.time_budget, budget=budget)
                if cb_multi is not None:
                    cb_multi['sample'] += (f'; run by rank 0 after the timed region while the other {world - 1} '
                                           f'rank(s) waited idle')
            finally:
                os.sched_setaffinity(0, mask)
        dist.barrier()
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    roof = kernel_roofline(tot, prec)
    # traffic: HBM/fabric bytes per launch from the PMC passes (tools/gpu.sh pmc -> tools/pmc_summary.py
    # -> profiles/conv_traffic.json), attached only when those passes ran THIS library (the file's
    # mtaz_src_sha256 stamp equals the loaded library's source hash) on this workload; else null, with
    # the reason in traffic_source (a kernel change without a new PMC pass must not
    # carry a stale figure)
    from minitchess_alphazero_amd import _lib
    lib_hash = _lib.lib().mtaz_version().decode().rsplit('mtaz-src-sha256=', 1)[-1]
    traffic, why = None, f'no {os.path.relpath(args.traffic_json, HERE)}'
    if os.path.exists(args.traffic_json):
        try:
            tj = json.load(open(args.traffic_json))
            if tj.get('mtaz_src_sha256') != lib_hash:
                why = (f'stale: PMC passes of library {str(tj.get("mtaz_src_sha256"))[:16]}, running '
                       f'{lib_hash[:16]}')
            elif not (tj.get('games') == args.games and tj.get('sims') == args.sims
                      and roof['kernel'].startswith(tj.get('kernel', '?'))):
                why = f'PMC passes of another workload ({tj.get("games")} games, {tj.get("sims")} sims, {tj.get("kernel")})'
            else:
                traffic = tj.get('hbm_bytes_per_launch')
                why = (f'{os.path.relpath(args.traffic_json, HERE)}: PMC passes of this library '
                       f'({lib_hash[:16]}) on this workload')
        except Exception as e:
            why = f'unreadable: {e}'
    roof['traffic'] = traffic
    roof['traffic_source'] = why
    line = {
        'metric': METRIC,
        'value': games / dt,
        'unit': 'games/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': dt * 1e3 / args.steps,
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': PRECISION_NOTE[prec],
        'data': ('synthetic: self-play from STARTING_FEN, random-init weights (torch.manual_seed(0); Network())'
                 if not args.weights else f'synthetic: self-play from STARTING_FEN, trained checkpoint sha256 {weights_sha}'),
        'config': {'workload': (f'{G} parallel self-play games per GPU, {sims} sims/move, random-init policy net '
                                f'(BASELINE config 2; config 4 = 8 GPUs x 4096)') if not args.weights else
                               (f'{G} parallel self-play games per GPU, {sims} sims/move, trained checkpoint '
                                f'(BASELINE config 3)'),
                   'games_per_gpu': G, 'sims_per_move': sims, 'parallelism': f'games sharded over {world} GPU(s)'},
        **counters(tot, dt, games),
        'roofline': roof,
        # secondary roofline: the tree kernel k_select, HBM/latency-bound; algorithmic
        # bytes per simulation = SURVEY's estimate (path nodes: header + k edge reads + edge update,
        # leaf insert, hash probe, NN input) at k ~ 7.5, depth ~ 2
        'roofline_tree': {'bound': 'hbm', 'kernel': 'k_select', 'bytes_per_sim': TREE_BYTES_PER_SIM,
                          'achieved': tot['sims'] * TREE_BYTES_PER_SIM / (tot['select_ms'] * 1e-3) / 1e9
                          if tot['select_ms'] > 0 else None,
                          'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                          'frac': tot['sims'] * TREE_BYTES_PER_SIM / (tot['select_ms'] * 1e-3) / 1e9 / HBM_PEAK_GBS
                          if tot['select_ms'] > 0 else None,
                          'avg_launch_ms': tot['select_ms'] / tot['waves'] if tot['waves'] else None,
                          'share_of_wall': tot['select_ms'] / 1e3 / dt,
                          # k_leaf_compact (the leaf list in game order, one workgroup) follows every
                          # k_select launch; its time is outside the k_select roofline
                          'leaf_compact_avg_ms': tot['compact_ms'] / tot['waves'] if tot['waves'] else None},
        'host_threads': eng_threads,
        # numpy's legacy RNG (Dirichlet root noise, action choice): on the device (k_noise, k_choose;
        # rng_device_s = their kernel time over the timed steps, summed over ranks) or on the host
        'rng_device': bool(tot['rng_device']),
        'rng_device_s': tot['rng_dev_ms'] / 1e3,
        'host_rng_s': tot['host_rng_ms'] / 1e3,
        'host_sync_s': tot['sync_ms'] / 1e3,
        # host time between two moves' simulations (the GPU idles): action choice + records
        # (host_choice_s), apply, game states, move start, the first Dirichlet draws
        'host_gap_s': tot['gap_ms'] / 1e3,
        'host_choice_s': tot['choice_ms'] / 1e3,
        # CPU time of this rank's process over the timed region (all threads): host_cpus_busy = the
        # CPUs it keeps busy on average, against its share of the node (launch.rank_host_share)
        'host_cpu_s': tot['host_cpu_ms'] / 1e3 / world,
        'host_cpus_busy': tot['host_cpu_ms'] / 1e3 / world / dt,
        'sync_mode': sync_mode,
        'defer': args.defer,
        'mtaz_src_sha256': lib_hash,
    }
    if parity is not None:
        line['parity'] = parity
    if rank_share is not None:
        line['rank_share'] = rank_share
    if secondary is not None:
        line['secondary'] = secondary
    if at_default is not None:
        line['at_repo_default_sims'] = at_default
    line['host_cores'] = host_cores()
    if world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or line['host_cores']['usable']
        extra = (args.default_sims,) if args.default_sims and args.default_sims != sims else ()
        cb = cpu_baseline(args.cpu_plan, threads, sims, extra, deadline=args.time_budget, budget=budget,
                          one_thread=one_thread)
        if cb is not None:
            line['cpu_baseline'] = cb
            line['vs_cpu_baseline'] = line['value'] / cb['value']
            r36 = cb['runs'].get(f'{args.default_sims}sims/all')
            if at_default is not None and r36 is not None:
                at_default['cpu_baseline_games_per_s'] = r36['games_per_s']
                at_default['cpu_baseline_sims_per_s'] = r36['sims_per_s']
                at_default['vs_cpu_baseline'] = at_default['value'] / r36['games_per_s']
    if cb_multi is not None:
        line['cpu_baseline'] = cb_multi
        line['vs_cpu_baseline'] = line['value'] / cb_multi['value']
    budget['end_s'] = round(elapsed(), 1)
    line['budget'] = budget
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    bad = [p for p in (parity, (at_default or {}).get('parity')) if p is not None and not p['ok']]
    if bad:
        log(f'PARITY MISMATCH: {bad}')
        sys.exit(5)


if __name__ == '__main__':
    main()
