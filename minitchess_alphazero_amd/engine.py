"""The batched MI355X self-play engine (Python side of include/mtaz.h).

One Engine per GPU.  It owns `n_games` game slots, two MCTS transposition tables
per slot (the two SimpleAlphaZeroAgents of app/base.py:113), one numpy-legacy
MT19937 per slot (seeded seed_base + slot) and the packed network.

    eng = Engine(n_games=4096, sims=64, device=0)
    eng.set_weights(Network())          # torch.manual_seed(0) for the bench weights
    stats = eng.play()                  # full self-play of every slot
    episodes = eng.episodes()           # InfoRecorder-format records (exp/callbacks.py:40-54)

The fine-grained methods (set_games / move_begin / set_noise / simulate /
sim_select / leaves / sim_backup / move_end / apply / tree) expose one MCTS move
at a time; tests drive them with a host evaluator to pin the tree bit-for-bit
against the CPU oracle.
"""
import ctypes
from ctypes import c_double, c_float, c_int32, c_int64, c_uint8, c_uint16, c_uint32, c_void_p

import numpy as np

from . import _lib
from .environment import MOVE_CAP, RULES_FLAGS, STARTING_FEN, pos_from_fen, pos_to_fen

STAT_NAMES = ['plies', 'sims', 'nn_evals', 'terminal_sims', 'trunk_ms', 'trunk_boards', 'waves', 'host_rng_ms',
              'wall_ms', 'games', 'decisive', 'moves', 'trunk_launches', 'max_nodes', 'max_edges', 'sync_ms', 'net_precision',
              'select_ms', 'node_cap', 'edge_cap', 'compact_ms', 'memo_hits', 'pool_edges', 'pool_cap',
              'memo_batch_hits', 'choice_ms', 'gap_ms', 'extra_waves', 'rng_device', 'rng_dev_ms',
              'schedule']

# algorithmic work of one leaf evaluation: 319,122,946 MAC
FLOP_PER_EVAL = 638_245_892
# one trunk conv on one board: 30 positions x 256 out x 2304 K, 2 FLOP/MAC
FLOP_PER_CONV_BOARD = 2 * 30 * 256 * 2304


def _p(a, t):
    return _lib.ptr(a, t)


class Engine:
    # the network build mtaz_create selects: k_net_y, within 1e-5 of fp32 on every tested net
    DEFAULT_PRECISION = 'f16x3'

    def __init__(self, n_games, sims, device=0, cpuct=1, tau_change=6, dir_alpha=0.6, dir_eps=0.25, seed_base=0,
                 cast_mode=2, rules_flags=RULES_FLAGS, move_cap=MOVE_CAP):
        self.L = _lib.lib()
        self.G, self.sims, self.device = int(n_games), int(sims), int(device)
        self.cpuct = cpuct
        h = self.L.mtaz_create(self.device, self.G, self.sims, float(cpuct), int(tau_change), float(dir_alpha),
                               float(dir_eps), int(seed_base), int(cast_mode), int(rules_flags), int(move_cap))
        if not h:
            raise _lib.MtazError(_lib.E_DEVICE, self.L.mtaz_last_error().decode())
        self.h = c_void_p(h)
        self._weights_alive = None

    def close(self):
        if getattr(self, 'h', None):
            self.L.mtaz_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- weights / evaluation ---------------------------------------------------------------
    def set_weights(self, network_or_state_dict, slot=0):
        """SimulatePuppet.load_weights (app/base.py:126-129); BN folded on upload.  slot 1 holds
        a second network for two-network play (set_agent_networks)."""
        import torch
        from .network import weight_tensors
        dev = torch.device('cuda', self.device)
        ts = [t.detach().to(dev, torch.float32).contiguous() for t in weight_tensors(network_or_state_dict)]
        torch.cuda.synchronize(dev)
        ptrs = (c_void_p * len(ts))(*[t.data_ptr() for t in ts])
        numels = np.array([t.numel() for t in ts], np.int64)
        _lib.check(self.L.mtaz_set_weights_slot(self.h, int(slot), ptrs, _p(numels, c_int64), len(ts)))

    def set_agent_networks(self, slot_agent0=0, slot_agent1=0):
        """Which weight slot agent 0 (moves first) and agent 1 search with; (0, 0) = self-play."""
        _lib.check(self.L.mtaz_set_agent_slots(self.h, int(slot_agent0), int(slot_agent1)))

    def evaluate(self, positions):
        """Network.forward on packed positions [n,5] -> (logits [n,554], values [n]) (numpy)."""
        import torch
        dev = torch.device('cuda', self.device)
        pos = torch.from_numpy(np.ascontiguousarray(positions, np.uint32).view(np.int32)).to(dev)
        n = pos.shape[0]
        logits = torch.empty((n, 554), dtype=torch.float32, device=dev)
        values = torch.empty((n,), dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)
        _lib.check(self.L.mtaz_evaluate(self.h, c_void_p(pos.data_ptr()), n, c_void_p(logits.data_ptr()),
                                        c_void_p(values.data_ptr())))
        return logits.cpu().numpy(), values.cpu().numpy()

    def net_exponents(self, positions):
        """k_net_y's stored-units exponents on packed positions [n,5], from one launch of the
        stamp-instrumented build (mtaz_net_time, 4 boards per workgroup): (largest exponent [n],
        bit mask of the layers whose exponent is nonzero [n]; bit 0 = stem, 1 + L = conv L)."""
        import torch
        dev = torch.device('cuda', self.device)
        pos = torch.from_numpy(np.ascontiguousarray(positions, np.uint32).view(np.int32)).to(dev)
        n = pos.shape[0]
        nwg = (n + 3) // 4
        st = np.zeros(nwg * 10, np.uint64)
        ms = ctypes.c_float()
        torch.cuda.synchronize(dev)
        _lib.check(self.L.mtaz_net_time(self.h, c_void_p(pos.data_ptr()), n, 1, 1, ctypes.byref(ms),
                                        st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
        rec = st[nwg * 6:].reshape(-1)[:n]
        return (rec >> np.uint64(32)).astype(np.int64), (rec & np.uint64(0xffffffff)).astype(np.int64)

    # ---- batched self-play -----------------------------------------------------------------------
    def set_precision(self, precision):
        """'f16x3' (default, k_net_y: fp16 hi/lo split, three f16 MFMA passes, fp32-accurate to ~1e-7;
        within 1e-5 of the reference on every tested net), 'f16f8' (k_net_z: the split's cross
        terms on the block-scaled e4m3 MFMA, 1.4x faster; within 1e-5 on the seed-0 and C3 nets,
        NOT on the round-3 stress net: tests/test_gpu_stress.py; one exponent per workgroup, so past
        2^14 a play with the memo on fails with 'f16f8-range-with-memo') or 'fp32' (fp32 MFMA)."""
        _lib.check(self.L.mtaz_set_precision(self.h, {'fp32': 0, 'f16x3': 1, 'f16f8': 2}[precision]))

    def set_net_variant(self, variant):
        """Select a parity-tested build of the current precision's network kernel (0 = product;
        set_precision resets it).  f16x3 (k_net_y): 1 = 4 boards per workgroup in every round (no
        tail launch), 2 = the class tiles without the off-board tap skip, both bitwise equal to 0;
        5 = the product with the first round-4 tail instances
        (off-board cells on the padding squares, 2-way LDS bank conflicts; weights one k-block
        ahead; bitwise equal to 0).  f16f8 (k_net_z): 1 = 4 boards per workgroup in every
        round (no tail launches), 2097152 = the epilogue in unfused form, 8192 = e2m3 (fp6) cross
        terms, 25165824 = the round-2 K loop (per-step fragment addresses, 64-bit weight addresses),
        33554432 = the round-2 epilogue (unscaled conversions), 58720256 = both (the round-2
        product); all but 8192 bitwise equal to 0.  Other values are rejected; the A/B and
        timing-only diagnostic builds, and round 3's k_net_y (f16x3 variant 3: one stored-units
        exponent per workgroup, batch-dependent past 2^14), exist only in libmtaz_diag.so
        (MTAZ_LIB, tools/bench_net.py --diag, tests/diag_round3.py)."""
        _lib.check(self.L.mtaz_set_net_variant(self.h, int(variant)))

    def set_pipeline(self, groups):
        """play() over `groups` independent game groups on their own HIP streams (1 = off).
        Results are identical for any group count (games keep their global seeds)."""
        _lib.check(self.L.mtaz_set_pipeline(self.h, int(groups)))

    def set_memo(self, mode=1):
        """Leaf memo: 1 (default, or True) = a position the game's other agent already expanded
        takes its legal list, priors and value from that agent's table instead of the network;
        2 = also positions any game of the batch evaluated earlier in the play; 0 (False) = off.
        Results unchanged (include/mtaz.h mtaz_set_memo).  stats()['nn_evals'] counts the
        evaluations computed, 'memo_hits' the ones the memo supplied ('memo_batch_hits' of them from
        the batch memo); evaluations + hits is the reference's count."""
        _lib.check(self.L.mtaz_set_memo(self.h, int(mode)))

    def set_edge_capacity(self, per_tree, pool):
        """Edge storage: `per_tree` edges in each table's own region plus a pool of `pool` edges
        shared by the tables that outgrow theirs (include/mtaz.h mtaz_set_edge_capacity).  Clears
        every table."""
        _lib.check(self.L.mtaz_set_edge_capacity(self.h, int(per_tree), int(pool)))

    def set_host_threads(self, n=0):
        """Host threads of the per-move work (0 = the process's affinity mask, at most 16)."""
        _lib.check(self.L.mtaz_set_host_threads(self.h, int(n)))

    def set_defer(self, mode=2):
        """Deferred tails in play() (2, the default since round 6): a simulation wave evaluates only
        its whole rounds of 4 boards x CUs; the rest stay pending for the next wave, whose list puts
        the least advanced games first (a game selects again only after its leaf's backup, so its
        simulations run in order, exactly as in lockstep), and each move ends with the waves its
        lagging games still need.  1 = only a remainder a tail launch would take (at most 3 boards
        per CU) waits, a larger one runs as a partial round (round 5's default); 0 = every leaf every
        wave (the round-4 schedule).  With round 6's leaf order mode 2 is 1-2% faster than mode 1
        (profiles/r06/sched2).  Results are identical in every mode."""
        _lib.check(self.L.mtaz_set_defer(self.h, int(mode)))

    def set_lag_order(self, order=0):
        """Deferred-tail play's leaf order: 0 (default) = the least advanced games first (the
        leaders wait), 1 = round 5's order (lag behind the most advanced leaf).  Games are identical;
        only the waves a move needs change."""
        _lib.check(self.L.mtaz_set_lag_order(self.h, int(order)))

    def set_rng_device(self, on=1):
        """Where play() runs numpy's legacy RNG (the root Dirichlet noise of exp/agent.py:82 and the
        action choice of :114-118): 1 (default) = on the device (per-game MT19937 state in HBM, one
        k_noise and one k_choose launch per move), 0 = on the host.  Games are identical."""
        _lib.check(self.L.mtaz_set_rng_device(self.h, int(on)))

    def set_schedule(self, mode=1):
        """play()'s schedule: 0 (default) = moves in lockstep, 1 = free-running moves (a game that
        completes a move finishes it and starts the next on the device while the others keep
        simulating).  Games are identical; free-running needs the device RNG and one network."""
        _lib.check(self.L.mtaz_set_schedule(self.h, int(mode)))

    def wave_log(self, max_waves=1 << 17):
        """Per-wave log of the last play(): int32 [waves, 3] = (leaves evaluated, game-memo hits,
        batch-memo hits)."""
        out = np.zeros((max_waves, 3), np.int32)
        n = _lib.check(self.L.mtaz_wave_log(self.h, _p(out, c_int32), int(max_waves)))
        return out[:n]

    def set_sync_mode(self, mode=0):
        """How the host thread waits for the engine's stream: 0 = hipStreamSynchronize (default),
        1 = a blocking-sync event (the thread sleeps instead of holding a CPU).  Results unchanged."""
        _lib.check(self.L.mtaz_set_sync_mode(self.h, int(mode)))

    def set_seed_base(self, seed_base):
        """Game slot g of the next play() uses np.random.seed(seed_base + g) semantics."""
        _lib.check(self.L.mtaz_set_seed_base(self.h, int(seed_base)))

    def set_timing(self, on=True):
        self.L.mtaz_set_timing(self.h, 1 if on else 0)

    def play(self, n_games=None, from_current=False):
        n = self.G if n_games is None else int(n_games)
        _lib.check(self.L.mtaz_play(self.h, n, 1 if from_current else 0))
        self._n_played = n
        return self.stats()

    def stats(self):
        out = np.zeros(len(STAT_NAMES), np.float64)
        self.L.mtaz_stats(self.h, _p(out, c_double), len(STAT_NAMES))
        return dict(zip(STAT_NAMES, out.tolist()))

    def records(self):
        """Raw per-ply arrays of the last play(): dict of numpy arrays."""
        n = self._n_played
        plies = np.zeros(n, np.int32)
        tp, te = c_int64(), c_int64()
        _lib.check(self.L.mtaz_records_counts(self.h, _p(plies, c_int32), ctypes.byref(tp), ctypes.byref(te)))
        P, E = tp.value, te.value
        pos = np.zeros((max(P, 1), 5), np.uint32)
        action = np.zeros(max(P, 1), np.int32)
        k = np.zeros(max(P, 1), np.int32)
        codes = np.zeros(max(E, 1), np.uint16)
        visits = np.zeros(max(E, 1), np.uint32)
        reward = np.zeros(max(P, 1), np.float32)
        outcome = np.zeros(n, np.int32)
        _lib.check(self.L.mtaz_records_get(self.h, _p(pos, c_uint32), _p(action, c_int32), _p(k, c_int32),
                                           _p(codes, c_uint16), _p(visits, c_uint32), _p(reward, ctypes.c_float),
                                           _p(outcome, c_int32)))
        return {'plies': plies, 'pos': pos[:P], 'action': action[:P], 'k': k[:P], 'codes': codes[:E],
                'visits': visits[:E], 'reward': reward[:P], 'outcome': outcome}

    def episodes(self, n_games=None):
        """InfoRecorder records (exp/callbacks.py:40-54), one list of dicts per game (the first
        n_games games only, if given)."""
        r = self.records()
        out, p, e = [], 0, 0
        for g in range(len(r['plies']) if n_games is None else min(int(n_games), len(r['plies']))):
            ep = []
            for _ in range(int(r['plies'][g])):
                k = int(r['k'][p])
                N = r['visits'][e:e + k].astype(np.float64)
                ep.append({'observation': pos_to_fen(r['pos'][p]),
                           'legal_moves': [int(c) for c in r['codes'][e:e + k]],
                           'pi': (N / N.sum()).tolist(),
                           'action': int(r['action'][p]),
                           'reward': float(r['reward'][p])})
                p += 1
                e += k
            out.append(ep)
        return out

    # ---- fine-grained search ---------------------------------------------------------------------
    def set_games(self, fens_or_positions, agents=None, active=None):
        pos = np.zeros((self.G, 5), np.uint32)
        n = len(fens_or_positions)
        for i, x in enumerate(fens_or_positions):
            pos[i] = pos_from_fen(x) if isinstance(x, str) else np.asarray(x, np.uint32)
        ag = np.zeros(self.G, np.int32)
        if agents is not None:
            ag[:n] = agents
        act = np.zeros(self.G, np.uint8)
        act[:n] = 1 if active is None else np.asarray(active, np.uint8)
        _lib.check(self.L.mtaz_set_games(self.h, _p(pos, c_uint32), _p(ag, c_int32), _p(act, c_uint8), self.G))

    def games(self):
        pos = np.zeros((self.G, 5), np.uint32)
        ag = np.zeros(self.G, np.int32)
        act = np.zeros(self.G, np.uint8)
        oc = np.zeros(self.G, np.int32)
        _lib.check(self.L.mtaz_get_games(self.h, _p(pos, c_uint32), _p(ag, c_int32), _p(act, c_uint8), _p(oc, c_int32)))
        return pos, ag, act, oc

    def clear_trees(self, trees=None):
        if trees is None:
            _lib.check(self.L.mtaz_clear_trees(self.h, None, 0))
        else:
            t = np.asarray(trees, np.int32)
            _lib.check(self.L.mtaz_clear_trees(self.h, _p(t, c_int32), len(t)))

    def move_begin(self):
        k = np.zeros(self.G, np.int32)
        new = np.zeros(self.G, np.int32)
        _lib.check(self.L.mtaz_move_begin(self.h, _p(k, c_int32), _p(new, c_int32)))
        return k, new

    def set_noise(self, per_game):
        """per_game[g] = float64 array [draws, k] (or None) -> packed upload."""
        offs = np.zeros(self.G, np.int64)
        strides = np.zeros(self.G, np.int32)
        chunks, total = [], 0
        for g in range(self.G):
            offs[g] = total
            a = per_game[g] if g < len(per_game) else None
            if a is not None and np.size(a):
                a = np.ascontiguousarray(a, np.float64)
                strides[g] = a.shape[-1]                  # vector length = the root's legal count
                chunks.append(a.reshape(-1))
                total += a.size
        flat = np.concatenate(chunks) if chunks else np.zeros(1, np.float64)
        _lib.check(self.L.mtaz_set_noise(self.h, _p(flat, c_double), _p(offs, c_int64), _p(strides, c_int32), total))

    def simulate(self, first_sim, n_sims):
        _lib.check(self.L.mtaz_simulate(self.h, int(first_sim), int(n_sims)))

    def sim_select(self, sim):
        _lib.check(self.L.mtaz_sim_select(self.h, int(sim)))

    def leaves(self):
        cnt = c_int32()
        pos = np.zeros((self.G, 5), np.uint32)
        game = np.zeros(self.G, np.int32)
        k = np.zeros(self.G, np.int32)
        codes = np.zeros((self.G, _lib.KMAX), np.uint16)
        _lib.check(self.L.mtaz_leaves_get(self.h, ctypes.byref(cnt), _p(pos, c_uint32), _p(game, c_int32),
                                          _p(k, c_int32), _p(codes, c_uint16)))
        c = cnt.value
        return pos[:c], game[:c], k[:c], codes[:c]

    def set_leaves(self, P_rows, v):
        c = len(v)
        P = np.zeros((max(c, 1), _lib.KMAX), np.float32)
        for i, row in enumerate(P_rows):
            P[i, :len(row)] = row
        vv = np.asarray(v, np.float32).reshape(-1)
        if c == 0:
            vv = np.zeros(1, np.float32)
        _lib.check(self.L.mtaz_leaves_set(self.h, _p(P, ctypes.c_float), _p(vv, ctypes.c_float), c))

    def sim_evaluate(self):
        """The GPU network on the current leaf batch (select -> evaluate -> backup = simulate)."""
        _lib.check(self.L.mtaz_sim_evaluate(self.h))

    def leaf_results(self):
        """Device-written leaf priors and values of the last sim_evaluate: (P [c, KMAX] float32,
        row i's first k[i] entries valid in legal-list order; v [c] float32)."""
        P = np.zeros((self.G, _lib.KMAX), np.float32)
        v = np.zeros(self.G, np.float32)
        c = _lib.check(self.L.mtaz_leaves_result(self.h, _p(P, c_float), _p(v, c_float), self.G))
        return P[:c], v[:c]

    def sim_backup(self):
        _lib.check(self.L.mtaz_sim_backup(self.h))

    def move_end(self):
        codes = np.zeros((self.G, _lib.KMAX), np.uint16)
        visits = np.zeros((self.G, _lib.KMAX), np.uint32)
        k = np.zeros(self.G, np.int32)
        _lib.check(self.L.mtaz_move_end(self.h, _p(codes, c_uint16), _p(visits, c_uint32), _p(k, c_int32), _lib.KMAX))
        return codes, visits, k

    def apply(self, actions):
        a = np.zeros(self.G, np.int32)
        a[:len(actions)] = actions
        _lib.check(self.L.mtaz_apply(self.h, _p(a, c_int32)))

    def tree_arrays(self, t):
        """Table t = 2*game + agent as arrays (mtaz_tree_get): pos [n,5], e0, k, term, tval per node;
        codes, P, Q, N per edge, node i's children at [e0[i], e0[i] + k[i])."""
        nn, ne = c_int32(), c_int32()
        _lib.check(self.L.mtaz_tree_size(self.h, int(t), ctypes.byref(nn), ctypes.byref(ne)))
        n, e = nn.value, ne.value
        a = {'pos': np.zeros((max(n, 1), 5), np.uint32), 'e0': np.zeros(max(n, 1), np.uint32),
             'k': np.zeros(max(n, 1), np.uint16), 'term': np.zeros(max(n, 1), np.uint8),
             'tval': np.zeros(max(n, 1), np.float64), 'codes': np.zeros(max(e, 1), np.uint16),
             'P': np.zeros(max(e, 1), np.float32), 'Q': np.zeros(max(e, 1), np.float64),
             'N': np.zeros(max(e, 1), np.uint32)}
        _lib.check(self.L.mtaz_tree_get(self.h, int(t), _p(a['pos'], c_uint32), _p(a['e0'], c_uint32),
                                        _p(a['k'], c_uint16), _p(a['term'], c_uint8), _p(a['tval'], c_double),
                                        _p(a['codes'], c_uint16), _p(a['P'], c_float), _p(a['Q'], c_double),
                                        _p(a['N'], c_uint32)))
        a['n'] = n
        return a

    def set_tree(self, t, a):
        """Load table t from tree_arrays() output (possibly of another engine)."""
        _lib.check(self.L.mtaz_tree_set(self.h, int(t), int(a['n']), _p(a['pos'], c_uint32), _p(a['e0'], c_uint32),
                                        _p(a['k'], c_uint16), _p(a['term'], c_uint8), _p(a['tval'], c_double),
                                        _p(a['codes'], c_uint16), _p(a['P'], c_float), _p(a['Q'], c_double),
                                        _p(a['N'], c_uint32)))

    def tree(self, t):
        """Read-only view of table t = 2*game + agent in the reference's MCTS data layout:
        {'Q','N','P','legal_moves','terminal','visited'} keyed by FEN (exp/agent.py:29-36)."""
        nn, ne = c_int32(), c_int32()
        _lib.check(self.L.mtaz_tree_size(self.h, int(t), ctypes.byref(nn), ctypes.byref(ne)))
        n, e = nn.value, ne.value
        pos = np.zeros((max(n, 1), 5), np.uint32)
        e0 = np.zeros(max(n, 1), np.uint32)
        k = np.zeros(max(n, 1), np.uint16)
        term = np.zeros(max(n, 1), np.uint8)
        tval = np.zeros(max(n, 1), np.float64)
        codes = np.zeros(max(e, 1), np.uint16)
        P = np.zeros(max(e, 1), np.float32)
        Q = np.zeros(max(e, 1), np.float64)
        N = np.zeros(max(e, 1), np.uint32)
        _lib.check(self.L.mtaz_tree_get(self.h, int(t), _p(pos, c_uint32), _p(e0, c_uint32), _p(k, c_uint16),
                                        _p(term, c_uint8), _p(tval, c_double), _p(codes, c_uint16), _p(P, c_float),
                                        _p(Q, c_double), _p(N, c_uint32)))
        data = {'Q': {}, 'N': {}, 'P': {}, 'terminal': {}, 'visited': set(), 'legal_moves': {}}
        for i in range(n):
            fen = pos_to_fen(pos[i])
            data['visited'].add(fen)
            if term[i]:
                data['terminal'][fen] = float(tval[i])
                continue
            a, b = int(e0[i]), int(e0[i]) + int(k[i])
            data['Q'][fen] = Q[a:b].copy()
            data['N'][fen] = N[a:b].astype(np.float64)
            data['P'][fen] = P[a:b].copy()
            data['legal_moves'][fen] = [int(c) for c in codes[a:b]]
        return data


def start_position():
    return pos_from_fen(STARTING_FEN)
