/* mtaz — MI355X-native AlphaZero self-play engine for MinitChess: C ABI.
 *
 * Drop-in boundary for the reference's self-play hot path.  The
 * reference path is pure Python (exp/agent.py + exp/environment.py + exp/policy.py,
 * driven by app/base.py:SimulatePuppet); every entry point below names the reference
 * interface it replaces.  Plain pointers and sizes only; "d_" pointers are device
 * (HBM) pointers, everything else is host memory.  Positions are 5 x uint32 packed
 * keys (see minitchess_alphazero_amd/csrc/rules.h: struct Pos).
 *
 * Return convention: 0 (or a non-negative count) on success, negative on failure
 * with mtaz_last_error() describing it.  MTAZ_E_ILLEGAL / MTAZ_E_TERMINATED map to
 * the reference's IlegalMoveException / TerminatedEpisodeStepException
 * (exp/environment.py:8-13), which the Python layer re-raises as BaseException
 * subclasses exactly like the reference.
 */
#ifndef MTAZ_H
#define MTAZ_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTAZ_ABI_VERSION 2

#define MTAZ_E_FAIL (-1)
#define MTAZ_E_ILLEGAL (-2)     /* exp/environment.py:11 IlegalMoveException          */
#define MTAZ_E_TERMINATED (-3)  /* exp/environment.py:8  TerminatedEpisodeStepException */
#define MTAZ_E_DEVICE (-4)
#define MTAZ_E_CAPACITY (-5)

/* rules_flags bits (RULES.md) */
#define MTAZ_RF_DOUBLE_STEP 0x1u
#define MTAZ_RF_PROMO_ALL 0x2u
#define MTAZ_RF_INSUFFICIENT 0x4u
#define MTAZ_RF_FIVEFOLD 0x8u
#define MTAZ_RF_SEVENTYFIVE 0x10u
#define MTAZ_RF_DEFAULT 0x1Eu

/* ---- library -------------------------------------------------------------------- */
int mtaz_abi_version(void);
const char* mtaz_version(void);
const char* mtaz_last_error(void);
/* Load the 554-code action space.  Replaces the MOVES_DICT / MOVES_DICT_INV load of
 * exp/environment.py:15-20 (same JSON file format as exp/moves_dict.json). */
int mtaz_load_codec(const char* moves_dict_json_path);

/* ---- single-position rules on the host (MinitChessEpisode, exp/environment.py:22-85) */
int mtaz_pos_from_fen(const char* fen, uint32_t pos[5]);           /* chess.Board(fen)    :25 */
int mtaz_pos_to_fen(const uint32_t pos[5], char* buf, int cap);    /* Board.fen()         :36 */
/* sorted legal codes, duplicates kept (exp/environment.py:48-50); returns k */
int mtaz_pos_legal(const uint32_t pos[5], uint32_t rules_flags, uint16_t* codes, int cap);
/* Board.result() mapped as exp/environment.py:39-45: 0 ongoing, 1 decisive, 2 draw.
 * reps = occurrences of the position in the game history (1 without history). */
int mtaz_pos_outcome(const uint32_t pos[5], uint32_t rules_flags, int move_cap, int reps);
/* MinitChessEpisode.step(action) (exp/environment.py:68-82): decode, queen retry, push */
int mtaz_pos_step(const uint32_t pos[5], int code, uint32_t rules_flags, uint32_t out[5]);
/* 1 if the move of `code` is a capture or a pawn move (python-chess is_zeroing) */
int mtaz_pos_zeroing(const uint32_t pos[5], int code);
/* Network.process_observation (exp/policy.py:96-105): 60 tokens + clock */
int mtaz_pos_encode(const uint32_t pos[5], uint8_t tokens[60], float* clock);

/* ---- numpy legacy RandomState (np.random.* at exp/agent.py:82,115,118) ----------------- */
size_t mtaz_rng_state_size(void);
void mtaz_rng_seed(void* state, uint32_t seed);                         /* np.random.seed(s) */
double mtaz_rng_double(void* state);                                   /* random_sample()   */
void mtaz_rng_dirichlet(void* state, double alpha, int k, double* out); /* dirichlet([a]*k)  */
int64_t mtaz_rng_choice_p(void* state, const double* p, int k);        /* choice(k, p=p)    */
int64_t mtaz_rng_randint(void* state, int64_t m);                      /* choice(m)         */
/* The device build of the same generator (mtaz_play's default, mtaz_set_rng_device): stream s =
 * RandomState(seeds[s]) draws n_vec dirichlet([alpha] * ks[s]) vectors (0 < alpha < 1), written as
 * rows of ks[s] doubles, stream after stream, into out (host memory), then one random_sample() into
 * tail[s].  Runs the kernels' own sampler code (csrc/mtaz_rng.hip: MT19937 words in LDS, 64 gamma
 * attempts per wavefront, glibc's log/pow ported in csrc/glibc_math.h).  Replaces the host draws of
 * exp/agent.py:82 (np.random.dirichlet). */
int mtaz_rng_dirichlet_device(int device, const uint32_t* seeds, const int32_t* ks, int n_streams, int n_vec,
                              double alpha, double* out, double* tail);

/* ---- batched device kernels (minimum slice) ------------------------------------------- */
/* Per position: sorted legal codes (KMAX=256 per row), count, 554-bit mask (18 words),
 * outcome.  Replaces MinitChessEpisode._update_attributes (exp/environment.py:34-50). */
int mtaz_legal_batch(int device, const uint32_t* d_pos, int n, uint32_t rules_flags, int move_cap, uint16_t* d_codes,
                     int32_t* d_counts, uint32_t* d_masks, int32_t* d_outcomes, void* stream);
/* Network.process_observation for a batch (exp/policy.py:96-105) */
int mtaz_encode_batch(int device, const uint32_t* d_pos, int n, uint8_t* d_tokens, float* d_clocks, void* stream);
/* Replay memory ingest (exp/dataset.py:6-20 push + the row half of collate_fn,
 * exp/learner.py:23-37), all pointers device memory: row i of a packed record batch (pos,
 * legal list length k, entry start e0 into codes / visits, reward) is written to ring slot
 * (head + i) % cap as tokens [60] u8, clock f32, dense pi [554] f32 (N / N.sum() in float64,
 * repeated codes: last entry wins) and reward f32.  n <= cap; d_e0[i] + d_k[i] must lie inside
 * codes / visits (the caller's prefix sum).  Enqueued on `stream` (no sync). */
int mtaz_replay_put(int device, int n, const uint32_t* d_pos, const int32_t* d_k, const int64_t* d_e0,
                    const uint16_t* d_codes, const uint32_t* d_visits, const float* d_reward, int64_t cap,
                    int64_t head, uint8_t* d_tokens, float* d_clocks, float* d_pi, float* d_reward_out, void* stream);

/* ---- engine ------------------------------------------------------------------------- */
typedef struct mtaz_engine mtaz_engine;

/* One engine per GPU.  Holds n_games game slots, two MCTS tables per slot (the two
 * SimpleAlphaZeroAgents of app/base.py:113), numpy-legacy RNG per slot seeded
 * seed_base + slot, and the network.  Replaces SimulatePuppet's agents/env/policy
 * construction (app/base.py:74-84, :113-114).  numpy_cast_mode: 2 = numpy>=2 promotion
 * (NEP 50), 1 = numpy 1.x.  NULL on failure. */
mtaz_engine* mtaz_create(int device, int n_games, int sims, double cpuct, int tau_change, double dir_alpha,
                         double dir_eps, uint64_t seed_base, int numpy_cast_mode, uint32_t rules_flags, int move_cap);
void mtaz_destroy(mtaz_engine* h);
/* SimulatePuppet.load_weights (app/base.py:126-129): the 133 float32 device tensors of
 * Network.state_dict() in order, num_batches_tracked skipped.  BN is folded and conv
 * weights re-laid out into engine-owned HBM; the caller's tensors are not retained. */
int mtaz_set_weights(mtaz_engine* h, const float* const* d_tensors, const int64_t* numels, int n);
/* Network.forward (exp/policy.py:71-80) on n device positions: logits [n][554], values [n]. */
int mtaz_evaluate(mtaz_engine* h, const uint32_t* d_pos, int n, float* d_logits, float* d_values);

/* Batched self-play: n_games full episodes from STARTING_FEN (or the roots set by
 * mtaz_set_games when from_current != 0).  Replaces erlyx.run_episodes under
 * SimulatePuppet.run_episodes (app/base.py:108-124). */
int mtaz_play(mtaz_engine* h, int n_games, int from_current);
/* Episode records (exp/callbacks.py:31-54 InfoRecorder): per game the ply count; per
 * ply the observation position, action, legal list length, then the legal codes and
 * root visit counts N (pi = N / sum N) concatenated over plies. */
int mtaz_records_counts(mtaz_engine* h, int32_t* plies_per_game, int64_t* total_plies, int64_t* total_entries);
int mtaz_records_get(mtaz_engine* h, uint32_t* pos, int32_t* action, int32_t* k, uint16_t* codes, uint32_t* visits,
                     float* reward, int32_t* outcome);
/* Episode wire format (app/base.py:63-69, MQTTDataset.push): one MQTT payload per game,
 * byte-identical to json.dumps({'episode': InfoRecorder records, 'userid': userid,
 * 'weights_version': weights_version, 'minitchess_alphazero_version': version}) (NULL
 * strings are JSON null), from packed records laid out as mtaz_records_get writes them.
 * Payload g is out[offsets[g] .. offsets[g+1]); returns the total byte count (offsets[n_games]
 * too).  When out is NULL or the total exceeds cap nothing is written: call again with a
 * buffer of the returned size.  Host-only; no engine or device needed. */
int64_t mtaz_records_json(int n_games, const int32_t* plies, const uint32_t* pos, const int32_t* action,
                          const int32_t* k, const uint16_t* codes, const uint32_t* visits, const float* reward,
                          const char* userid, const char* weights_version, const char* version, char* out,
                          int64_t cap, int64_t* offsets);
/* CPython repr(float) of x (the float spelling of the payloads above); returns its length */
int mtaz_repr_double(double x, char* buf, int cap);
/* counters of the last mtaz_play: see minitchess_alphazero_amd/engine.py STAT_NAMES */
int mtaz_stats(mtaz_engine* h, double* out, int n);
/* record per-wave network HIP events during mtaz_play (trunk span for fp32, the fused
 * network kernel for fp16x3) */
int mtaz_set_timing(mtaz_engine* h, int on);
/* network arithmetic: 1 = k_net_y (default), fp16x3 split MFMA, within 1e-5 of the reference on
 * every tested net; 2 = k_net_z, f16 Wh*Xh + e4m3 cross terms: its scope is nets whose layer
 * bounds stay below 2^14 (within 1e-5 on the seed-0 and C3 nets; past 2^14 its results depend on
 * the batch and it refuses the leaf memo, mtaz_set_memo); 0 = fp32 MFMA */
int mtaz_set_precision(mtaz_engine* h, int precision);
/* game slot g of the next mtaz_play is seeded np.random.seed(seed_base + g) */
int mtaz_set_seed_base(mtaz_engine* h, uint64_t seed_base);
/* host threads of the per-move work (Dirichlet draws, action choice; 0 = the CPUs of the process's
 * affinity mask, at most 16).  Pipeline groups split them. */
int mtaz_set_host_threads(mtaz_engine* h, int n);
/* how the host thread waits for the engine's stream at its sync points (root states, visit counts,
 * error flags): 0 = hipStreamSynchronize (default), 1 = an event created with hipEventBlockingSync,
 * so the waiting thread sleeps instead of holding a CPU (8 ranks share one node's host cores:
 * bench.py --sync-mode, --rank-share).  Results are identical in both modes. */
int mtaz_set_sync_mode(mtaz_engine* h, int mode);
/* Deferred tails in mtaz_play (2 = default since round 6: every remainder waits, partial rounds too;
 * 1 = remainders of at most 3 boards per CU, which would take a tail launch, wait; 0 = off).  The network runs in full rounds of 4 boards
 * per CU; a simulation wave whose leaf count n is not a multiple of that round (4 x CUs) used to
 * end with a tail launch whose 1-3-board workgroups stream all weights for few boards.  With
 * deferral a wave evaluates only the whole rounds; the remaining leaves stay pending and lead the
 * next wave's list, their games selecting again only after that leaf's backup, and each move
 * ends with the waves its lagging games still need (every leaf evaluated).  Every game still runs
 * its simulations one at a time and in order (exp/agent.py:41-45), on the same tables, noise
 * draws and network results, so games, tables and records are identical in both modes; only the
 * wave each simulation runs in moves.  The fine-grained API (mtaz_sim_select ...) is unaffected. */
int mtaz_set_defer(mtaz_engine* h, int mode);
/* Which leaves a deferred-tail wave evaluates first (its list's order; the rest of the list waits):
 * 0 (default, round 6) = the least advanced games first (simulations started in the play, relative to
 * the least advanced leaf: 0, 1, 2, 3+; game order within), so the leaders wait and no game falls far
 * behind the others, which sets how many waves a move's end needs; 1 = round 5's order (lag behind
 * the most advanced leaf: 3+, 2, 1, 0), where one game far ahead put most leaves in the 3+ bucket
 * and game order then chose whom to defer.  Results are identical; for the A/B. */
int mtaz_set_lag_order(mtaz_engine* h, int order);
/* Where mtaz_play runs numpy's legacy RNG (exp/agent.py:82 Dirichlet noise, :114-118 action choice):
 * 1 (default) = on the device: per-game MT19937 state in HBM, each move's Dirichlet draws in one
 * launch (k_noise: one wavefront per game, 64 gamma attempts at once) and the action choice in
 * another (k_choose); 0 = on the host (C++ MT19937 / legacy gamma / choice with glibc's log and pow,
 * drawn in chunks that overlap the simulations).  Both give every game's RandomState(seed_base + g)
 * stream draw for draw, so games are identical.  The device sampler covers 0 < dir_alpha < 1 (the
 * reference's 0.6); other alphas run on the host. */
int mtaz_set_rng_device(mtaz_engine* h, int on);
/* mtaz_play's schedule: 0 (default) = moves in lockstep (every game's move ends in the same wave;
 * per-move host hand-offs); 1 = free-running moves: a game whose move is complete records it,
 * chooses its action, steps and starts its next move on the device (one k_turn launch per wave,
 * one wavefront per game that finished a move) while the other games keep simulating; the host
 * only reads the active-game count every 16 waves and the records at the end.  Every game runs the
 * same simulations on the same tables, draws and network results in both, so the records are
 * identical; on the bench workload free-running is 1.5% slower (more waves, k_turn on every wave's
 * critical path).
 * Free-running needs the device RNG (mtaz_set_rng_device 1, dir_alpha < 1) and one network for both
 * agents; mtaz_play falls back to lockstep otherwise (stat 'schedule' says which ran). */
int mtaz_set_schedule(mtaz_engine* h, int mode);
/* per-wave log of the last mtaz_play (up to max_waves): out[3 * w + 0] leaves evaluated,
 * [+1] game-memo hits, [+2] batch-memo hits; returns the number of waves written */
int mtaz_wave_log(mtaz_engine* h, int32_t* out, int max_waves);
/* network-only timing harness: avg ms over `iters` launches on n device positions; with
 * stamped != 0 also, from one more launch of the stamp-instrumented build (4 boards per
 * workgroup, nwg = ceil(n / 4)), stamps_out[nwg * 10]: per workgroup [nwg][stem, conv K loops,
 * epilogues, heads cycles, total cycles, total 100 MHz ticks], then (k_net_y) per board
 * [nwg][4]: (largest stored-units exponent << 32) | bit mask of the layers whose exponent is
 * nonzero (bit 0 = stem, 1 + L = conv L) (tools/bench_net.py, tests/test_gpu_stress.py) */
int mtaz_net_time(mtaz_engine* h, const uint32_t* d_pos, int n, int iters, int stamped, float* ms_out,
                  uint64_t* stamps_out);
/* select a network kernel code variant of the current precision for A/B timing (0 = the
 * product kernel; the bits are listed in minitchess_alphazero_amd/engine.py set_net_variant) */
int mtaz_set_net_variant(mtaz_engine* h, int variant);
/* Two-network play (the arena of exp/learner.py:97-145): upload a network into weight slot 0
 * or 1 (mtaz_set_weights fills slot 0), and map agent 0 (the first mover, exp/agent.py:11-14)
 * and agent 1 to slots.  With different slots, mtaz_play evaluates each move's leaves with the
 * network of the agent to move (games from STARTING_FEN move in lockstep). */
int mtaz_set_weights_slot(mtaz_engine* h, int slot, const float* const* d_tensors, const int64_t* numels, int n);
int mtaz_set_agent_slots(mtaz_engine* h, int slot_agent0, int slot_agent1);
/* mtaz_play over `groups` independent game groups (1 = off; must divide n_games): each group
 * has its own HIP stream and host thread, so one group's tree kernels and network tail run
 * while another's network occupies the GPU.  Games keep their global seeds, so results are
 * identical for any group count.  Applies to full-batch mtaz_play(h, n_games, 0) only. */
int mtaz_set_pipeline(mtaz_engine* h, int groups);
/* Leaf memo (1 = per game, the default; 2 = per game + batch; 0 = off).  The reference evaluates
 * its network on every leaf it expands (exp/agent.py:64-71), a pure function of the position; each
 * of a game's two agents keeps its own table (app/base.py:113), so a position one agent expanded
 * earlier is evaluated again when the other agent reaches it.  With the memo the second expansion
 * copies the first one's legal list, priors and value (or terminal value) from the other table:
 * every table, visit count and move is unchanged, the network runs on fewer leaves.  Mode 2 also
 * keeps every evaluated position of the play (all games, until the next mtaz_play, mtaz_clear_trees
 * of all tables or mtaz_set_weights) in an HBM table that later simulations of any game read.  Off
 * automatically when the agents use different weight slots (mtaz_set_agent_slots).
 * A memo hit hands on a result computed in another network launch, which is exact for precisions 0
 * and 1 (every board computed independently of its batch).  Precision 2 (k_net_z) keeps one
 * dynamic-range exponent per workgroup: once a layer's bound passes 2^14 its results depend on the
 * other boards of the workgroup, so a play with memo >= 1 that reaches that range fails
 * (MTAZ_E_CAPACITY, "f16f8-range-with-memo"); with memo 0 it plays, outside the sharding identity. */
int mtaz_set_memo(mtaz_engine* h, int mode);
/* Edge storage of the MCTS tables (exp/agent.py:29-36 keeps a list of Q/N/P per node; here a
 * node's children are a contiguous edge range).  Each of the 2 * n_games tables owns a region of
 * per_tree edges; a node whose children do not fit takes them from a pool of `pool` edges shared
 * by all tables, so no single table's size is a limit, only the pool's exhaustion (then
 * MTAZ_E_CAPACITY, "edge-capacity").  Defaults: 16 and 8 * n_games * 2 edges per node of a table.
 * Reallocates and clears every table (between games only); pipeline groups keep the default. */
int mtaz_set_edge_capacity(mtaz_engine* h, int64_t per_tree, int64_t pool);

/* ---- fine-grained search (MonteCarloTreeSearch.simulate, exp/agent.py:41-45, and
 *      SimpleAlphaZeroPolicy.get_distribution, exp/policy.py:115-122) --------------- */
int mtaz_set_games(mtaz_engine* h, const uint32_t* roots, const int32_t* agents, const uint8_t* active, int n);
int mtaz_get_games(mtaz_engine* h, uint32_t* roots, int32_t* agents, uint8_t* active, int32_t* outcome);
/* MonteCarloInit.on_episode_begin -> agent.init_mcts() (exp/callbacks.py:61-62): tree = 2*game + agent.
 * trees == NULL clears every table and empties the shared edge pool; a partial list clears those
 * tables but does not return the pool edges they had taken (the pool is reclaimed by the next
 * clear of all tables, which mtaz_play does) */
int mtaz_clear_trees(mtaz_engine* h, const int32_t* trees, int n);
/* root legal count and "root not yet visited" per game (decides the Dirichlet draws) */
int mtaz_move_begin(mtaz_engine* h, int32_t* root_k, int32_t* root_new);
/* Dirichlet vectors for this move: game g, draw j, child c at noise[offsets[g] + j*strides[g] + c]
 * (strides[g] = the root's legal count k; NULL = the counts of this move's mtaz_move_begin, an
 * error without one since mtaz_create / mtaz_set_games) */
int mtaz_set_noise(mtaz_engine* h, const double* noise, const int64_t* offsets, const int32_t* strides, int64_t total);
/* run sims [first, first+n) with the GPU network as leaf evaluator */
int mtaz_simulate(mtaz_engine* h, int first_sim, int n_sims);
/* host-evaluator mode: select -> (get leaves, caller computes P and v) -> set -> backup */
int mtaz_sim_select(mtaz_engine* h, int sim);
int mtaz_leaves_get(mtaz_engine* h, int32_t* count, uint32_t* pos, int32_t* game, int32_t* k, uint16_t* codes);
int mtaz_leaves_set(mtaz_engine* h, const float* P, const float* v, int count);
/* the GPU network on the current leaf batch (what mtaz_simulate runs between select and backup):
 * writes each leaf's priors P = softmax(logits[legal list]) and value v, the leaf evaluation of
 * exp/agent.py:66-71 */
int mtaz_sim_evaluate(mtaz_engine* h);
/* read those device-written leaf results: P [count][KMAX] (first k entries of row i valid, the
 * legal-list order of mtaz_leaves_get), v [count]; returns the leaf count (error if > count) */
int mtaz_leaves_result(mtaz_engine* h, float* P, float* v, int count);
int mtaz_sim_backup(mtaz_engine* h);
/* root children codes and visit counts [n_games][kout] */
int mtaz_move_end(mtaz_engine* h, uint16_t* codes, uint32_t* visits, int32_t* k, int kout);
/* MinitChessEpisode.step for every active game + game-level result (with history) */
int mtaz_apply(mtaz_engine* h, const int32_t* actions);
/* read-only tree view for parity tests (mcts['N'|'Q'|'P'|'legal_moves'|'terminal']): edges = the
 * summed legal-list length of the non-terminal nodes; tree_get writes node i's children compactly
 * at [e0[i], e0[i] + k[i]) of codes / P / Q / N, in node order */
int mtaz_tree_size(mtaz_engine* h, int tree, int32_t* nodes, int32_t* edges);
int mtaz_tree_get(mtaz_engine* h, int tree, uint32_t* pos, uint32_t* e0, uint16_t* k, uint8_t* term, double* tval,
                  uint16_t* codes, float* P, double* Q, uint32_t* N);
/* load a table from the mtaz_tree_get layout (n nodes; the hash index and visit sums are rebuilt):
 * moves a MonteCarloTreeSearch into a larger engine when a later simulate() asks for more
 * simulations than its first (exp/agent.py:41-45 has no such limit).  Edges that do not fit the
 * table's own region take a fresh block of the shared pool; pool edges the replaced table held are
 * NOT returned (as for a partial mtaz_clear_trees): load into a cleared table, and reclaim the pool
 * with a clear of all tables (mtaz_clear_trees(h, NULL, 0); mtaz_play does one) */
int mtaz_tree_set(mtaz_engine* h, int tree, int n, const uint32_t* pos, const uint32_t* e0, const uint16_t* k,
                  const uint8_t* term, const double* tval, const uint16_t* codes, const float* P, const double* Q,
                  const uint32_t* N);

#ifdef __cplusplus
}
#endif
#endif /* MTAZ_H */
