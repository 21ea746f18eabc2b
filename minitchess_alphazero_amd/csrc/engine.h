// Engine state shared between the device TU (mtaz_device.hip) and the host TU
// (mtaz_host.cpp).  All per-game / per-tree state lives in HBM as SoA arrays.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rules.h"

namespace mtaz {

// Action codec (exp/moves_dict.json; SURVEY a-6).  enc[side][from*30+to] -> code
// or -1; dec[side][code] -> from | to << 8.  side 0 = white, 1 = black.
struct Codec {
  int16_t enc[2][900];
  uint16_t dec[2][NUM_ACTIONS];
};

constexpr int KMAX = 256;              // max legal-list length handled (error beyond)
constexpr int MASK_WORDS = 18;         // 554-bit legal mask padded to 576 bits
constexpr uint32_t NONE = 0xffffffffu;

enum ErrBits : int32_t {
  ERR_NODES = 1, ERR_EDGES = 2, ERR_DEPTH = 4, ERR_KMAX = 8, ERR_SQRT = 16, ERR_ROOT = 32,
  ERR_ILLEGAL = 64, ERR_HIST = 128, ERR_HASH = 256,
};

// A node's scalars in one 16-B record (one load per level of the descent)
struct alignas(16) NodeHdr {
  uint32_t e0;            // first edge (a global edge index: the tree's own region or the pool)
  uint32_t sumN;          // sum of child N (exact; numpy N.sum())
  uint32_t kt;            // bits 0..15: number of children (legal list length, duplicates
                          // kept); HDR_TERM: terminal (exp/agent.py:59-63)
  float tval;             // terminal: the stored value (= -reward: -1 or -0, exact in float);
                          // otherwise the leaf value v the network returned (exp/agent.py:67,72),
                          // kept for the per-game leaf memo (Params::memo)
};
constexpr uint32_t HDR_TERM = 1u << 16;
__host__ __device__ __forceinline__ int hdr_k(const NodeHdr& h) { return (int)(h.kt & 0xffffu); }
__host__ __device__ __forceinline__ bool hdr_term(const NodeHdr& h) { return (h.kt & HDR_TERM) != 0; }

// MCTS transposition DAG per (game, agent): exp/agent.py:29-36 keeps
// {Q, N, P, terminal, visited, legal_moves} keyed by FEN; here a node is the
// packed Pos key in an open-addressing table, its children a contiguous edge
// range (SoA: code u16, P f32, Q f64, N u32, child node).  Tree t owns nodes [t*NC, (t+1)*NC),
// hash slots [t*HC, ...) and the edge region [t*EC, (t+1)*EC).  A node's k edges go to its
// tree's region while they fit, else to the shared edge pool [pool_base, pool_base + pool_cap)
// (one atomicAdd per spilled node), so one tree outgrowing its region costs nothing; only an
// exhausted pool is an error.  Edge indices (NodeHdr::e0, path edges) are global.
struct Trees {
  Pos* node_pos;
  NodeHdr* node_hdr;
  uint32_t* hash;         // node index + 1, 0 = empty
  uint32_t* n_nodes;      // [T]
  uint32_t* n_edges;      // [T]
  uint16_t* e_code;
  float* e_P;
  double* e_Q;
  uint32_t* e_N;
  uint32_t* e_child;      // the child's node index once the edge has been followed, else NONE
  uint32_t* pool_used;    // [1] edges handed out from the pool
  int NC, HC, EC;
  uint32_t pool_base, pool_cap;
};

struct Games {
  Pos* root;              // current game position = MCTS root
  uint32_t* root_node;    // hint: the root's node in the agent's tree (NONE = unknown; k_select checks it)
  int32_t* agent;         // tree slot (0/1) of the agent to move
  uint8_t* active;        // 1 while the game runs
  int32_t* outcome;       // game result (Outcome)
  int32_t* root_new;      // root absent from the agent's table at move start
  int32_t* root_k;        // legal-list length of the root
  // this move's Dirichlet vectors: draw j of game g at noise[noise_off[g] + j*noise_js[g] + c]
  // (mtaz_set_noise: per-game contiguous, js = k; mtaz_play: draw-major, js = the move's total k,
  // so that a range of draws is one contiguous upload)
  int64_t* noise_off;
  int32_t* noise_js;
  double* noise;
  uint32_t* path_node;    // [G*DMAX] chain of (node, edge) of the current sim
  uint32_t* path_edge;
  int32_t* path_len;
  // deferred-tail play (mtaz_set_defer): simulations this move has started per game (the noise
  // draw index of the next one); a game whose leaf was deferred keeps it in Leaves::gnode and
  // selects again only after that leaf's backup
  int32_t* simc;
  Pos* hist;              // [G*HMAX] game positions before each move (repetition)
  int32_t* nhist;
  int DMAX, HMAX;
  // numpy legacy RandomState per game on the device (mtaz_rng.hip): the MT19937 block of game g at
  // mt_key[g*624 .. +624] and the index of its next word (numpy's state.pos)
  uint32_t* mt_key;
  int32_t* mt_pos;
  // simulations each game has started in the play (k_leaf_compact orders pending leaves by how far
  // their game is behind the most advanced one; with free-running moves games are on different moves)
  int32_t* stot;
  // free-running moves: the Dirichlet vectors drawn so far in the game's current move (k_turn draws them
  // in chunks as the simulations come to need them, round 6)
  int32_t* ndraw;
  // free-running moves (mtaz_set_schedule 1, k_turn): each game's InfoRecorder records written on the
  // device, ply p of game g at [g * PLY + p]; its legal lists and root visit counts appended to its
  // region [g * RC, g * RC + rec_cur[g]) (RC = PLY x KMAX)
  int32_t* nply;
  int32_t* rec_cur;
  Pos* rec_pos;
  int32_t* rec_action;
  int32_t* rec_k;
  uint16_t* rec_codes;
  uint32_t* rec_visits;
  int PLY;
  int64_t RC;
};

struct Leaves {
  // k_select writes game g's leaf (node, position) at index g, NONE when the simulation ended
  // without one; k_leaf_compact then lists the leaves densely in game order (no contended
  // counter: one atomic per game on a single address serialised the select kernel)
  uint32_t* gnode;        // [G]
  Pos* gpos;              // [G]
  int32_t* count;         // [1]
  int32_t* game;          // [G]
  int32_t* tree;          // [G]
  uint32_t* node;         // [G]
  Pos* pos;               // [G]
  float* P;               // [G*KMAX] priors (softmax over the legal logits)
  float* v;               // [G]
  uint8_t* ghit;          // [G] 1 / 2 when game g's simulation took its leaf from the game / batch memo
};

// Batch leaf memo (Params::memo == 2): network results of the positions this engine evaluated
// since the play started, shared by all its games.  Open addressing on the packed position
// (linear probing); k_backup inserts each evaluated leaf (a slot claimed by atomicCAS on its
// state: 0 empty, 1 being written, 2 ready), k_select of later simulations looks positions up.
// Positions with more than MEMO_K legal moves are not kept.
constexpr int MEMO_K = 32;
constexpr uint32_t MEMO_PROBES = 64;   // insert and lookup give up after this many slots (a full table only loses hits)
struct BatchMemo {
  uint32_t* state;        // [cap]
  Pos* key;               // [cap]
  float* v;               // [cap]
  uint16_t* k;            // [cap]
  uint16_t* codes;        // [cap][MEMO_K]
  float* P;               // [cap][MEMO_K]
  uint32_t cap;           // power of two (0 = not allocated)
};

struct Params {
  int G, sims;
  float cpuct_f;
  double cpuct;
  int cast_mode;          // 2 = numpy>=2 promotion, 1 = numpy 1.x value-based casting
  uint32_t flags;
  int move_cap;
  const double* sqrt_tab; // sqrt(n) for n < sqrt_n (exactly what np.sqrt returns)
  int sqrt_n;
  int32_t* err;
  // leaf memo (0 = off, 1 = per game, 2 = per game + batch): a position the game's other agent
  // already expanded takes its legal list, priors and value from that agent's table (and with 2, a
  // position any game of the batch had evaluated, from the BatchMemo) instead of a network
  // evaluation.  The network is a pure function of the position (exp/agent.py:64-71 evaluates
  // process_observation(fen) alone) and per-board deterministic, so the tables, and every result,
  // are those without the memo.  Off when the two agents search with different networks (arena).
  int memo;
  double alpha;           // Dirichlet concentration of the root noise (exp/agent.py:82: 0.6)
  int tau;                // fullmove number from which moves are argmax picks (exp/agent.py:113)
  // deferred-tail play's leaf order (k_leaf_compact; mtaz_set_lag_order): 0 (default, round 6) =
  // by simulations ahead of the least advanced leaf, ascending (buckets 0, 1, 2, 3+); 1 = round 5's:
  // by lag behind the most advanced leaf, descending (3+, 2, 1, 0)
  int lag_order;
};

struct Dev {
  Trees tr;
  Games gm;
  Leaves lf;
  Params pr;
  BatchMemo bm;
};

// ---- network -------------------------------------------------------------------------
// Packed weights (BN folded, eval mode).  Conv 3x3 weights are pre-swizzled into the
// B-fragment order of v_mfma_f32_32x32x2_f32: [cotile 8][kstep/4 288][lane 64][4],
// kstep s covers k = 2s, 2s+1 with k = tap*256 + ci.
struct NetWeights {
  const float* emb;       // [7][4]
  const float* stem_w;    // [256][72]  (ci*9 + tap), BN folded
  const float* stem_b;    // [256]
  const float* conv_w;    // [18][8*288*64*4]
  const float* conv_b;    // [18][256]
  const float* pconv_w;   // [2][256] folded
  const float* pconv_b;   // [2]
  const float* plin_w;    // [554][61]
  const float* plin_b;    // [554]
  const float* vconv_w;   // [256]
  const float* vconv_b;   // [1]
  const float* vl1_w;     // [256][31]
  const float* vl1_b;     // [256]
  const float* vl2_w;     // [256]
  const float* vl2_b;     // [1]
  // fp16x3 trunk: per layer the BN-folded weights scaled by 2^e_L and split hi = f16(w),
  // lo = f16(w - hi), as the A operand of v_mfma_f32_16x16x32_f16 (k_net_y; k_net_z reads the
  // hi parts): [L 18][cotile 16][kblock 72][part][lane 64][8 x f16], lane l holds
  // W[co = 16*cotile + (l&15)][k = 32*kblock + 8*(l>>4) + j], k = tap*256 + ci
  const float* convx_inv; // [18] 2^-e_L
  const float* stemx_inv; // [1] the stem's
  const uint4* convy;
  // round 4's k_net_y: the same split weights k-block-major, [L 18][kblock 72][cotile 16][part]
  // [lane 64][8 x f16], so that one k-block's 8 fragments of a wave sit at one scalar base plus
  // immediates (buffer loads with no per-load scalar arithmetic)
  const uint4* convyk;
  // stem: [cotile 16][kblock 3][part][lane 64][8 x f16], co = 16*cotile + (l&15),
  // tap = 4*kblock + (l>>4) (taps 9..11 zero), channel j; scale stemx_inv
  const uint4* stemy;
  // k_net_y dynamic range: [2L] = max over output channels of the L1 norm of conv L's folded
  // weights, [2L+1] = max |folded bias| (L < 18); [36], [37] the same for the stem; [38] =
  // max |embedding|.  Each rounded up to float.
  const float* yrange;
  // k_net_z (f16 + e4m3 cross terms): the split weights' hi and lo parts of convy, each scaled by
  // a per-layer power of two and rounded to OCP e4m3, as the A operand of
  // v_mfma_scale_f32_16x16x128_f8f6f4: [L 18][cotile 16][tap 9][chunk 2][part hi/lo][half 2]
  // [lane 64][16 B]; lane l holds W[co = zrow_co(cotile, l&15)][ci = 128*chunk + 32*(l>>4) + j]
  // (j = 16*half + byte) of that tap.  conv8_sc[2L + part] = the e8m0 scale that undoes the
  // part's power of two (127 - a).
  const uint4* conv8;
  const int32_t* conv8_sc;
  // k_net_z VAR 8192 (cross terms in e2m3 = fp6): the same hi / lo parts as conv8, each block of
  // 32 K (one output channel, tap, 32 input channels) in e2m3 with its own e8m0 scale:
  // [L 18][cotile 16][group 36 = (tap, chunk, part)][112 x 16 B]; per group and lane l
  // (co = zrow_co(cotile, l&15), channels 128*chunk + 32*(l>>4) + q): bytes 0..15 of the 24-B
  // fp6 vector at 16 B x l, bytes 16..23 at 1024 + 8 l, the scale (u32, byte 0) at 1536 + 4 l.
  // Value q of the vector (bits 6q..6q+5) is channel q of the 32-channel block.
  const uint4* conv6;
  // k_net_z's copies of convy and stemy (both parts) with the output channels of each pair of
  // 16-row tiles interleaved, and conv8 / conv6 in the same row order: row r of tile T is
  // channel zrow_co(T, r), so that the epilogue's lane g holds 8 consecutive channels of a tile pair
  // (one 16-B f16 store and two 8-B e4m3 stores per square)
  const uint4* convz;
  const uint4* stemz;
};
__host__ __device__ __forceinline__ int zrow_co(int T, int r) { return 32 * (T >> 1) + 8 * (r >> 2) + 4 * (T & 1) + (r & 3); }
constexpr int CONV_LAYERS = 18;
constexpr size_t CONV_W_FLOATS = (size_t)8 * 288 * 64 * 4;   // 589,824 = 256*2304
constexpr size_t CONVX_U4_PER_LAYER = (size_t)16 * 72 * 2 * 64;  // 147,456 x 16 B = 2.36 MB (convy)
enum NetPrecision { NET_FP32 = 0, NET_F16X3 = 1, NET_F16F8 = 2 };
constexpr size_t CONV8_U4_PER_LAYER = (size_t)16 * 9 * 2 * 2 * 2 * 64;   // 73,728 x 16 B = 1.18 MB
constexpr size_t CONV6_U4_PER_LAYER = (size_t)16 * 36 * 112;   // 64,512 x 16 B = 1.03 MB
constexpr int ERR_F16 = 512;   // activation exceeded the f16 range in the fp16x3 trunk
// k_net_z's one stored-units exponent per WORKGROUP left 0 (a bound passed 2^14): its results then
// depend on the boards sharing the workgroup.  An error only where a leaf memo would hand such a
// result to another batch (check_err(h, true) with memo >= 1); evaluate paths clear it.
constexpr int ERR_ZRANGE = 1024;
// k_choose: a randint rejection loop outran the 64 words reserved for it (probability < 2^-64)
constexpr int ERR_RNG = 2048;
// k_select: the PUCT argmax found no child (cannot happen: a NaN score counts as the maximum, as in
// numpy's argmax); the simulation stops instead of following an edge past the node's k
constexpr int ERR_PUCT = 4096;

struct NetBuffers {
  float* x0;              // [B][256][32]
  float* x1;
  float* t;
  float* logits;          // [B][554] (evaluate mode only)
  int B;
};

// ---- launchers (defined in mtaz_device.hip) ------------------------------------------------
int dev_upload_codec(const Codec& c);
void launch_legal_batch(const Pos* pos, int n, uint32_t flags, int move_cap, uint16_t* codes, int32_t* counts,
                        uint32_t* masks, int32_t* outcomes, hipStream_t s);
void launch_encode_batch(const Pos* pos, int n, uint8_t* tokens, float* clocks, hipStream_t s);
void launch_replay_put(const Pos* pos, const int32_t* k, const int64_t* e0, const uint16_t* codes,
                       const uint32_t* visits, const float* reward, int n, int64_t cap, int64_t head,
                       uint8_t* tokens, float* clocks, float* pi, float* reward_out, hipStream_t s);
// all_trees: also empties the edge pool (a partial reset leaves the pool's edges allocated)
void launch_reset_trees(const Dev& d, const int32_t* trees, int ntrees, bool all_trees, hipStream_t s);
void launch_move_begin(const Dev& d, hipStream_t s);
// k_select + k_leaf_compact; count_log (optional, device) receives [leaf count, memo hits], ev_mid
// (optional) is recorded between the two kernels
// defer (mtaz_set_defer): 0 = every game selects simulation `sim` and every leaf is evaluated this
// wave; 1 = games select their own next simulation (Games::simc) unless a deferred leaf is
// pending, the leaf list is ordered by lag (largest first), and when `cut` is set only the whole
// rounds of `round` leaves are evaluated (the rest stay pending for the next wave)
void launch_select(const Dev& d, int sim, hipStream_t s, int32_t* count_log = nullptr, hipEvent_t ev_mid = nullptr,
                   int defer = 0, int cut = 0, int round = 0);
// after a deferred-tail move's regular waves: the waves still needed (max over games of the
// simulations not yet started + a pending leaf) into *out
void launch_remaining(const Dev& d, int32_t* out, hipStream_t s);
#ifdef MTAZ_NET_DIAG
int diag_select_stamps(unsigned long long* out8, int reset);   // k_select phase cycles (diag library)
#endif
void launch_net(const Dev& d, const NetWeights& w, const NetBuffers& nb, const Pos* pos, const int32_t* count, int max_b,
                int mode, float* values_out, hipStream_t s, hipEvent_t trunk_begin, hipEvent_t trunk_end);
// fused fp16x3 network (stem + 18 convs + heads in one launch, 4 boards per workgroup):
// k_net_y on v_mfma_f32_16x16x32_f16 (mtaz_net16.hip)
void launch_net_f16x3(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                      float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                      int variant);
// round 3's k_net_y (mtaz_net16_r3.hip; f16x3 variant 3): one stored-units exponent per workgroup
void launch_net_f16x3_r3(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                         float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                         int variant);
// diagnostic instantiation with per-phase s_memtime stamps (never the product path)
void launch_net_f16x3_stamped(const Dev& d, const NetWeights& w, const Pos* pos, int n, float* logits_out,
                              float* values_out, unsigned long long* stamps, hipStream_t s, int variant);
// k_net_z (mtaz_net8.hip): the same fused network with the split's cross terms Wh*Xl + Wl*Xh on
// the block-scaled e4m3 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4), Wh*Xh on the f16 MFMA
void launch_net_z(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                  float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                  int variant);
void launch_net_z_stamped(const Dev& d, const NetWeights& w, const Pos* pos, int n, float* logits_out,
                          float* values_out, unsigned long long* stamps, hipStream_t s, int variant);
void launch_backup(const Dev& d, hipStream_t s);
void launch_memo_clear(const Dev& d, hipStream_t s);
void launch_move_end(const Dev& d, uint16_t* codes_out, uint32_t* visits_out, int kout, hipStream_t s);
void launch_apply(const Dev& d, const int32_t* actions, hipStream_t s);
// free-running moves: (start) every active game begins its move, or (!start) every game whose move is
// complete finishes it (record, action choice, game step) and begins the next; then the active count
void launch_turn(const Dev& d, int start, hipStream_t s);
void launch_count_active(const Dev& d, int32_t* out, hipStream_t s);
// the games' appended legal lists / visit counts packed game after game at off[g] (host-computed)
void launch_rec_pack(const Dev& d, const int64_t* off, uint16_t* codes, uint32_t* visits, hipStream_t s);
void launch_gather_leaf_codes(const Dev& d, uint16_t* codes_out, int32_t* k_out, hipStream_t s);
// device legacy RNG (mtaz_rng.hip): seed every game's MT19937 with seed_base + g; this move's
// Dirichlet draws (Games::noise_off / noise_js layout); the action choice from the root rows of
// k_move_end into actions[g]; the test entry of mtaz_rng_dirichlet_device
void launch_rng_seed(const Dev& d, uint64_t seed_base, hipStream_t s);
void launch_noise(const Dev& d, hipStream_t s);
void launch_choose(const Dev& d, const uint16_t* codes, const uint32_t* visits, int kout, int32_t* actions, hipStream_t s);
void launch_rng_dirichlet_test(const uint32_t* seeds, const int32_t* ks, const int64_t* offs, int n_streams, int n_vec,
                               double alpha, double* out, double* tail, uint32_t* scratch, hipStream_t s);

// net modes
enum NetMode { NET_LEAVES = 0, NET_FULL_LOGITS = 1 };

}  // namespace mtaz
