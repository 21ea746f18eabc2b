// Device side of the MinitChess AlphaZero self-play engine (gfx950 / MI355X).
//
//   * rules kernels      batched legal-list / 554-bit mask / outcome / encoder
//                        (exp/environment.py:34-50, exp/policy.py:82-105)
//   * MCTS kernels       one wavefront per game: transposition-table lookup, PUCT
//                        over the children with a wave-wide first-index argmax,
//                        expansion, terminal handling, backup (exp/agent.py:41-88)
//   * network kernels    embedding+stem, 18 residual 3x3 convs on fp32 MFMA
//                        (v_mfma_f32_32x32x2_f32, exact f32 products), fused heads
//                        with a legal-only softmax (exp/policy.py:71-80, exp/agent.py:67-69)
#include <vector>

#include "engine.h"
#include "legacy_rng.h"

namespace mtaz {

static __constant__ Codec d_codec;

int dev_upload_codec(const Codec& c) {
  return hipMemcpyToSymbol(HIP_SYMBOL(d_codec), &c, sizeof(Codec)) == hipSuccess ? 0 : -1;
}

// ---------------------------------------------------------------------------------------
// wave helpers (64 lanes)
// inclusive prefix sum over the wave's 64 lanes (every lane active): DPP row shifts 1, 2, 4, 8 scan
// each 16-lane row, row broadcasts 15 and 31 carry the rows' totals (VALU only; round 5a: six
// __shfl_up steps, each an LDS permute round trip)
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15 into rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31 into rows 2, 3
  return x;
}

// one DPP step of the argmax: take the (u, i) that `ctrl` brings in where it is larger (u greater, or
// equal u and a smaller index); lanes outside row_mask bring in their own pair
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ void argmax_dpp_step(double& u, int& i) {
  const long long ub = __double_as_longlong(u);
  const int lo = (int)(uint32_t)ub, hi = (int)(ub >> 32);
  const int olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, ROW_MASK, 0xf, false);
  const int ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, ROW_MASK, 0xf, false);
  const int oi = __builtin_amdgcn_update_dpp(i, i, CTRL, ROW_MASK, 0xf, false);
  const double ou = __longlong_as_double(((long long)ohi << 32) | (long long)(uint32_t)olo);
  if (ou > u || (ou == u && oi < i)) {
    u = ou;
    i = oi;
  }
}

// the wave's argmax of u with the first index among equals (every lane active); returned uniform
__device__ __forceinline__ int wave_argmax_dpp(double u, int i) {
  argmax_dpp_step<0xb1, 0xf>(u, i);    // quad_perm [1,0,3,2]
  argmax_dpp_step<0x4e, 0xf>(u, i);    // quad_perm [2,3,0,1]
  argmax_dpp_step<0x141, 0xf>(u, i);   // row_half_mirror: each 8-lane half-row
  argmax_dpp_step<0x140, 0xf>(u, i);   // row_mirror: each 16-lane row
  argmax_dpp_step<0x142, 0xa>(u, i);   // row_bcast:15 into rows 1, 3
  argmax_dpp_step<0x143, 0xc>(u, i);   // row_bcast:31 into rows 2, 3: lane 63 holds the wave's
  return __builtin_amdgcn_readlane(i, 63);
}

__device__ __forceinline__ BB dev_apply_code(const BB& b, int code) {
  const int side = b.white ? 0 : 1;
  const uint16_t ft = d_codec.dec[side][code];
  const int from = ft & 0xff, to = ft >> 8;
  // exp/environment.py:71-76: uci4 first, else uci4+'q' -> a pawn reaching the last
  // rank always promotes to a queen, whichever duplicate code was chosen.
  const int promo = (((b.pawn >> from) & 1u) && (to / 5 == (b.white ? 5 : 0))) ? QUEEN : 0;
  return make_move(b, from, to, promo);
}

// The rule tables (knight / king / pawn attacks, rays: 1,444 B) copied into the workgroup's LDS:
// move generation looks them up per lane with lane-varying squares, which from the constant
// bank are vector loads through the texture path (tools/select_stamps.py: 58% of k_select's
// cycles went to move generation with the tables there).  Call with the one 64-lane wave of a
// 64-thread workgroup, then barrier.  All of a lane's loads are issued before its first LDS store:
// round 5a's strided loop (stride blockDim.x) compiled to a remainder loop that waited for each
// load in turn, six dependent round trips at the start of every k_select.
__device__ __forceinline__ void load_rules_lds(RuleTables* s_rt) {
  constexpr int NW = (int)(sizeof(RuleTables) / 4), PER = (NW + 63) / 64;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&d_rules);
  uint32_t* dst = reinterpret_cast<uint32_t*>(s_rt);
  const int lane = threadIdx.x & 63;
  uint32_t v[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) v[j] = lane + 64 * j < NW ? src[lane + 64 * j] : 0u;
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (lane + 64 * j < NW) dst[lane + 64 * j] = v[j];
}

// LDS scratch of one wave's move generation
struct LegalLds {
  uint16_t raw[KMAX], sorted[KMAX];
  uint16_t pm[KMAX];            // pseudo moves from | to << 8 (at most 15 x 15 = 225 < KMAX)
};

// Sorted legal codes with duplicates (exp/environment.py:48-50) computed by one wave, lane-parallel
// over pseudo moves: lane s < 30 lists the pseudo targets of its piece, the wave prefix-sums them
// into one list, then each lane tests one pseudo move (own king not attacked after it: the
// oracle's Board._gen_legal), and the legal ones are scattered with their multiplicity (a pawn
// reaching the last rank is listed once per promotion piece) and ranked by code.  The list is a
// sorted multiset, so it does not depend on the order the moves are found in.
// Must be called by all 64 lanes in uniform control flow.  Returns k or -1 (> KMAX).
__device__ int wave_legal(const BB& b, uint32_t flags, const RuleTables& RT, LegalLds& L) {
  const int lane = threadIdx.x & 63;
  const uint32_t own = b.white ? b.w : b.b;
  const int side = b.white ? 0 : 1;
  uint32_t ps = 0;
  if (lane < NSQ && ((own >> lane) & 1u)) ps = pseudo_targets(b, lane, flags, RT);
  const int cnt = popc(ps);
  const int incl = wave_incl_scan(cnt);
  const int nps = __builtin_amdgcn_readlane(incl, 63);     // <= 15 * 15: own pieces x other squares
  if (nps > KMAX) return -1;                // (unreachable from legal play; keeps L.pm in bounds)
  int off = incl - cnt;
  for (uint32_t m = ps; m; m &= m - 1) L.pm[off++] = (uint16_t)(lane | (lsb(m) << 8));
  __syncthreads();
  const int ksq0 = king_sq(b, b.white);
  int total = 0;
  for (int base = 0; base < nps; base += 64) {
    const int i = base + lane;
    int mult = 0, code = 0;
    if (i < nps) {
      const int from = L.pm[i] & 0xff, to = L.pm[i] >> 8;
      BB n = b;
      clear_sq(n, (1u << from) | (1u << to));
      set_piece(n, to, piece_type_at(b, from), b.white);
      const int k = ((b.king >> from) & 1u) ? to : ksq0;
      if (k < 0 || !attacked(n, k, !b.white, RT)) {
        mult = move_mult(b, from, to, flags);
        code = d_codec.enc[side][from * 30 + to];
      }
    }
    const int mincl = wave_incl_scan(mult);
    int o = total + mincl - mult;
    total += __builtin_amdgcn_readlane(mincl, 63);
    if (total > KMAX) return -1;
    for (int r = 0; r < mult; ++r) L.raw[o++] = (uint16_t)code;
  }
  __syncthreads();
  if (total <= 64) {
    // rank by code, then list index: lane j holds code j and reads the others with readlane (the
    // loop index is uniform), not from LDS (round 5a: one dependent LDS read per code and lane)
    const int c = lane < total ? (int)L.raw[lane] : 0xffff;
    int rank = 0;
    for (int i = 0; i < total; ++i) {
      const int o = __builtin_amdgcn_readlane(c, i);
      rank += (o < c) || (o == c && i < lane);
    }
    if (lane < total) L.sorted[rank] = (uint16_t)c;
  } else {
    for (int j = lane; j < total; j += 64) {
      const uint16_t c = L.raw[j];
      int rank = 0;
      for (int i = 0; i < total; ++i) {
        const uint16_t o = L.raw[i];
        rank += (o < c) || (o == c && i < j);
      }
      L.sorted[rank] = c;
    }
  }
  __syncthreads();
  return total;
}

// sequential legal count (one thread), used once per ply at game level
__device__ int legal_count(const BB& b, uint32_t flags) {
  const uint32_t own = b.white ? b.w : b.b;
  uint32_t m = own;
  int k = 0;
  while (m) {
    const int s = lsb(m);
    m &= m - 1;
    uint32_t tg = legal_targets(b, s, flags);
    while (tg) {
      const int to = lsb(tg);
      tg &= tg - 1;
      k += move_mult(b, s, to, flags);
    }
  }
  return k;
}

// ---------------------------------------------------------------------------------------
// rules kernels (minimum slice)
__global__ __launch_bounds__(64) void k_legal_batch(const Pos* __restrict__ pos, int n, uint32_t flags, int move_cap,
                                                    uint16_t* __restrict__ codes, int32_t* __restrict__ counts,
                                                    uint32_t* __restrict__ masks, int32_t* __restrict__ outcomes) {
  __shared__ LegalLds s_l;
  __shared__ RuleTables s_rt;
  __shared__ uint32_t s_mask[MASK_WORDS];
  const int i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  load_rules_lds(&s_rt);
  const BB b = unpack(pos[i]);
  if (lane < MASK_WORDS) s_mask[lane] = 0;
  __syncthreads();
  const int k = wave_legal(b, flags, s_rt, s_l);
  if (k < 0) {
    if (lane == 0) { counts[i] = -1; outcomes[i] = -1; }
    return;
  }
  for (int j = lane; j < k; j += 64) {
    codes[(size_t)i * KMAX + j] = s_l.sorted[j];
    atomicOr(&s_mask[s_l.sorted[j] >> 5], 1u << (s_l.sorted[j] & 31));
  }
  __syncthreads();
  if (lane < MASK_WORDS) masks[(size_t)i * MASK_WORDS + lane] = s_mask[lane];
  if (lane == 0) {
    counts[i] = k;
    outcomes[i] = outcome(b, k, in_check(b, s_rt), flags, move_cap, 1, s_rt);
  }
}

__global__ void k_encode_batch(const Pos* __restrict__ pos, int n, uint8_t* __restrict__ tokens, float* __restrict__ clocks) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const BB b = unpack(pos[i]);
  uint8_t t[60];
  encode_tokens(b, t);
  for (int j = 0; j < 60; ++j) tokens[(size_t)i * 60 + j] = t[j];
  clocks[i] = encode_clock(b);
}

// Replay memory ingest (exp/dataset.py:6-20 + the row half of collate_fn,
// exp/learner.py:23-37): row i of a packed record batch is encoded into ring slot
// (head + i) % cap: tokens + clock as k_encode_batch, the dense 554-wide pi target
// pi[code] = float32(N / N.sum()) in float64 (exp/policy.py:120), and the reward.  Legal lists
// are sorted, so a repeated code (promotions) is a run of equal codes, and the reference's
// last-write-wins assignment keeps the run's last entry: each code is written once.  One
// wavefront per row; the row is built in LDS and stored coalesced.
__global__ void k_replay_put(const Pos* __restrict__ pos, const int32_t* __restrict__ k, const int64_t* __restrict__ e0,
                             const uint16_t* __restrict__ codes, const uint32_t* __restrict__ visits,
                             const float* __restrict__ reward, int n, int64_t cap, int64_t head,
                             uint8_t* __restrict__ tokens, float* __restrict__ clocks, float* __restrict__ pi,
                             float* __restrict__ reward_out) {
  __shared__ float row[NUM_ACTIONS];
  const int i = blockIdx.x, lane = threadIdx.x;
  if (i >= n) return;
  const int64_t slot = (head + i) % cap;
  const int kk = k[i];
  const int64_t e = e0[i];
  for (int c = lane; c < NUM_ACTIONS; c += 64) row[c] = 0.f;
  uint64_t sum = 0;
  for (int j = lane; j < kk; j += 64) sum += visits[e + j];
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  __syncthreads();
  for (int j = lane; j < kk; j += 64) {
    const uint16_t c = codes[e + j];
    if (j == kk - 1 || codes[e + j + 1] != c) row[c] = (float)((double)visits[e + j] / (double)sum);
  }
  __syncthreads();
  float* out = pi + slot * NUM_ACTIONS;
  for (int c = lane; c < NUM_ACTIONS; c += 64) out[c] = row[c];
  if (lane == 0) {
    const BB b = unpack(pos[i]);
    uint8_t t[60];
    encode_tokens(b, t);
    for (int j = 0; j < 60; ++j) tokens[slot * 60 + j] = t[j];
    clocks[slot] = encode_clock(b);
    reward_out[slot] = reward[i];
  }
}

void launch_replay_put(const Pos* pos, const int32_t* k, const int64_t* e0, const uint16_t* codes,
                       const uint32_t* visits, const float* reward, int n, int64_t cap, int64_t head,
                       uint8_t* tokens, float* clocks, float* pi, float* reward_out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_replay_put, dim3(n), dim3(64), 0, s, pos, k, e0, codes, visits, reward, n, cap, head, tokens,
                     clocks, pi, reward_out);
}

void launch_legal_batch(const Pos* pos, int n, uint32_t flags, int move_cap, uint16_t* codes, int32_t* counts,
                        uint32_t* masks, int32_t* outcomes, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_legal_batch, dim3(n), dim3(64), 0, s, pos, n, flags, move_cap, codes, counts, masks, outcomes);
}

void launch_encode_batch(const Pos* pos, int n, uint8_t* tokens, float* clocks, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_encode_batch, dim3((n + 127) / 128), dim3(128), 0, s, pos, n, tokens, clocks);
}

// ---------------------------------------------------------------------------------------
// transposition table (open addressing, linear probing; one wave owns a tree at a time).
// Returns the node, or NONE with *slot = the empty slot the probe stopped at (where
// tree_insert puts the position: nothing else writes the table in between), or NONE with
// *slot = HC when the table is full.
__device__ __forceinline__ uint32_t tree_find(const Trees& T, int t, const Pos& p, uint32_t* slot) {
  const uint32_t mask = (uint32_t)T.HC - 1;
  const uint32_t* ht = T.hash + (size_t)t * T.HC;
  const Pos* np = T.node_pos + (size_t)t * T.NC;
  uint32_t h = pos_hash(p) & mask;
  for (int probe = 0; probe < T.HC; ++probe) {
    const uint32_t v = ht[h];
    if (v == 0) {
      *slot = h;
      return NONE;
    }
    if (pos_eq(np[v - 1], p)) return v - 1;
    h = (h + 1) & mask;
  }
  *slot = (uint32_t)T.HC;
  return NONE;
}

// tree_find with its first probe done by the caller: v = the table's word at slot h (the position's
// home slot), vp = the position of node v - 1 (read when v != 0)
__device__ __forceinline__ uint32_t tree_find_first(const Trees& T, int t, const Pos& p, uint32_t h, uint32_t v,
                                                    const Pos& vp, uint32_t* slot) {
  if (v == 0) {
    *slot = h;
    return NONE;
  }
  if (pos_eq(vp, p)) return v - 1;
  const uint32_t mask = (uint32_t)T.HC - 1;
  const uint32_t* ht = T.hash + (size_t)t * T.HC;
  const Pos* np = T.node_pos + (size_t)t * T.NC;
  for (int probe = 1; probe < T.HC; ++probe) {
    h = (h + 1) & mask;
    const uint32_t w = ht[h];
    if (w == 0) {
      *slot = h;
      return NONE;
    }
    if (pos_eq(np[w - 1], p)) return w - 1;
  }
  *slot = (uint32_t)T.HC;
  return NONE;
}

// single lane; `n_nodes` = the tree's node count (read at kernel start: only this wave adds nodes)
__device__ uint32_t tree_insert(const Trees& T, int t, const Pos& p, uint32_t slot, uint32_t n_nodes, int32_t* err) {
  if (n_nodes >= (uint32_t)T.NC) {
    atomicOr(err, ERR_NODES);
    return NONE;
  }
  if (slot >= (uint32_t)T.HC) {
    atomicOr(err, ERR_HASH);
    return NONE;
  }
  T.n_nodes[t] = n_nodes + 1;
  T.node_pos[(size_t)t * T.NC + n_nodes] = p;
  T.hash[(size_t)t * T.HC + slot] = n_nodes + 1;
  return n_nodes;
}

// exp/agent.py:47-52: for (node, a) in reversed(chain): value = -value;
// Q[a] = (N[a]*Q[a] + value) / (N[a] + 1); N[a] += 1.  Exact fp64, no contraction.  The levels
// are independent (level d sees (-1)^(depth - d) v, and a chain never repeats a node: the
// fullmove number grows along it), so lane d updates level d.  Call with all lanes of a wave.
__device__ __forceinline__ void backup_path(const Trees& T, int t, const uint32_t* pn, const uint32_t* pe, int depth,
                                            double v, int lane) {
#pragma clang fp contract(off)
  const size_t nbase = (size_t)t * T.NC;
  for (int d = lane; d < depth; d += 64) {
    const double vd = ((depth - d) & 1) ? -v : v;
    const size_t e = pe[d];
    const uint32_t Ni = T.e_N[e];
    const double N = (double)Ni;
    const double Q = T.e_Q[e];
    const double prod = N * Q;
    const double num = prod + vd;
    T.e_Q[e] = num / (N + 1.0);
    T.e_N[e] = Ni + 1;
    T.node_hdr[nbase + pn[d]].sumN += 1;
  }
}

__global__ void k_reset_trees(Trees T, const int32_t* __restrict__ trees, int ntrees, int all_trees) {
  const int j = blockIdx.y;
  if (j >= ntrees) return;
  const int t = trees[j];
  uint32_t* ht = T.hash + (size_t)t * T.HC;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < T.HC; i += gridDim.x * blockDim.x) ht[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    T.n_nodes[t] = 0;
    T.n_edges[t] = 0;
    if (all_trees && j == 0) *T.pool_used = 0;
  }
}

void launch_reset_trees(const Dev& d, const int32_t* trees, int ntrees, bool all_trees, hipStream_t s) {
  if (ntrees <= 0) return;
  hipLaunchKernelGGL(k_reset_trees, dim3(4, ntrees), dim3(256), 0, s, d.tr, trees, ntrees, all_trees ? 1 : 0);
}

// Move start: does the agent's table already hold the root (exp/agent.py:57)?  The host
// needs k and "root is new" to draw exactly sims - root_new Dirichlet vectors (:81-82).
// Also leaves the root's node index as k_select's hint (Games::root_node).
__global__ __launch_bounds__(64) void k_move_begin(Dev D) {
  __shared__ LegalLds s_l;
  __shared__ RuleTables s_rt;
  const int g = blockIdx.x, lane = threadIdx.x;
  if (lane == 0) {   // a move starts with no simulation begun and no leaf pending
    D.gm.simc[g] = 0;
    D.lf.gnode[g] = NONE;
  }
  if (!D.gm.active[g]) {
    if (lane == 0) { D.gm.root_k[g] = 0; D.gm.root_new[g] = 0; }
    return;
  }
  const int t = 2 * g + D.gm.agent[g];
  const Pos root = D.gm.root[g];
  uint32_t slot;
  const uint32_t n = tree_find(D.tr, t, root, &slot);
  if (lane == 0) D.gm.root_node[g] = n;
  if (n != NONE) {
    if (lane == 0) {
      const NodeHdr hd = D.tr.node_hdr[(size_t)t * D.tr.NC + n];
      if (hdr_term(hd)) atomicOr(D.pr.err, ERR_ROOT);
      D.gm.root_k[g] = hdr_k(hd);
      D.gm.root_new[g] = 0;
    }
    return;
  }
  load_rules_lds(&s_rt);
  const BB b = unpack(root);
  __syncthreads();
  const int k = wave_legal(b, D.pr.flags, s_rt, s_l);
  if (lane == 0) {
    if (k <= 0) atomicOr(D.pr.err, k < 0 ? ERR_KMAX : ERR_ROOT);
    D.gm.root_k[g] = k;
    D.gm.root_new[g] = 1;
  }
}

void launch_move_begin(const Dev& d, hipStream_t s) {
  hipLaunchKernelGGL(k_move_begin, dim3(d.pr.G), dim3(64), 0, s, d);
}

// One simulation for every active game (exp/agent.py:41-88): descend from the root by
// PUCT until an unvisited node (expand: terminal -> back up, else queue the leaf for
// the network) or a stored terminal (back up -terminal, the reference's sign quirk).
// The descent follows node indices, not hash lookups: the root's from Games::root_node
// (checked against the node's stored position and the tree's node count, so a stale hint
// only costs a lookup), a child's from its edge (Trees::e_child, filled the first time the
// edge is followed).  The position is still carried along (the leaf's network input, the
// lookup of a child not yet linked).  Per level: one node-header load, then one pass over
// the children's P, Q, N, code and child index.
#ifdef MTAZ_NET_DIAG
// diagnostic library only: k_select phase cycles per game, summed over launches (plain adds, one
// wave per game per launch: atomics on shared counters would themselves serialise the kernel)
// [waves, find, select, legal, outcome, insert/init/backup, total, depth]
constexpr int SEL_STAMP_GAMES = 65536;
__device__ unsigned long long g_sel_cyc[SEL_STAMP_GAMES * 8];
#define SEL_T(i)                                      \
  {                                                   \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    sel_acc[i] += t_ - sel_t;                         \
    sel_t = t_;                                       \
  }
#define SEL_FIN()                                                                        \
  if (lane == 0 && g < SEL_STAMP_GAMES) {                                                \
    sel_acc[6] = __builtin_amdgcn_s_memtime() - sel_t0;                                  \
    sel_acc[0] = 1;                                                                      \
    sel_acc[7] = depth;                                                                  \
    for (int i_ = 0; i_ < 8; ++i_) g_sel_cyc[(size_t)g * 8 + i_] += sel_acc[i_];         \
  }
#else
#define SEL_T(i)
#define SEL_FIN()
#endif

__global__ __launch_bounds__(64) void k_select(Dev D, int sim, int defer) {
#pragma clang fp contract(off)
  __shared__ LegalLds s_l;
  __shared__ RuleTables s_rt;
  const int g = blockIdx.x, lane = threadIdx.x;
  // One round of loads for the game's words (the gates, agent, root, root-node hint, noise
  // address, both tables' counters) and the rule tables.  Round 5a read the gates one behind
  // another and the tree's counters behind the agent: five dependent round trips before the root's
  // header, about 1.9 us each even on an idle chip (tools/select_stamps.py at 256 games).
  // (the game's active byte read as part of its aligned word: a byte load went out, and was waited
  // for, ahead of the other loads)
  const bool act = ((reinterpret_cast<const uint32_t*>(D.gm.active)[g >> 2] >> (8 * (g & 3))) & 0xffu) != 0;
  const uint32_t pend = defer ? D.lf.gnode[g] : NONE;
  const int sc = defer ? D.gm.simc[g] : 0;
  const int st0 = defer ? D.gm.stot[g] : 0;
  const int ag = D.gm.agent[g];
  Pos pos = D.gm.root[g];
  uint32_t n = D.gm.root_node[g];
  const int64_t noff = D.gm.noise_off[g];
  const int32_t njs = D.gm.noise_js[g], rnew = D.gm.root_new[g];
  const uint2 nn2 = *reinterpret_cast<const uint2*>(D.tr.n_nodes + 2 * g);   // trees 2g, 2g + 1
  const uint2 ne2 = *reinterpret_cast<const uint2*>(D.tr.n_edges + 2 * g);
  load_rules_lds(&s_rt);
  // the values are needed here, so every load above is issued before the gates branch (the
  // compiler otherwise sinks each load into the branch that uses it, one round trip after another)
  asm volatile("" ::"v"((uint32_t)act), "v"(pend), "v"(sc), "v"(st0), "v"(ag), "v"(pos.sq[0]), "v"(pos.sq[1]), "v"(pos.sq[2]),
               "v"(pos.sq[3]), "v"(pos.info), "v"(n), "v"(noff), "v"(njs), "v"(rnew), "v"(nn2.x), "v"(nn2.y),
               "v"(ne2.x), "v"(ne2.y));
  if (!defer) {
    if (lane == 0) {
      D.lf.gnode[g] = NONE;
      D.lf.ghit[g] = 0;
    }
    if (!act) return;
  } else {
    // deferred-tail play: the game's own next simulation, unless its last leaf is still pending
    // (deferred by k_leaf_compact) or it has started all of them.  A game's simulations run in
    // order, one at a time, exactly as in lockstep; only the wave each one runs in moves.
    if (lane == 0) D.lf.ghit[g] = 0;
    if (!act || pend != NONE) return;
    if (sc >= D.pr.sims) return;
    if (lane == 0) {
      D.gm.simc[g] = sc + 1;
      D.gm.stot[g] = st0 + 1;
    }
    sim = sc;
  }
#ifdef MTAZ_NET_DIAG
  unsigned long long sel_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long sel_t0 = __builtin_amdgcn_s_memtime();
  unsigned long long sel_t = sel_t0;
#endif
  const Trees& T = D.tr;
  const int t = 2 * g + ag;
  const size_t nbase = (size_t)t * T.NC;
  const uint32_t ebase = (uint32_t)t * (uint32_t)T.EC;   // the tree's own edge region
  uint32_t* pn = D.gm.path_node + (size_t)g * D.gm.DMAX;
  uint32_t* pe = D.gm.path_edge + (size_t)g * D.gm.DMAX;
  const uint32_t n_nodes = ag ? nn2.y : nn2.x, n_edges = ag ? ne2.y : ne2.x;
  int depth = 0;
  // this simulation's Dirichlet vector (read at the root only)
  const double* noise = D.gm.noise + noff + (int64_t)(sim - rnew) * njs;
  // the hinted node's position and header in one round trip (the header is used only if the
  // position matches)
  const size_t nh = nbase + (n < (uint32_t)T.NC ? n : 0u);
  const Pos hpos = T.node_pos[nh];
  NodeHdr hd_pre = T.node_hdr[nh];
  if (n >= n_nodes || !pos_eq(hpos, pos)) n = NONE;
  bool linked = n != NONE;      // n is pos's node, known without a lookup
  bool pre = linked;            // hd_pre is n's header
  uint32_t pedge = NONE;        // the edge that led here (tree-local), NONE at the root
  __syncthreads();
  for (;;) {
    if (!linked) {
      // The position's first probes in this tree's table, the game's other table (memo >= 1) and
      // the batch memo (memo 2) go out in one round of loads, the probed slots' positions in the
      // next (round 5a: each lookup behind the previous one, six round trips before an expansion
      // that misses all three); a collision continues the probe sequence as tree_find does.
      const uint32_t hp = pos_hash(pos), h0 = hp & ((uint32_t)T.HC - 1);
      const bool memo1 = D.pr.memo != 0, memo2 = D.pr.memo >= 2 && D.bm.cap != 0;
      const uint32_t v0 = T.hash[(size_t)t * T.HC + h0];
      const uint32_t v1 = memo1 ? T.hash[(size_t)(t ^ 1) * T.HC + h0] : 0u;
      const uint32_t hb = memo2 ? (hp & (D.bm.cap - 1)) : 0u;
      const uint32_t bs = memo2 ? D.bm.state[hb] : 0u;
      Pos bkey{}, p0{}, p1{};
      if (memo2) bkey = D.bm.key[hb];
      if (v0 != 0u) p0 = T.node_pos[nbase + v0 - 1];
      if (v1 != 0u) p1 = T.node_pos[(size_t)(t ^ 1) * T.NC + v1 - 1];
      uint32_t slot;
      n = tree_find_first(T, t, pos, h0, v0, p0, &slot);
      SEL_T(1);
      if (n == NONE) {
        // ---- expansion (exp/agent.py:57-73) ----
        // Leaf memo (Params::memo): the game's other table may hold this position already; its
        // legal list, terminal value or network priors and value are then those a fresh
        // expansion would compute (rules and network are functions of the position alone), and
        // the simulation backs up here instead of queueing a leaf.  Tree t ^ 1 is idle during
        // tree t's search (the agents alternate by ply), so it is read without synchronisation.
        // With the batch memo (Params::memo 2), a position another game evaluated in an earlier
        // simulation of this play comes from the BatchMemo the same way.
        uint32_t m = NONE;
        NodeHdr mh{0u, 0u, 0u, 0.0f};
        const uint16_t* msrc_code = nullptr;
        const float* msrc_P = nullptr;
        uint8_t mkind = 0;   // 1 = the game's other table, 2 = the batch memo
        if (memo1) {
          uint32_t s2;
          m = tree_find_first(T, t ^ 1, pos, h0, v1, p1, &s2);
          if (m != NONE) {
            mkind = 1;
            mh = T.node_hdr[(size_t)(t ^ 1) * T.NC + m];
            msrc_code = T.e_code + mh.e0;
            msrc_P = T.e_P + mh.e0;
          } else if (memo2) {
            const BatchMemo& B = D.bm;
            const uint32_t mask = B.cap - 1;
            uint32_t h = hb;
            for (uint32_t probe = 0; probe < MEMO_PROBES; ++probe, h = (h + 1) & mask) {
              if ((probe ? B.state[h] : bs) == 0u) break;
              if (pos_eq(probe ? B.key[h] : bkey, pos)) {
                m = h;
                mkind = 2;
                mh = NodeHdr{0u, 0u, (uint32_t)B.k[h], B.v[h]};
                msrc_code = B.codes + (size_t)h * MEMO_K;
                msrc_P = B.P + (size_t)h * MEMO_K;
                break;
              }
            }
          }
        }
        int k;
        bool term;
        float tv;   // terminal: -reward (-1 or -0); memo hit: the stored leaf value
        if (m != NONE) {
          k = hdr_k(mh);
          term = hdr_term(mh);
          tv = mh.tval;
        } else {
          const BB b = unpack(pos);
          k = wave_legal(b, D.pr.flags, s_rt, s_l);
          SEL_T(3);
          if (k < 0) {
            if (lane == 0) atomicOr(D.pr.err, ERR_KMAX);
            return;
          }
          const int oc = outcome(b, k, in_check(b, s_rt), D.pr.flags, D.pr.move_cap, 1, s_rt);
          term = oc != ONGOING;
          tv = (oc == DECISIVE) ? -1.0f : -0.0f;
        }
        SEL_T(4);
        uint32_t nn = NONE, ne0 = 0;
        if (lane == 0) {
          nn = tree_insert(T, t, pos, slot, n_nodes, D.pr.err);
          if (nn != NONE && !term) {
            if (n_edges + (uint32_t)k <= (uint32_t)T.EC) {   // the tree's own region
              ne0 = ebase + n_edges;
              T.n_edges[t] = n_edges + k;
            } else {                                          // spill to the shared pool
              const uint32_t q = atomicAdd(T.pool_used, (uint32_t)k);
              if (q + (uint32_t)k <= T.pool_cap) {
                ne0 = T.pool_base + q;
              } else {
                // the pool is exhausted: the call fails (ERR_EDGES), but the node is already in the
                // hash; until the move ends, later visits must find a valid header, not whatever
                // the slot held (an earlier play's edge range, possibly beyond a smaller pool):
                // a terminal of value 0 backs up harmlessly
                T.node_hdr[nbase + nn] = NodeHdr{0u, 0u, HDR_TERM, 0.0f};
                atomicOr(D.pr.err, ERR_EDGES);
                nn = NONE;
              }
            }
          }
          if (nn != NONE) {
            if (term) {
              T.node_hdr[nbase + nn] = NodeHdr{0u, 0u, HDR_TERM, tv};
            } else {
              T.node_hdr[nbase + nn] = NodeHdr{ne0, 0u, (uint32_t)k, m != NONE ? tv : 0.0f};
              if (m == NONE) {
                D.lf.gnode[g] = nn;
                D.lf.gpos[g] = pos;
                D.gm.path_len[g] = depth;
              } else {
                D.lf.ghit[g] = mkind;
              }
            }
            if (pedge != NONE) T.e_child[pedge] = nn;
            else D.gm.root_node[g] = nn;
          }
        }
        nn = (uint32_t)__builtin_amdgcn_readlane((int)nn, 0);   // lane 0 decided (every lane active)
        ne0 = (uint32_t)__builtin_amdgcn_readlane((int)ne0, 0);
        if (nn != NONE) {
          if (!term) {
            for (int c = lane; c < k; c += 64) {
              const size_t e = (size_t)ne0 + c;
              T.e_code[e] = m != NONE ? msrc_code[c] : s_l.sorted[c];
              T.e_P[e] = m != NONE ? msrc_P[c] : 0.f;
              T.e_Q[e] = 0.0;
              T.e_N[e] = 0;
              T.e_child[e] = NONE;
            }
            if (m != NONE) backup_path(T, t, pn, pe, depth, (double)tv, lane);   // exp/agent.py:72
          } else {
            backup_path(T, t, pn, pe, depth, (double)tv, lane);                  // exp/agent.py:59-63
          }
        }
        SEL_T(5);
        SEL_FIN();
        return;
      }
      // found by lookup (a transposition, or the root without a valid hint): link it
      if (lane == 0) {
        if (pedge != NONE) T.e_child[pedge] = n;
        else D.gm.root_node[g] = n;
      }
    }
    const NodeHdr hd = pre ? hd_pre : T.node_hdr[nbase + n];
    pre = false;
    if (hdr_term(hd)) {
      backup_path(T, t, pn, pe, depth, -(double)hd.tval, lane);
      SEL_T(5);
      SEL_FIN();
      return;
    }
    // ---- selection (exp/agent.py:79-85) ----
    const uint32_t e0 = hd.e0;
    const int k = hdr_k(hd);
    const uint32_t S = hd.sumN;
    if (S >= (uint32_t)D.pr.sqrt_n) {
      if (lane == 0) atomicOr(D.pr.err, ERR_SQRT);
      return;
    }
    const double sq = D.pr.sqrt_tab[S];
    const bool root = depth == 0;
    double best_u = -__builtin_inf();
    int best_i = 0x7fffffff;
    uint32_t best_cc = 0;   // winner's code | linked child (the child index in a second word)
    uint32_t best_ch = NONE;
    for (int c = lane; c < k; c += 64) {
      const size_t e = (size_t)e0 + c;
      const float Pf = T.e_P[e];
      const double Q = T.e_Q[e];
      const double N = (double)T.e_N[e];
      const uint32_t code = T.e_code[e], child = T.e_child[e];
      double tt;
      if (root) {
        // P = 0.75*P (float32) + 0.25*dirichlet (float64)  -> float64
        const float p75 = 0.75f * Pf;
        const double pp = (double)p75 + 0.25 * noise[c];
        tt = (D.pr.cpuct * pp) * sq;
      } else if (D.pr.cast_mode == 2) {
        const float cp = D.pr.cpuct_f * Pf;       // float32 array * python scalar
        tt = (double)cp * sq;                     // * np.float64 scalar -> float64 (NEP 50)
      } else {
        const float cp = D.pr.cpuct_f * Pf;
        tt = (double)(cp * (float)sq);            // numpy 1.x: stays float32
      }
      double u = Q + tt / (1.0 + N);
      u = u != u ? __builtin_inf() : u;   // numpy's argmax takes the first NaN as the maximum
      if (u > best_u) { best_u = u; best_i = c; best_cc = code; best_ch = child; }
    }
    // wave argmax of (u, first index) by DPP steps (quad permutes, half-row and row mirrors, row
    // broadcasts 15 and 31: VALU only, the wave's winner in lane 63), then the winner's code and
    // child read from the lane that held it (round 4: five ds_bpermute shuffles per butterfly step,
    // six steps).  The order (u descending, index ascending) is total, so every reduction tree
    // gives the butterfly's winner.
    const int a = wave_argmax_dpp(best_u, best_i);
    if ((unsigned)a >= (unsigned)k) {   // (no child compared above: never with the NaN rule; no edge read past k)
      if (lane == 0) atomicOr(D.pr.err, ERR_PUCT);
      return;
    }
    best_cc = (uint32_t)__builtin_amdgcn_readlane((int)best_cc, a & 63);
    best_ch = (uint32_t)__builtin_amdgcn_readlane((int)best_ch, a & 63);
    if (depth >= D.gm.DMAX) {
      if (lane == 0) atomicOr(D.pr.err, ERR_DEPTH);
      return;
    }
    if (lane == 0) {
      pn[depth] = n;
      pe[depth] = e0 + a;
    }
    ++depth;
    pedge = e0 + a;
    pos = pack(dev_apply_code(unpack(pos), (int)best_cc));
    n = best_ch;
    linked = n != NONE;
    SEL_T(2);
  }
}

// a position as five words in registers (k_leaf_compact): i < 0 gives zeros
__device__ __forceinline__ void load_pos_words(uint32_t (&w)[5], const Pos* __restrict__ src, int i) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(src + (i < 0 ? 0 : i));
#pragma unroll
  for (int f = 0; f < 5; ++f) w[f] = i < 0 ? 0u : q[f];
}
__device__ __forceinline__ void store_pos_words(Pos* __restrict__ dst, int i, const uint32_t (&w)[5]) {
  uint32_t* q = reinterpret_cast<uint32_t*>(dst + i);
#pragma unroll
  for (int f = 0; f < 5; ++f) q[f] = w[f];
}

// The leaf batch: one workgroup; per chunk of 4,096 games thread i holds games 4i..4i+3 in registers
// (their leaf, agent and position in one round of loads: loads placed after the stores would wait
// for them), a block scan of the per-thread counts places its leaves.  Classic play lists the
// leaves in game order.  Deferred-tail play (defer) lists them by lag, largest first, game order
// within a lag (lag = waves since the game selected the leaf's simulation: a pending leaf of an
// earlier wave comes before the new ones), and with `cut` evaluates only the whole rounds of
// `round` leaves (4 boards x the CUs: the network's full rounds), the rest staying pending.
// Also logs the evaluated count and the memo hits of the game and batch memos (count_log[0..2]).
__global__ __launch_bounds__(1024) void k_leaf_compact(Dev D, int32_t* __restrict__ count_log, int wave, int defer,
                                                       int cut, int round) {
  constexpr int PER = 4, NBK = 4;
  __shared__ int s_w[16];
  __shared__ int s_w2[16][2];
  __shared__ int s_hits[2];
  __shared__ int s_bk[NBK];   // leaves per lag bucket (pass 1), then the bucket's next slot
  __shared__ int s_smax, s_smin;
  const int G = D.pr.G, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const bool ahead = D.pr.lag_order == 0;   // buckets by simulations ahead of the least advanced leaf
  if (tid < 2) s_hits[tid] = 0;
  if (tid < NBK) s_bk[tid] = 0;
  if (tid == 0) {
    s_smax = 0;
    s_smin = 0x7fffffff;
  }
  __syncthreads();
  if (defer && G <= 1024 * PER) {
    // deferred-tail play, one chunk (G <= 4,096): every game's leaf, agent, position and lag loaded
    // once into registers; block reductions give the most advanced leaf and the bucket sizes, then
    // one block scan per bucket places the leaves
    const int g0 = tid * PER;
    uint32_t nd[PER];
    int ag[PER], sc[PER], bk[PER];
    uint32_t ps[PER][5];   // positions as words (an array of Pos compiles to scratch copies)
    int hits = 0, bhits = 0, m = 0, mn = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const bool in = g0 + j < G;
      nd[j] = in ? D.lf.gnode[g0 + j] : NONE;
      ag[j] = in ? D.gm.agent[g0 + j] : 0;
      load_pos_words(ps[j], D.lf.gpos, in ? g0 + j : -1);
      sc[j] = in ? D.gm.stot[g0 + j] - 1 : 0;   // (the play's simulation count: games may be on different moves)
      const int hk = in ? (int)D.lf.ghit[g0 + j] : 0;
      hits += hk == 1;
      bhits += hk == 2;
      if (nd[j] != NONE) {
        m = max(m, sc[j]);
        mn = min(mn, sc[j]);
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      m = max(m, __shfl_xor(m, o, 64));
      mn = min(mn, __shfl_xor(mn, o, 64));
    }
    if (lane == 0) {
      atomicMax(&s_smax, m);
      atomicMin(&s_smin, mn);
    }
    __syncthreads();
    const int smx = s_smax, smn = s_smin;
    // the thread's leaves per bucket and its memo hits, 16-bit fields of three words (every field's
    // block total is at most G <= 4,096, so no field carries into the next): one block scan of the
    // three words places every bucket's leaves and gives the totals (round 5a: one block scan per
    // bucket and a store pass per bucket, 22 us per launch)
    uint32_t w01 = 0, w23 = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (ahead) {
        const int d = sc[j] - smn;
        bk[j] = d < NBK - 1 ? (d > 0 ? d : 0) : NBK - 1;
      } else {
        const int lag = smx - sc[j];
        bk[j] = NBK - 1 - (lag < NBK - 1 ? (lag > 0 ? lag : 0) : NBK - 1);
      }
      if (nd[j] != NONE) {
        const uint32_t one = 1u << (16 * (bk[j] & 1));
        if (bk[j] < 2) w01 += one;
        else w23 += one;
      }
    }
    const uint32_t wh = (uint32_t)hits | ((uint32_t)bhits << 16);
    const uint32_t i01 = (uint32_t)wave_incl_scan((int)w01), i23 = (uint32_t)wave_incl_scan((int)w23);
    const uint32_t ih = (uint32_t)wave_incl_scan((int)wh);
    if (lane == 63) {
      s_w[w] = (int)i01;
      s_w2[w][0] = (int)i23;
      s_w2[w][1] = (int)ih;
    }
    __syncthreads();
    uint32_t p01 = i01 - w01, p23 = i23 - w23, t01 = 0, t23 = 0, th = 0;   // exclusive prefixes, totals
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t x01 = (uint32_t)s_w[i], x23 = (uint32_t)s_w2[i][0];
      p01 += i < w ? x01 : 0u;
      p23 += i < w ? x23 : 0u;
      t01 += x01;
      t23 += x23;
      th += (uint32_t)s_w2[i][1];
    }
    const int tot0 = (int)(t01 & 0xffffu), tot1 = (int)(t01 >> 16), tot2 = (int)(t23 & 0xffffu);
    const int total = tot0 + tot1 + tot2 + (int)(t23 >> 16);
    int sb[NBK] = {(int)(p01 & 0xffffu), tot0 + (int)(p01 >> 16), tot0 + tot1 + (int)(p23 & 0xffffu),
                   tot0 + tot1 + tot2 + (int)(p23 >> 16)};   // the thread's next slot in each bucket
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (nd[j] != NONE) {
        int slot = sb[0];
#pragma unroll
        for (int q = 1; q < NBK; ++q) slot = bk[j] == q ? sb[q] : slot;
#pragma unroll
        for (int q = 0; q < NBK; ++q) sb[q] += bk[j] == q;
        const int g = g0 + j;
        D.lf.game[slot] = g;
        D.lf.tree[slot] = 2 * g + ag[j];
        D.lf.node[slot] = nd[j];
        store_pos_words(D.lf.pos, slot, ps[j]);
      }
    }
    if (tid == 0) {
      const int rem = round > 0 ? total % round : 0;
      const int n = (cut && round > 0 && total >= round && (cut == 2 || rem <= 3 * (round / 4))) ? total - rem : total;
      *D.lf.count = n;
      if (count_log) {
        count_log[0] = n;
        count_log[1] = (int)(th & 0xffffu);
        count_log[2] = (int)(th >> 16);
      }
    }
    return;
  }
  if (defer) {   // pass 0: the most and the least advanced leaf's simulation index
    int m = 0, mn = 0x7fffffff;
    for (int g = tid; g < G; g += 1024)
      if (D.lf.gnode[g] != NONE) {
        m = max(m, D.gm.stot[g] - 1);
        mn = min(mn, D.gm.stot[g] - 1);
      }
    for (int o = 32; o > 0; o >>= 1) {
      m = max(m, __shfl_xor(m, o, 64));
      mn = min(mn, __shfl_xor(mn, o, 64));
    }
    if (lane == 0) {
      atomicMax(&s_smax, m);
      atomicMin(&s_smin, mn);
    }
    __syncthreads();
  }
  // lag bucket of game g's leaf, 0 = listed first: the least advanced leaves (round 5: the largest
  // lag behind the most advanced leaf)
  const int smax = s_smax, smin = s_smin;
  auto bucket = [&](int g) {
    if (!defer) return 0;
    if (ahead) {
      const int d = (D.gm.stot[g] - 1) - smin;
      return d < NBK - 1 ? (d > 0 ? d : 0) : NBK - 1;
    }
    const int lag = smax - (D.gm.stot[g] - 1);
    return NBK - 1 - (lag < NBK - 1 ? (lag > 0 ? lag : 0) : NBK - 1);
  };
  if (defer) {   // pass 1: leaves per bucket
    int cb[NBK] = {0, 0, 0, 0};
    for (int g = tid; g < G; g += 1024)
      if (D.lf.gnode[g] != NONE) {
        const int b = bucket(g);
#pragma unroll
        for (int q = 0; q < NBK; ++q) cb[q] += b == q;
      }
#pragma unroll
    for (int q = 0; q < NBK; ++q) {
      int x = cb[q];
      for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
      if (lane == 0 && x) atomicAdd(&s_bk[q], x);
    }
    __syncthreads();
    if (tid == 0) {   // exclusive prefix: each bucket's first slot
      int acc = 0;
      for (int q = 0; q < NBK; ++q) {
        const int x = s_bk[q];
        s_bk[q] = acc;
        acc += x;
      }
    }
    __syncthreads();
  }
  int base = 0, hits = 0, bhits = 0;
  for (int c0 = 0; c0 < G; c0 += 1024 * PER) {
    const int g0 = c0 + tid * PER;
    uint32_t nd[PER];
    int ag[PER], bk[PER];
    uint32_t ps[PER][5];   // positions as words (an array of Pos compiles to scratch copies)
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const bool in = g0 + j < G;
      nd[j] = in ? D.lf.gnode[g0 + j] : NONE;
      ag[j] = in ? D.gm.agent[g0 + j] : 0;
      load_pos_words(ps[j], D.lf.gpos, in ? g0 + j : -1);
      bk[j] = (in && nd[j] != NONE) ? bucket(g0 + j) : 0;
      const int hk = in ? (int)D.lf.ghit[g0 + j] : 0;
      hits += hk == 1;
      bhits += hk == 2;
    }
    // one block scan per bucket (classic play: bucket 0 only)
    for (int q = 0; q < (defer ? NBK : 1); ++q) {
      int c = 0;
#pragma unroll
      for (int j = 0; j < PER; ++j) c += nd[j] != NONE && bk[j] == q;
      const int incl = wave_incl_scan(c);
      if (lane == 63) s_w[w] = incl;
      __syncthreads();
      int slot = (defer ? s_bk[q] : base) + incl - c, tot = 0;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int x = s_w[i];
        slot += i < w ? x : 0;
        tot += x;
      }
      __syncthreads();   // s_w is rewritten by the next scan, s_bk read
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if (nd[j] != NONE && bk[j] == q) {
          const int g = g0 + j;
          D.lf.game[slot] = g;
          D.lf.tree[slot] = 2 * g + ag[j];
          D.lf.node[slot] = nd[j];
          store_pos_words(D.lf.pos, slot, ps[j]);
          ++slot;
        }
      }
      if (defer) {
        if (tid == 0) s_bk[q] += tot;
        __syncthreads();
      }
      base += tot;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    hits += __shfl_xor(hits, o, 64);
    bhits += __shfl_xor(bhits, o, 64);
  }
  if (lane == 0 && hits) atomicAdd(&s_hits[0], hits);
  if (lane == 0 && bhits) atomicAdd(&s_hits[1], bhits);
  __syncthreads();
  if (tid == 0) {
    // the evaluated count: every leaf, or (cut) the whole rounds of them when there is one and the
    // rest would have gone to a tail launch (at most 3 boards per CU); a remainder above that runs
    // as a partial round of 4-board workgroups in the main launch, which costs about what a full
    // round does for nearly a round of boards, and is evaluated now
    // (cut 2: every remainder waits, the partial rounds too)
    const int rem = round > 0 ? base % round : 0;
    const int n = (cut && round > 0 && base >= round && (cut == 2 || rem <= 3 * (round / 4))) ? base - rem : base;
    *D.lf.count = n;
    if (count_log) {
      count_log[0] = n;
      count_log[1] = s_hits[0];
      count_log[2] = s_hits[1];
    }
  }
}

// one simulation's selection: k_select, then the leaf list and the evaluated count
void launch_select(const Dev& d, int sim, hipStream_t s, int32_t* count_log, hipEvent_t ev_mid, int defer, int cut,
                   int round) {
  hipLaunchKernelGGL(k_select, dim3(d.pr.G), dim3(64), 0, s, d, sim, defer);
  if (ev_mid) (void)hipEventRecord(ev_mid, s);
  hipLaunchKernelGGL(k_leaf_compact, dim3(1), dim3(1024), 0, s, d, count_log, sim, defer, cut, round);
}

// waves a deferred-tail move still needs: max over active games of (sims not started) + (a leaf pending)
__global__ __launch_bounds__(256) void k_remaining(Dev D, int32_t* __restrict__ out) {
  __shared__ int s_m;
  if (threadIdx.x == 0) s_m = 0;
  __syncthreads();
  int m = 0;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < D.pr.G; g += gridDim.x * 256)
    if (D.gm.active[g]) {
      const int r = (D.pr.sims - D.gm.simc[g]) + (D.lf.gnode[g] != NONE ? 1 : 0);
      m = r > m ? r : m;
    }
  for (int o = 32; o > 0; o >>= 1) {
    const int x = __shfl_xor(m, o, 64);
    m = x > m ? x : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(&s_m, m);
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(out, s_m);
}

void launch_remaining(const Dev& d, int32_t* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, 4, s);
  hipLaunchKernelGGL(k_remaining, dim3(16), dim3(256), 0, s, d, out);
}

#ifdef MTAZ_NET_DIAG
int diag_select_stamps(unsigned long long* out8, int reset) {
  std::vector<unsigned long long> v((size_t)SEL_STAMP_GAMES * 8);
  if (hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_sel_cyc), v.size() * 8) != hipSuccess) return -1;
  if (out8) {
    for (int i = 0; i < 8; ++i) out8[i] = 0;
    for (size_t g = 0; g < (size_t)SEL_STAMP_GAMES; ++g)
      for (int i = 0; i < 8; ++i) out8[i] += v[g * 8 + i];
  }
  if (reset) {
    std::fill(v.begin(), v.end(), 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_sel_cyc), v.data(), v.size() * 8) != hipSuccess) return -1;
  }
  return 0;
}
#endif

// Leaf expansion finish + backup (exp/agent.py:68-72): store P, back up v.  One wave per leaf:
// lanes copy the priors and update one path level each.
__global__ __launch_bounds__(256) void k_backup(Dev D) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= *D.lf.count) return;
  const Trees& T = D.tr;
  const int g = D.lf.game[i], t = D.lf.tree[i];
  const uint32_t n = D.lf.node[i];
  const size_t nbase = (size_t)t * T.NC;
  const uint32_t* pn = D.gm.path_node + (size_t)g * D.gm.DMAX;
  const uint32_t* pe = D.gm.path_edge + (size_t)g * D.gm.DMAX;
  // one round of loads for what depends only on the leaf's slot and game: its header, value and
  // first 64 priors, the path length and the lane's path level (read before the length is known:
  // a level past it is not used), so that the backup's loads go out ahead of the memo's CAS chain
  // (round 5a: header, priors, memo, then the path, each behind the previous)
  const NodeHdr hd = T.node_hdr[nbase + n];
  const float vf = D.lf.v[i];
  const int depth = D.gm.path_len[g];
  const bool lvl = lane < D.gm.DMAX;
  const uint32_t pe0 = lvl ? pe[lane] : 0u, pn0 = lvl ? pn[lane] : 0u;
  const float P0 = D.lf.P[(size_t)i * KMAX + lane];
  const Pos p = D.lf.pos[i];
  const int k = hdr_k(hd);
  {
    // exp/agent.py:47-52 as backup_path, level d = lane from the loads above, then any level >= 64
    const double v = (double)vf;
    if (lane < depth) {
      const double vd = ((depth - lane) & 1) ? -v : v;
      const uint32_t Ni = T.e_N[pe0];
      const double N = (double)Ni;
      const double Q = T.e_Q[pe0];
      const double prod = N * Q;
      const double num = prod + vd;
      T.e_Q[pe0] = num / (N + 1.0);
      T.e_N[pe0] = Ni + 1;
      T.node_hdr[nbase + pn0].sumN += 1;
    }
    for (int d = lane + 64; d < depth; d += 64) {
      const double vd = ((depth - d) & 1) ? -v : v;
      const size_t e = pe[d];
      const uint32_t Ni = T.e_N[e];
      const double N = (double)Ni;
      const double Q = T.e_Q[e];
      const double prod = N * Q;
      const double num = prod + vd;
      T.e_Q[e] = num / (N + 1.0);
      T.e_N[e] = Ni + 1;
      T.node_hdr[nbase + pn[d]].sumN += 1;
    }
  }
  for (int c = lane; c < k; c += 64) T.e_P[(size_t)hd.e0 + c] = c < 64 ? P0 : D.lf.P[(size_t)i * KMAX + c];
  if (lane == 0) T.node_hdr[nbase + n].tval = vf;   // kept for the leaf memo (Params::memo)
  if (D.pr.memo >= 2 && D.bm.cap && k <= MEMO_K) {
    // batch memo insert: claim a slot (0 -> 1), write, publish (-> 2); a slot another leaf of this
    // launch claimed is passed over (at worst a position is kept twice, with identical results).
    // Readers (k_select) run in later launches on the same stream, so the kernel boundary orders
    // the entry's writes before any lookup: no fence, and the publish is a plain store.  Within
    // this launch a prober may see state 2 before the key: it then passes over the slot or, on a
    // stale key equal to its own, skips the insert (a memo miss later, never a wrong entry).
    const BatchMemo& B = D.bm;
    uint32_t slot = NONE;
    if (lane == 0) {
      const uint32_t mask = B.cap - 1;
      uint32_t h = pos_hash(p) & mask;
      for (uint32_t probe = 0; probe < MEMO_PROBES; ++probe, h = (h + 1) & mask) {
        const uint32_t st = atomicCAS(&B.state[h], 0u, 1u);
        if (st == 0u) {
          slot = h;
          break;
        }
        if (st == 2u && pos_eq(B.key[h], p)) break;
      }
    }
    slot = (uint32_t)__builtin_amdgcn_readlane((int)slot, 0);
    if (slot != NONE) {
      for (int c = lane; c < k; c += 64) {
        B.codes[(size_t)slot * MEMO_K + c] = T.e_code[(size_t)hd.e0 + c];
        static_assert(MEMO_K <= 64, "a memo entry's priors are the lanes' first priors");
        B.P[(size_t)slot * MEMO_K + c] = P0;   // c = lane
      }
      if (lane == 0) {
        B.key[slot] = p;
        B.v[slot] = vf;
        B.k[slot] = (uint16_t)k;
        B.state[slot] = 2u;
      }
    }
  }
  if (lane == 0) D.lf.gnode[g] = NONE;   // evaluated: no longer pending (deferred-tail play)
}

void launch_memo_clear(const Dev& d, hipStream_t s) {
  if (d.bm.cap) (void)hipMemsetAsync(d.bm.state, 0, (size_t)d.bm.cap * 4, s);
}

void launch_backup(const Dev& d, hipStream_t s) {
  hipLaunchKernelGGL(k_backup, dim3((d.pr.G + 3) / 4), dim3(256), 0, s, d);
}

__global__ void k_gather_leaf_codes(Dev D, uint16_t* __restrict__ codes, int32_t* __restrict__ kout) {
  const int i = blockIdx.x;
  if (i >= *D.lf.count) return;
  const Trees& T = D.tr;
  const int t = D.lf.tree[i];
  const uint32_t n = D.lf.node[i];
  const NodeHdr hd = T.node_hdr[(size_t)t * T.NC + n];
  const int k = hdr_k(hd);
  const uint32_t e0 = hd.e0;
  for (int c = threadIdx.x; c < k; c += blockDim.x) codes[(size_t)i * KMAX + c] = T.e_code[(size_t)e0 + c];
  if (threadIdx.x == 0) kout[i] = k;
}

void launch_gather_leaf_codes(const Dev& d, uint16_t* codes_out, int32_t* k_out, hipStream_t s) {
  hipLaunchKernelGGL(k_gather_leaf_codes, dim3(d.pr.G), dim3(64), 0, s, d, codes_out, k_out);
}

// Root visit counts after the search (exp/policy.py:119-121: pi = N / N.sum()).
__global__ __launch_bounds__(64) void k_move_end(Dev D, uint16_t* __restrict__ codes, uint32_t* __restrict__ visits, int kout) {
  const int g = blockIdx.x, lane = threadIdx.x;
  if (!D.gm.active[g]) return;
  const Trees& T = D.tr;
  const int t = 2 * g + D.gm.agent[g];
  uint32_t slot;
  const uint32_t n = tree_find(T, t, D.gm.root[g], &slot);
  if (n == NONE) {
    if (lane == 0) atomicOr(D.pr.err, ERR_ROOT);
    return;
  }
  const NodeHdr hd = T.node_hdr[(size_t)t * T.NC + n];
  const int k = hdr_k(hd);
  const uint32_t e0 = hd.e0;
  if (k > kout) {
    if (lane == 0) atomicOr(D.pr.err, ERR_KMAX);
    return;
  }
  for (int c = lane; c < k; c += 64) {
    codes[(size_t)g * kout + c] = T.e_code[(size_t)e0 + c];
    visits[(size_t)g * kout + c] = T.e_N[(size_t)e0 + c];
  }
}

void launch_move_end(const Dev& d, uint16_t* codes_out, uint32_t* visits_out, int kout, hipStream_t s) {
  hipLaunchKernelGGL(k_move_end, dim3(d.pr.G), dim3(64), 0, s, d, codes_out, visits_out, kout);
}

// Game step (exp/environment.py:68-82) + game-level result with history (fivefold
// repetition compares the positions since the last zeroing move).  One thread; returns whether the
// game goes on, with its new root in *next.
__device__ bool game_step(const Dev& D, int g, int code, Pos* next) {
  const Pos p = D.gm.root[g];
  const BB b = unpack(p);
  bool ok = code >= 0 && code < NUM_ACTIONS;
  int from = 0, to = 0;
  if (ok) {
    const uint16_t ft = d_codec.dec[b.white ? 0 : 1][code];
    from = ft & 0xff;
    to = ft >> 8;
    const uint32_t own = b.white ? b.w : b.b;
    ok = ((own >> from) & 1u) && ((legal_targets(b, from, D.pr.flags) >> to) & 1u);
  }
  const int nh = D.gm.nhist[g];
  if (!ok || nh >= D.gm.HMAX) {
    atomicOr(D.pr.err, ok ? ERR_HIST : ERR_ILLEGAL);
    D.gm.active[g] = 0;
    D.gm.outcome[g] = -1;
    return false;
  }
  Pos* hist = D.gm.hist + (size_t)g * D.gm.HMAX;
  hist[nh] = p;
  const BB nb = dev_apply_code(b, code);
  const Pos np = pack(nb);
  int reps = 1;
  for (int i = nh; i >= 0 && i > nh - nb.half; --i)
    if (pos_eq_board_turn(hist[i], np)) ++reps;
  const int k = legal_count(nb, D.pr.flags);
  const int oc = outcome(nb, k, in_check(nb), D.pr.flags, D.pr.move_cap, reps);
  D.gm.root[g] = np;
  D.gm.agent[g] ^= 1;
  D.gm.nhist[g] = nh + 1;
  D.gm.outcome[g] = oc;
  if (oc != ONGOING) D.gm.active[g] = 0;
  *next = np;
  return oc == ONGOING;
}

__global__ void k_apply(Dev D, const int32_t* __restrict__ actions) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= D.pr.G || !D.gm.active[g]) return;
  Pos np;
  (void)game_step(D, g, actions[g], &np);
}

void launch_apply(const Dev& d, const int32_t* actions, hipStream_t s) {
  hipLaunchKernelGGL(k_apply, dim3((d.pr.G + 127) / 128), dim3(128), 0, s, d, actions);
}

// Dirichlet vectors per k_turn draw in free-running play: about 40 gammas, which the wave's 64
// attempts of one round usually cover (shape 0.6 accepts ~4 in 5)
__device__ __forceinline__ int turn_noise_chunk(int k) { return k >= 40 ? 1 : 40 / k; }

// Free-running moves (mtaz_set_schedule 1).  A game whose move is complete (all
// `sims` simulations started, no leaf pending: its last backup ran in the previous wave) finishes
// it here, one wavefront per game, at the start of a wave, and its next move's first simulation
// runs in the same wave's k_select, so no game waits for the others' moves:
//   record (exp/callbacks.py:40-47): root position, legal list, visit counts, the action;
//   action choice (exp/agent.py:110-119) from the root's visit counts on the game's RandomState;
//   game step (exp/environment.py:68-82, k_apply's rules and repetition history);
//   move start as k_move_begin (exp/agent.py:57: is the new root in the agent's table? k, new);
//   the first chunk of the new move's sims - root_new Dirichlet vectors (exp/agent.py:81-82) into the
//   game's own noise region [g * sims * KMAX, ...) with stride k; a game in mid-move draws its next
//   chunk here once its next simulation needs a vector not drawn yet (round 6).
// The game's stream runs choice(move t) then noise(move t + 1), the reference's order.  `start`: the
// play's first move of every active game (move start + first noise chunk only).
__global__ __launch_bounds__(64) void k_turn(Dev D, int start) {
#pragma clang fp contract(off)
  __shared__ LegalLds s_l;
  __shared__ RuleTables s_rt;
  __shared__ uint32_t s_mt[2][rng::MT_N];
  __shared__ double s_g[rng::GAMMA_BUF];   // the choice's pi (KMAX), then the gammas
  __shared__ double s_inv[64];
  __shared__ unsigned long long s_u;
  __shared__ Pos s_root;
  __shared__ int s_go;
  const int g = blockIdx.x, lane = threadIdx.x;
  if (!D.gm.active[g]) return;
  if (!start && (D.gm.simc[g] < D.pr.sims || D.lf.gnode[g] != NONE)) {
    // mid-move: the next chunk of the move's Dirichlet vectors once the game's next simulation needs
    // a vector not drawn yet (simulation j takes vector j - root_new, exp/agent.py:81-82).  The
    // vectors come in order from the game's stream, all before the move's action choice, so the
    // stream is drawn exactly as in one launch per move; drawn in chunks, a move start no longer puts
    // all of them on the wave's critical path (round 6: 70 us per wave for 64 vectors)
    const int sc = D.gm.simc[g], rnew = D.gm.root_new[g], nd = D.gm.ndraw[g], k = D.gm.root_k[g];
    const int need = D.pr.sims - rnew;
    if (sc - rnew < nd || nd >= need || k <= 0 || k > KMAX) return;
    const int c = min(turn_noise_chunk(k), need - nd);
    rng::WaveMT mt{s_mt};
    mt.load(D.gm.mt_key + (size_t)g * rng::MT_N, D.gm.mt_pos[g], lane);
    rng::wave_dirichlet(mt, D.pr.alpha, k, c, D.gm.noise + D.gm.noise_off[g] + (int64_t)nd * k, k, s_g, s_inv, lane);
    mt.store(D.gm.mt_key + (size_t)g * rng::MT_N, D.gm.mt_pos + g, lane);
    if (lane == 0) D.gm.ndraw[g] = nd + c;
    return;
  }
  const Trees& T = D.tr;
  rng::WaveMT mt{s_mt};
  mt.load(D.gm.mt_key + (size_t)g * rng::MT_N, D.gm.mt_pos[g], lane);
  Pos root = D.gm.root[g];
  int ag = D.gm.agent[g];
  if (!start) {
    const int t = 2 * g + ag;
    const size_t nbase = (size_t)t * T.NC;
    uint32_t n = D.gm.root_node[g], slot;
    if (n >= (uint32_t)D.tr.n_nodes[t] || !pos_eq(T.node_pos[nbase + n], root)) n = tree_find(T, t, root, &slot);
    if (n == NONE) {
      if (lane == 0) atomicOr(D.pr.err, ERR_ROOT);
      return;
    }
    const NodeHdr hd = T.node_hdr[nbase + n];
    const int k = hdr_k(hd), p = D.gm.nply[g];
    const uint32_t e0 = hd.e0;
    const int64_t cur = D.gm.rec_cur[g];
    if (k <= 0 || k > KMAX || p >= D.gm.PLY || cur + k > D.gm.RC) {
      if (lane == 0) atomicOr(D.pr.err, k <= 0 ? ERR_ROOT : k > KMAX ? ERR_KMAX : ERR_HIST);
      return;
    }
    uint16_t* rc = D.gm.rec_codes + (size_t)g * D.gm.RC + cur;
    uint32_t* rv = D.gm.rec_visits + (size_t)g * D.gm.RC + cur;
    for (int c = lane; c < k; c += 64) {
      rc[c] = T.e_code[(size_t)e0 + c];
      rv[c] = T.e_N[(size_t)e0 + c];
    }
    const int idx = rng::wave_choose(mt, T.e_N + e0, k, (int)(root.info >> 16), D.pr.tau, s_g, &s_u, D.pr.err, lane);
    if (lane == 0) {
      const int action = idx >= 0 ? (int)T.e_code[(size_t)e0 + idx] : -1;
      const size_t r = (size_t)g * D.gm.PLY + p;
      D.gm.rec_pos[r] = root;
      D.gm.rec_action[r] = action;
      D.gm.rec_k[r] = k;
      D.gm.nply[g] = p + 1;
      D.gm.rec_cur[g] = (int32_t)(cur + k);
      Pos np;
      s_go = game_step(D, g, action, &np) ? 1 : 0;
      s_root = np;
    }
    __syncthreads();
    if (!s_go) {
      mt.store(D.gm.mt_key + (size_t)g * rng::MT_N, D.gm.mt_pos + g, lane);
      return;
    }
    root = s_root;   // (game_step's stores, passed to the other lanes through LDS)
    ag ^= 1;
  }
  // the new move (k_move_begin): the root in the agent's table?  its legal count
  const int t = 2 * g + ag;
  uint32_t slot;
  const uint32_t n = tree_find(T, t, root, &slot);
  int k = 0, rnew = 0;
  if (n != NONE) {
    const NodeHdr hd = T.node_hdr[(size_t)t * T.NC + n];
    if (hdr_term(hd) && lane == 0) atomicOr(D.pr.err, ERR_ROOT);
    k = hdr_k(hd);
  } else {
    load_rules_lds(&s_rt);
    const BB b = unpack(root);
    __syncthreads();
    k = wave_legal(b, D.pr.flags, s_rt, s_l);
    rnew = 1;
    if (k <= 0 && lane == 0) atomicOr(D.pr.err, k < 0 ? ERR_KMAX : ERR_ROOT);
  }
  const int64_t noff = (int64_t)g * D.pr.sims * KMAX;
  if (lane == 0) {
    D.gm.root_node[g] = n;
    D.gm.root_k[g] = k;
    D.gm.root_new[g] = rnew;
    D.gm.simc[g] = 0;
    D.gm.noise_off[g] = noff;
    D.gm.noise_js[g] = k;
  }
  // the move's first chunk of Dirichlet vectors (the rest as its simulations come to need them, above)
  const int c = (k > 0 && k <= KMAX) ? min(turn_noise_chunk(k), D.pr.sims - rnew) : 0;
  if (c > 0) rng::wave_dirichlet(mt, D.pr.alpha, k, c, D.gm.noise + noff, k, s_g, s_inv, lane);
  if (lane == 0) D.gm.ndraw[g] = c > 0 ? c : 0;
  mt.store(D.gm.mt_key + (size_t)g * rng::MT_N, D.gm.mt_pos + g, lane);
}

void launch_turn(const Dev& d, int start, hipStream_t s) {
  hipLaunchKernelGGL(k_turn, dim3(d.pr.G), dim3(64), 0, s, d, start);
}

// the active games' count into *out
__global__ __launch_bounds__(256) void k_count_active(Dev D, int32_t* __restrict__ out) {
  int c = 0;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < D.pr.G; g += gridDim.x * 256) c += D.gm.active[g] != 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

void launch_count_active(const Dev& d, int32_t* out, hipStream_t s) {
  (void)hipMemsetAsync(out, 0, 4, s);
  hipLaunchKernelGGL(k_count_active, dim3(16), dim3(256), 0, s, d, out);
}

// game g's appended legal lists and visit counts (rec_cur[g] entries) to codes / visits at off[g]
__global__ __launch_bounds__(256) void k_rec_pack(Dev D, const int64_t* __restrict__ off, uint16_t* __restrict__ codes,
                                                  uint32_t* __restrict__ visits) {
  const int g = blockIdx.x;
  const int n = D.gm.rec_cur[g];
  const size_t src = (size_t)g * D.gm.RC;
  const int64_t dst = off[g];
  for (int i = threadIdx.x; i < n; i += 256) {
    codes[dst + i] = D.gm.rec_codes[src + i];
    visits[dst + i] = D.gm.rec_visits[src + i];
  }
}

void launch_rec_pack(const Dev& d, const int64_t* off, uint16_t* codes, uint32_t* visits, hipStream_t s) {
  hipLaunchKernelGGL(k_rec_pack, dim3(d.pr.G), dim3(256), 0, s, d, off, codes, visits);
}

// ---------------------------------------------------------------------------------------
// network
__device__ __forceinline__ int padpos(int p) { return (p / 5 + 1) * 7 + (p % 5 + 1); }   // 8x7 zero-padded board

// Embedding(7,4) -> permute -> (8, 6, 5) -> Conv3x3(8->256)+BN+ReLU (exp/policy.py:58, :72-73).
// One 256-thread block per board, thread = output channel.
__global__ __launch_bounds__(256) void k_stem(const Pos* __restrict__ pos, const int32_t* __restrict__ count, int max_b,
                                              NetWeights W, float* __restrict__ out) {
  __shared__ float xin[8 * 56];
  __shared__ uint8_t tok[60];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nb = count ? *count : max_b;
  if (b >= nb) return;
  for (int i = tid; i < 8 * 56; i += 256) xin[i] = 0.f;
  if (tid == 0) encode_tokens(unpack(pos[b]), tok);
  __syncthreads();
  if (tid < 240) {
    const int c = tid / 30, p = tid % 30;         // c = plane*4 + e
    xin[c * 56 + padpos(p)] = W.emb[tok[(c >> 2) * 30 + p] * 4 + (c & 3)];
  }
  __syncthreads();
  const int co = tid;
  float w[72];
#pragma unroll
  for (int j = 0; j < 72; ++j) w[j] = W.stem_w[co * 72 + j];
  const float bias = W.stem_b[co];
  float* o = out + (size_t)b * 8192 + co * 32;
  for (int p = 0; p < 30; ++p) {
    const int pp = padpos(p);
    float acc = bias;
#pragma unroll
    for (int ci = 0; ci < 8; ++ci)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) acc += w[ci * 9 + tap] * xin[ci * 56 + pp + (tap / 3 - 1) * 7 + (tap % 3 - 1)];
    o[p] = fmaxf(acc, 0.f);
  }
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Residual-trunk 3x3 conv (256 -> 256) + folded BN (+ residual) + ReLU as an implicit
// GEMM on fp32 MFMA: M = board positions (one 32-row tile per board, rows 30/31 are
// padding), N = output channels, K = 9 taps x 256 input channels = 2304.
// Block = 256 threads (4 waves) x 2 boards; the two input boards sit in LDS as
// [ci][board][8x7 padded] fp32 (114,688 B), so the whole K loop runs barrier-free from
// LDS + L2-resident pre-swizzled weights (one float4 per lane per 4 k-steps).
// Wave w computes output channels [64w, 64w+64) for both boards: 4 accumulators of
// 32x32 (v_mfma_f32_32x32x2_f32: lane l holds A[row l&31][k l>>5], B[k l>>5][col l&31]).
__global__ __launch_bounds__(256, 1) void k_conv3x3(const float* __restrict__ in, const float* __restrict__ resid,
                                                    float* __restrict__ out, const float4* __restrict__ wpk,
                                                    const float* __restrict__ bias, const int32_t* __restrict__ count,
                                                    int max_b) {
  __shared__ float lds[2 * 256 * 56];
  const int nb = count ? *count : max_b;
  const int b0 = blockIdx.x * 2;
  if (b0 >= nb) return;
  const int tid = threadIdx.x;
  // stage: in[b][ci][0..31] as 8 float4 per (board, ci).  Thread tid owns float4 q = tid&7
  // of channels ci = (tid>>3) + 32j, j = 0..7, for both boards: all 16 loads are issued
  // before the first LDS write.
  const int q = tid & 7, p0 = q * 4;
  float4 st[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int bb = j >> 3, ci = (tid >> 3) + 32 * (j & 7);
    st[j] = (b0 + bb < nb) ? reinterpret_cast<const float4*>(in + (size_t)(b0 + bb) * 8192 + ci * 32)[q]
                           : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  {
    float4* l4 = reinterpret_cast<float4*>(lds);
    for (int i = tid; i < 2 * 256 * 56 / 4; i += 256) l4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  const int pp0 = padpos(p0), pp1 = padpos(p0 + 1), pp2 = padpos(p0 + 2), pp3 = padpos(p0 + 3);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int bb = j >> 3, ci = (tid >> 3) + 32 * (j & 7);
    float* dst = lds + (ci * 2 + bb) * 56;
    dst[pp0] = st[j].x;
    dst[pp1] = st[j].y;
    if (p0 + 2 < 30) dst[pp2] = st[j].z;      // q = 7 covers positions 28..31 (30, 31 are padding)
    if (p0 + 3 < 30) dst[pp3] = st[j].w;
  }
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63;
  const int row = lane & 31, kh = lane >> 5;
  const int pp = padpos(row < 30 ? row : 29);       // rows 30/31: any valid address, outputs discarded
  const float4* w0 = wpk + (size_t)(2 * wave) * 288 * 64 + lane;
  const float4* w1 = wpk + (size_t)(2 * wave + 1) * 288 * 64 + lane;
  f32x16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
  // Chunked accumulation: every tap's 256 k (32 groups) accumulates from zero and is then added
  // into the master sums m** (round to nearest), so that each output takes 9 roundings at its full
  // magnitude instead of one per MFMA (1152 two-product steps); as in k_net_y (mtaz_net16.hip, CH)
  f32x16 m00 = {0}, m01 = {0}, m10 = {0}, m11 = {0};
  // Software pipeline over the 288 groups of 4 k-steps (k = tap*256 + ci): the weight
  // float4s of group s+2 and the 8 A values of group s+1 are issued before the 16 MFMAs
  // of group s; sched_barrier keeps the compiler from sinking them next to their use.
  auto a_ptr = [&](int s4) {
    const int tap = s4 >> 5, q = s4 & 31;
    return lds + kh * 112 + pp + (tap / 3 - 1) * 7 + (tap % 3 - 1) + q * 4 * 224;
  };
  float4 wb0[2], wb1[2];
  wb0[0] = w0[0];
  wb1[0] = w1[0];
  wb0[1] = w0[64];
  wb1[1] = w1[64];
  float an[8];
  {
    const float* a = a_ptr(0);
    an[0] = a[0]; an[1] = a[56]; an[2] = a[224]; an[3] = a[280];
    an[4] = a[448]; an[5] = a[504]; an[6] = a[672]; an[7] = a[728];
  }
#pragma unroll 2
  for (int s4 = 0; s4 < 288; ++s4) {
    const float4 cb0 = wb0[s4 & 1], cb1 = wb1[s4 & 1];
    float ac[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) ac[j] = an[j];
    if (s4 + 2 < 288) {
      wb0[s4 & 1] = w0[(s4 + 2) * 64];
      wb1[s4 & 1] = w1[(s4 + 2) * 64];
    }
    if (s4 + 1 < 288) {
      const float* a = a_ptr(s4 + 1);
      an[0] = a[0]; an[1] = a[56]; an[2] = a[224]; an[3] = a[280];
      an[4] = a[448]; an[5] = a[504]; an[6] = a[672]; an[7] = a[728];
    }
    __builtin_amdgcn_sched_barrier(0);
    acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[0], cb0.x, acc00, 0, 0, 0);
    acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[0], cb1.x, acc01, 0, 0, 0);
    acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[1], cb0.x, acc10, 0, 0, 0);
    acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[1], cb1.x, acc11, 0, 0, 0);
    acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[2], cb0.y, acc00, 0, 0, 0);
    acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[2], cb1.y, acc01, 0, 0, 0);
    acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[3], cb0.y, acc10, 0, 0, 0);
    acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[3], cb1.y, acc11, 0, 0, 0);
    acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[4], cb0.z, acc00, 0, 0, 0);
    acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[4], cb1.z, acc01, 0, 0, 0);
    acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[5], cb0.z, acc10, 0, 0, 0);
    acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[5], cb1.z, acc11, 0, 0, 0);
    acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[6], cb0.w, acc00, 0, 0, 0);
    acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[6], cb1.w, acc01, 0, 0, 0);
    acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[7], cb0.w, acc10, 0, 0, 0);
    acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(ac[7], cb1.w, acc11, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if ((s4 & 31) == 31) {
      m00 += acc00; m01 += acc01; m10 += acc10; m11 += acc11;
      acc00 = (f32x16){0}; acc01 = (f32x16){0}; acc10 = (f32x16){0}; acc11 = (f32x16){0};
    }
  }
  acc00 = m00; acc01 = m01; acc10 = m10; acc11 = m11;   // (288 = 9 x 32: the last chunk is added)
  // epilogue: col = lane&31 -> channel; rows (r&3) + 8(r>>2) + 4*kh -> positions
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {
    const int b = b0 + bb;
    if (b >= nb) continue;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const f32x16 acc = bb == 0 ? (ct == 0 ? acc00 : acc01) : (ct == 0 ? acc10 : acc11);
      const int co = (2 * wave + ct) * 32 + row;
      const float bv = bias[co];
      const size_t obase = (size_t)b * 8192 + co * 32;
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int r0 = 8 * g4 + 4 * kh;
        float4 v = make_float4(acc[4 * g4 + 0] + bv, acc[4 * g4 + 1] + bv, acc[4 * g4 + 2] + bv, acc[4 * g4 + 3] + bv);
        if (resid) {
          const float4 r = *reinterpret_cast<const float4*>(resid + obase + r0);
          v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
        }
        v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
        *reinterpret_cast<float4*>(out + obase + r0) = v;
      }
    }
  }
}

// Heads (exp/policy.py:62-69, :76-79) + leaf prior extraction (exp/agent.py:67-69):
// pconv/vconv 1x1 + BN + ReLU, value MLP + tanh, policy logits for the legal codes only
// and a float32 softmax over them (duplicates included).  One block per board.
__global__ __launch_bounds__(256) void k_heads(Dev D, NetWeights W, const float* __restrict__ x, const Pos* __restrict__ pos,
                                               const int32_t* __restrict__ count, int max_b, int mode,
                                               float* __restrict__ logits_out, float* __restrict__ values_out) {
  __shared__ float xs[256 * 31];
  __shared__ float fp[64], fv[32];
  __shared__ float red[256];
  __shared__ float sl[KMAX];
  __shared__ uint16_t scode[KMAX];
  __shared__ int sk;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int nb = count ? *count : max_b;
  if (b >= nb) return;
  for (int idx = tid; idx < 256 * 30; idx += 256) {
    const int c = idx / 30, p = idx - c * 30;
    xs[c * 31 + p] = x[(size_t)b * 8192 + c * 32 + p];
  }
  if (tid == 0) {
    const BB bb = unpack(pos[b]);
    const float clk = encode_clock(bb);
    fp[60] = clk;
    fv[30] = clk;
  }
  if (mode == NET_LEAVES && tid == 0) {
    const int t = D.lf.tree[b];
    const uint32_t n = D.lf.node[b];
    sk = hdr_k(D.tr.node_hdr[(size_t)t * D.tr.NC + n]);
  }
  __syncthreads();
  if (mode == NET_LEAVES) {
    const int t = D.lf.tree[b];
    const uint32_t n = D.lf.node[b];
    const uint32_t e0 = D.tr.node_hdr[(size_t)t * D.tr.NC + n].e0;
    for (int c = tid; c < sk; c += 256) scode[c] = D.tr.e_code[(size_t)e0 + c];
  }
  if (tid < 90) {
    const int o = tid / 30, p = tid - o * 30;
    const float* wr = o < 2 ? W.pconv_w + o * 256 : W.vconv_w;
    float s = 0.f;
    for (int c = 0; c < 256; ++c) s += wr[c] * xs[c * 31 + p];
    s += o < 2 ? W.pconv_b[o] : W.vconv_b[0];
    s = fmaxf(s, 0.f);
    if (o < 2) fp[o * 30 + p] = s; else fv[p] = s;
  }
  __syncthreads();
  // value: Linear(31,256) ReLU Linear(256,1) Tanh
  {
    float h = W.vl1_b[tid];
    for (int i = 0; i < 31; ++i) h += W.vl1_w[tid * 31 + i] * fv[i];
    h = fmaxf(h, 0.f);
    red[tid] = W.vl2_w[tid] * h;
  }
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  if (tid == 0) {
    const float v = tanhf(red[0] + W.vl2_b[0]);
    if (mode == NET_LEAVES) D.lf.v[b] = v; else values_out[b] = v;
  }
  __syncthreads();
  if (mode == NET_FULL_LOGITS) {
    for (int a = tid; a < NUM_ACTIONS; a += 256) {
      float l = W.plin_b[a];
      for (int j = 0; j < 61; ++j) l += W.plin_w[a * 61 + j] * fp[j];
      logits_out[(size_t)b * NUM_ACTIONS + a] = l;
    }
    return;
  }
  const int k = sk;
  for (int c = tid; c < k; c += 256) {
    const int a = scode[c];
    float l = W.plin_b[a];
    for (int j = 0; j < 61; ++j) l += W.plin_w[a * 61 + j] * fp[j];
    sl[c] = l;
  }
  __syncthreads();
  // softmax over the k gathered logits (k <= KMAX = 256: one element per thread)
  red[tid] = tid < k ? sl[tid] : -__builtin_inff();
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] = fmaxf(red[tid], red[tid + s]);
    __syncthreads();
  }
  const float mx = red[0];
  __syncthreads();
  const float ex = tid < k ? expf(sl[tid] - mx) : 0.f;
  red[tid] = ex;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const float sum = red[0];
  if (tid < k) D.lf.P[(size_t)b * KMAX + tid] = ex / sum;
}

void launch_net(const Dev& d, const NetWeights& w, const NetBuffers& nbuf, const Pos* pos, const int32_t* count, int max_b,
                int mode, float* values_out, hipStream_t s, hipEvent_t trunk_begin, hipEvent_t trunk_end) {
  if (max_b <= 0) return;
  hipLaunchKernelGGL(k_stem, dim3(max_b), dim3(256), 0, s, pos, count, max_b, w, nbuf.x0);
  if (trunk_begin) (void)hipEventRecord(trunk_begin, s);
  float* xc = nbuf.x0;
  float* xn = nbuf.x1;
  const int grid = (max_b + 1) / 2;
  for (int blk = 0; blk < 9; ++blk) {
    const int la = 2 * blk, lb = 2 * blk + 1;
    hipLaunchKernelGGL(k_conv3x3, dim3(grid), dim3(256), 0, s, xc, (const float*)nullptr, nbuf.t,
                       reinterpret_cast<const float4*>(w.conv_w + la * CONV_W_FLOATS), w.conv_b + la * 256, count, max_b);
    hipLaunchKernelGGL(k_conv3x3, dim3(grid), dim3(256), 0, s, nbuf.t, (const float*)xc, xn,
                       reinterpret_cast<const float4*>(w.conv_w + lb * CONV_W_FLOATS), w.conv_b + lb * 256, count, max_b);
    float* tmp = xc;
    xc = xn;
    xn = tmp;
  }
  if (trunk_end) (void)hipEventRecord(trunk_end, s);
  hipLaunchKernelGGL(k_heads, dim3(max_b), dim3(256), 0, s, d, w, xc, pos, count, max_b, mode, nbuf.logits, values_out);
}

}  // namespace mtaz
