// k_net_y (round 4): the fused fp16x3 policy/value network (exp/policy.py:71-80 + the leaf priors
// of exp/agent.py:67-69) on v_mfma_f32_16x16x32_f16, with the 3x3 convs' off-board taps skipped.
//
// Arithmetic: round 3's k_net_y (mtaz_net16_r3.hip): fp16 hi/lo split of weights and activations,
// three f16 MFMA passes Wh*Xh + Wh*Xl + Wl*Xh per k-block, chunks of 12 k-blocks accumulated from
// zero and added into fp32 master sums, in-place LDS image, fused heads.  Per output element every
// MFMA chain, chunk boundary and master-sum add is round 3's, so on a net that needs no range
// scaling the results are bitwise round 3's (test_gpu_net.py).
//
// What is new:
//  1. CLASS TILES + TAP SKIP.  A 3x3 conv on the 6 x 5 board reads zeros for the taps that fall
//     off the board: 23% of the (square, tap) pairs.  Round 3 tiled the N dimension by board
//     (squares 0-15, 16-31 of each board), so every 16-square tile had on-board sources for every
//     tap and every MFMA ran.  Here a workgroup's 4 boards x 32 squares are regrouped into 8 tiles
//     of 16 by the squares' position class: 3 tiles of interior squares (all 9 taps), the top row
//     T (no dr = -1 taps), the bottom row B (no dr = +1), the left file L (no dc = -1), the right
//     file R (no dc = +1), and X (the right corners + the padding squares 30, 31; no dc = +1).
//     A tile whose 16 squares all read zeros for a tap skips that tap's MFMAs: 57 of 72 tile-taps
//     run (-21% MFMAs).  Skipping a k-block whose products are all zero leaves every accumulator
//     bit unchanged (C + 0 = C), so the regrouping changes no result.
//  2. ONE STORED-UNITS EXPONENT PER BOARD.  The image holds x * 2^-xs[b] with xs
//     chosen from board b's own bound, so no runtime max crosses boards: a board's results do not
//     depend on which boards share its workgroup, for every net (round 3: only below 2^14).
//
// Workgroup = 4 boards (NVB < 4: the tail instances; 1 and 2 boards on round 3's per-board tiles,
// 3 boards on class tiles of their own, TMAP3), 256 threads.
// Wave w owns output channels [64w, 64w + 64) as 4 channel tiles of 16, times 8 N tiles of 16
// squares: 32 accumulator tiles (128 AGPRs) + 32 master sums.  A conv's K = 2304 runs as 72
// k-blocks of 32 contiguous k = tap*256 + ci (tap = 3(dr + 1) + (dc + 1)), in 3 rows of taps
// (dr) of 24 k-blocks; the row loop is a runtime loop, the 24 k-blocks of a row are unrolled, so
// the dc-dependent skips (L, R, X) are compile-time and the dr-dependent ones (T, B) are one
// uniform branch per half-step.
#include <type_traits>
#include <utility>

#include "net_common.h"

namespace mtaz {

using namespace netc;
typedef float f32x4v __attribute__((ext_vector_type(4)));

namespace ny {

// weight prefetch depth of the 1- and 2-board tail instances (k-blocks ahead; PD + 1 must divide
// 24); build-time knobs for tools/build_exp_libs.py A/Bs, the product uses the defaults
#ifndef MTAZ_Y_PD1
#define MTAZ_Y_PD1 5
#endif
#ifndef MTAZ_Y_PD2
#define MTAZ_Y_PD2 3
#endif
constexpr int KBY = 72;                     // k-blocks of 32 per conv
constexpr int CELLS_B = 16384;              // per board and part: 32 squares x 32 chunks x 16 B
constexpr int PART_B = CELLS_B + 512;       // + 512 B unused (round 3's zero line; keeps the heads' offset)
constexpr int BOARD_B = 2 * PART_B;         // board b's parts hi, lo at b * BOARD_B (+ PART_B)
constexpr int IMG_B = XB * BOARD_B;         // 135,168 B
constexpr int TAB_B = 9 * 2 * 64 * 16;      // fragment offset table [tap][half][lane][4 tiles]
constexpr int SMEM_B = IMG_B + AUXB + TAB_B;
static_assert(IMG_B == ZIMGB, "heads_out reads the feature region right after the image");
static_assert(SMEM_B <= 163840, "LDS");

// The image.  Square r of board b, channel chunk q (8 channels), part (hi / lo) at
//   b * BOARD_B + part * PART_B + 256 q + 8192 (r >> 4) + 16 ((r + 4b) & 15):
// chunk-major within 16-square halves (round 3's layout), with the bank group of a cell rotated
// by 4 per board.  A fragment read (each 16-lane LDS group = the 16 squares of one tile, any
// chunk per lane) touches 16 distinct bank groups when the tile's 16 (board, square) pairs have
// distinct (square + 4 board) mod 16, which the class tiles below are built to have (every tap
// shifts all 16 by the same square offset).  The padding squares 30, 31 of every board are kept
// ZERO (the epilogue stores zeros there), so an off-board tap reads one of those 8 cells (4 boards
// x 2 squares, bank groups 2, 3 mod 4) at the same chunk as an on-board tap: a lane's fragment
// address is its table entry + 1024 (k-block mod 8), the step an immediate of the ds_read, with
// no per-lane arithmetic.  The cell is chosen on the bank the source would have had when one is
// (else that bank ^ 2): tools/net_tiles.py counts 12 extra LDS cycles over the 57 tile-taps.
__device__ __forceinline__ int cell(int b, int r) { return b * BOARD_B + 8192 * (r >> 4) + 16 * ((r + 4 * b) & 15); }
// the zero cell (square 30 or 31 of some board) read in place of an off-board source whose cell
// would have had bank group wb
__device__ __forceinline__ int zcell(int wb) {
  wb = (wb & 2) ? wb : wb ^ 2;
  const int r = 30 + (wb & 1);
  return cell(((wb - r) & 15) >> 2, r);
}

// The class tiles of a 4-board workgroup: lane n of tile t holds board (v & 3), square (v >> 2).
// Half 0: tiles 0, 1 interior squares (rows 1-4, files 1-3), 2 = R (file 4, rows 1-4), 3 = T (top
// row, files 0-3); half 1: 4 interior, 5 = L (file 0, rows 1-4), 6 = X (squares 4 and 29, the
// right corners, and the padding squares 30, 31), 7 = B (bottom row, files 0-3).  Each tile holds
// every (square + 4 board) mod 16 once; the halves carry 2-4 compile-time active tiles each at
// every tap.  Generated and checked (conflict-free for every tap; the skip rule below exact) by
// tools/net_tiles.py.  Lane n's bank group at the centre tap is n.
__constant__ uint8_t TMAP4[8][16] = {
    {64, 68, 72, 46, 65, 84, 24, 28, 32, 85, 25, 44, 48, 52, 26, 45},
    {49, 53, 27, 31, 50, 69, 88, 92, 66, 70, 89, 29, 33, 86, 90, 30},
    {98, 38, 57, 76, 99, 39, 58, 77, 96, 36, 59, 78, 97, 37, 56, 79},
    {0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15},
    {34, 87, 91, 95, 35, 54, 73, 47, 51, 55, 74, 93, 67, 71, 75, 94},
    {83, 23, 42, 61, 80, 20, 43, 62, 81, 21, 40, 63, 82, 22, 41, 60},
    {19, 117, 121, 125, 16, 118, 122, 126, 17, 119, 123, 127, 18, 116, 120, 124},
    {113, 102, 106, 110, 114, 103, 107, 111, 115, 100, 104, 108, 112, 101, 105, 109}};

// The 3-board tail instance's class tiles (round 4b; tools/net_tiles.py build3, checked there):
// t0, t1 interior squares; t2 = T + 4 X squares (skips the tap dr = -1, dc = +1: gated in tap row
// 0); t4 = L + 4 interior; t5 = R + 4 X (no dc = +1 taps); t6 = B + 4 X (skips dr = +1, dc = +1:
// gated in tap row 2).  49 of 54 tile-taps run.  Under the (square + 4 board) bank rotation t0, t1
// and t5 keep 1, 2 and 3 duplicate bank groups (2-way conflicts on those reads).
__constant__ uint8_t TMAP3[8][16] = {
    {49, 53, 94, 46, 50, 69, 88, 28, 32, 85, 25, 29, 48, 52, 26, 45},
    {34, 54, 72, 74, 65, 84, 73, 92, 66, 70, 89, 93, 33, 86, 90, 30},
    {0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 18, 116, 120, 124},
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0},
    {64, 68, 42, 61, 80, 20, 24, 62, 81, 21, 40, 44, 82, 22, 41, 60},
    {98, 117, 57, 76, 16, 38, 58, 77, 96, 36, 121, 78, 97, 37, 56, 125},
    {113, 102, 106, 110, 114, 118, 122, 126, 17, 100, 104, 108, 112, 101, 105, 109},
    {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}};

// (board | square << 2) of lane n of tile t = 4 half + i; the 1- and 2-board tail instances (and
// the 3-board one of variant 5) keep round 3's per-board tiles: tile (half h, i) = board i,
// squares 16 h + n
template <int NVB, bool CLS3>
__device__ __forceinline__ int tile_bp(int t, int n) {
  if constexpr (NVB == XB) return TMAP4[t][n];
  if constexpr (CLS3) return TMAP3[t][n];
  return (t & 3) | ((16 * (t >> 2) + n) << 2);
}

// Compile-time activity of tile t at k-block u (0..23) of a tap row (dc = u / 8 - 1).  4 boards:
// T (3) and B (7) depend on the row (dr) and are gated at run time.  3 boards (class tiles): t5
// runs no dc = +1 k-block; t2 and t6 skip theirs in tap row 0 and 2 (gated).
constexpr bool act(int nvb, bool skip, int u, int t) {
  if ((t & 3) >= nvb) return false;
  if (!skip) return true;
  if (nvb == XB) return t == 5 ? u >= 8 : (t == 2 || t == 6) ? u < 16 : true;
  return t == 5 ? u < 16 : true;
}
constexpr bool gated(int nvb, bool skip, int u, int t) {
  if (!skip) return false;
  if (nvb == XB) return t == 3 || t == 7;
  return (t == 2 || t == 6) && u >= 16;
}
// the first k-block of the 12-k-block chunk holding u at which tile t runs (its MFMA chain of the
// chunk starts there from C = 0)
constexpr int first_u(int nvb, bool skip, int u, int t) {
  const int c0 = u < 12 ? 0 : 12;
  for (int v = c0; v < c0 + 12; ++v)
    if (act(nvb, skip, v, t)) return v;
  return -1;
}

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

}  // namespace ny

// fma(f32(f16 half of pk), b, c) (v_fma_mix; exact in f32 where used, as round 3's)
__device__ __forceinline__ float ny_mix_lo(uint32_t pk, float b, float c) {
  float r;
  asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(pk), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float ny_mix_hi(uint32_t pk, float b, float c) {
  float r;
  asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(pk), "v"(b), "v"(c));
  return r;
}
// {f16(y0 - f32(h0)), f16(y1 - f32(h1))} packed (y - hi is exact in f32)
__device__ __forceinline__ uint32_t ny_lo_pair(uint32_t hi_pk, float y0, float y1) {
  uint32_t r;
  asm volatile(
      "v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(r)
      : "v"(hi_pk), "v"(y0), "v"(y1));
  return r;
}
// fp32 add as one v_add_f32 (not paired into v_pk_add_f32, which costs ~13 cycles beside MFMAs)
__device__ __forceinline__ float ny_add(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void ny_add4(f32x4v& m, const f32x4v& a) {
  m[0] = ny_add(m[0], a[0]);
  m[1] = ny_add(m[1], a[1]);
  m[2] = ny_add(m[2], a[2]);
  m[3] = ny_add(m[3], a[3]);
}
// wave-wide max of unsigned v, in lane 63: DPP steps (quad permutes, half-row and row mirrors, row
// broadcasts 15 / 31) instead of six dependent ds_bpermute round trips
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xb1, 0xf, 0xf, false));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4e, 0xf, 0xf, false));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xf, 0xf, false));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xf, 0xf, false));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x142, 0xa, 0xf, false));
  v = __builtin_elementwise_max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}
// ReLU on the float's bits (signed integer max with 0): negative values and -0 give +0, no
// canonicalisation; a NaN stays a NaN (and reaches the overflow check)
__device__ __forceinline__ float relu_bits(float x) {
  return __int_as_float(__builtin_elementwise_max(__float_as_int(x), 0));
}
template <class T>
__device__ __forceinline__ T sel4(int b, T x0, T x1, T x2, T x3) {
  return b == 0 ? x0 : b == 1 ? x1 : b == 2 ? x2 : x3;
}

// VAR: 0 = product; 1 = class tiles without the tap skip (every MFMA runs: the bit-identity
// reference of the skip, and its A/B); 2 = the tail instances as first built in round 4 (off-board
// cells on the padding squares, weights one k-block ahead), for the A/B of the round-4b tails
template <bool STAMP, int VAR, int NVB = XB>
__device__ __forceinline__ void net_y_body(char* smem, const int bid, const Dev& D, const NetWeights& W,
                                           const Pos* __restrict__ pos, const int32_t* __restrict__ count,
                                           int max_b, int mode, float* __restrict__ logits_out,
                                           float* __restrict__ values_out, unsigned long long* __restrict__ stamps,
                                           int ncu) {
  using namespace ny;
  static_assert(NVB >= 1 && NVB <= XB, "boards per workgroup");
  constexpr bool TAIL_R3 = (VAR & 2) != 0;   // tails as first built in round 4 (per-board tiles, zero cells, ring)
  constexpr bool CLS3 = NVB == 3 && !TAIL_R3;  // the 3-board instance on class tiles (round 4b)
  constexpr bool SKIP = (NVB == XB || CLS3) && (VAR & 1) == 0;
  // diagnostic forms (libmtaz_diag.so only; wrong results by construction, for timing and the
  // clock under the power limit), each keeping the MFMA operands real data: 8 = no
  // weight loads in the conv K loops (the layer prologue fills every slot of the ring with a real
  // k-block, which the loop then reuses), 16 = no activation fragment reads in the K loops (the
  // prologue reads both halves' fragments of the layer's first k-block), 32 = no conv epilogue
  // image stores (the image keeps the stem's real activations)
  constexpr bool D_NOW = (VAR & 8) != 0, D_NOF = (VAR & 16) != 0, D_NOE = (VAR & 32) != 0;
  int b0, nb;
  {   // tail-balanced board assignment (round 3): full rounds of 4 boards, then 1-3 per CU
    const int n = count ? *count : max_b;
    const int r = ncu > 0 ? n % (XB * ncu) : 0, per = ncu > 0 ? (r + ncu - 1) / ncu : XB;
    if constexpr (NVB == XB) {
      b0 = bid * XB;
      nb = per < XB ? n - r : n;
    } else {
      if (per != NVB) return;
      b0 = n - r + bid * NVB;
      nb = b0 + NVB < n ? b0 + NVB : n;
    }
  }
  if (b0 >= nb) return;
  constexpr int NW = 4, NT = 64 * NW, CT = 16 / NW;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, n = lane & 15, g = lane >> 4;
  unsigned long long t_prev = 0, st_stem = 0, st_k = 0, st_epi = 0, st_heads = 0;
  unsigned long long t_start = 0, r_start = 0;
  if constexpr (STAMP) {
    t_prev = t_start = __builtin_amdgcn_s_memtime();
    r_start = __builtin_amdgcn_s_memrealtime();
  }
  auto stamp = [&](unsigned long long& a) {
    if constexpr (STAMP) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      a += t - t_prev;
      t_prev = t;
    }
  };

  // this lane's (board | square << 2) in each tile, 8 bits per tile (tiles 0-3, 4-7)
  uint32_t bp_lo = 0, bp_hi = 0;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const uint32_t v = (t & 3) < NVB ? (uint32_t)tile_bp<NVB, CLS3>(t, n) : (31u << 2);
    if (t < 4) bp_lo |= v << (8 * t); else bp_hi |= v << (8 * (t - 4));
  }
  auto bp_of = [&](int t) -> int { return (int)(((t < 4 ? bp_lo : bp_hi) >> (8 * (t & 3))) & 0xffu); };

  f32x4v acc[CT * 8], mst[CT * 8];
#pragma unroll
  for (int i = 0; i < CT * 8; ++i) acc[i] = (f32x4v){0};
#pragma unroll
  for (int i = 0; i < CT * 8; ++i) mst[i] = (f32x4v){0};
  int overflow = 0;

  // Dynamic range, per board: board b's image holds x * 2^-xs[b] in f16 hi/lo, xs[b] chosen before
  // a layer's outputs are stored from a rigorous bound on board b's outputs: |z| <= G_L *
  // max_b(input) + B_L (+ max_b(residual) for conv B); G_L, B_L from the host
  // (NetWeights::yrange), max_b(input) measured by the previous epilogue over board b's squares
  // only.  xo = max(0, ilogb(bound) - 14) keeps every stored value below 2^15; the rescaling is by
  // powers of two, hence exact; an ordinary net keeps xs = 0 (and round 3's bits).
  int xs[4] = {0, 0, 0, 0};
  // stamped build: per board, the layers whose stored-units exponent is nonzero (bit 0 = stem, bit
  // 1 + L = conv L) and the largest exponent, written after the phase stamps (mtaz_net_time)
  uint32_t xs_mask[4] = {0u, 0u, 0u, 0u};
  int xs_max[4] = {0, 0, 0, 0};
  auto note_xs = [&](int layer) {
    if constexpr (STAMP) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        xs_mask[b] |= (uint32_t)(xs[b] != 0) << layer;
        xs_max[b] = xs[b] > xs_max[b] ? xs[b] : xs_max[b];
      }
    }
  };
  float mx_img[4], mx_blk[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int b = 0; b < 4; ++b) mx_img[b] = W.yrange[2 * CONV_LAYERS + 2];   // max |embedding|
  unsigned* mxs = reinterpret_cast<unsigned*>(smem + IMG_B + AUXB - 32);   // [2 slots][4 boards]
  if (tid < 8) mxs[tid] = 0u;
  int slot = 0;

  // Epilogue (stem and every conv): y = ReLU(sum * 2^(xs - e) + bias) stored in place as f16 hi/lo of
  // y * 2^-xo (board b's exponents); conv A seeds the master sums with conv B's residual in conv
  // B's units (x_stored * 2^(e_B + xs - xo)), otherwise resets them.  Lane l holds channels
  // 16ct + 4(l>>4) + r of its square in each tile: 8 B per part.  Ends with a barrier, after which
  // mx_img[b] holds board b's max of the new image (true units).
  auto epilogue = [&](float inv, const float* bias, auto conv_a_t, float s_next, const float* bound) {
    constexpr bool conv_a = decltype(conv_a_t)::value;
    // the lane's tile map is re-read here, so that its per-tile cell addresses are computed in the
    // epilogue instead of hoisted out of the layer loop into spilled registers
    asm volatile("" : "+v"(bp_lo), "+v"(bp_hi));
    // board b's exponents, packed 8 bits per board (biased by 128) so that a lane picks its board's
    // with one bit-field extract (no per-lane branch): dx = xs - xo (input and residual scale),
    // dn = -xo (bias scale)
    int xo[4];
    uint32_t pdx = 0, pdn = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      xo[b] = bound[b] >= 16384.f ? (int)((__float_as_uint(bound[b]) >> 23) & 0xffu) - 127 - 14 : 0;
      pdx |= (uint32_t)(xs[b] - xo[b] + 128) << (8 * b);
      pdn |= (uint32_t)(128 - xo[b]) << (8 * b);
    }
    uint32_t ymt[8];   // per tile: the max of the lane's real square (float bits; y >= 0)
#pragma unroll
    for (int t = 0; t < 8; ++t) ymt[t] = 0u;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int co0 = 16 * CT * wave + 16 * ct + 4 * g;
      const float4 bu = *reinterpret_cast<const float4*>(bias + co0);
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if ((t & 3) >= NVB) continue;
        const int v = bp_of(t), b = v & 3, p = v >> 2;
        const int dx = (int)__builtin_amdgcn_ubfe(pdx, 8 * b, 8) - 128;
        const int dn = (int)__builtin_amdgcn_ubfe(pdn, 8 * b, 8) - 128;
        const float is = __builtin_ldexpf(inv, dx), sv = __builtin_ldexpf(1.f, dn);
        f32x4v& acc_t = acc[ct * 8 + t];
        f32x4v& a = mst[ct * 8 + t];
        if (t >= 4) {   // half-1 tiles: the last chunk's sums are still pending
          a += acc_t;
          acc_t = (f32x4v){0};
        }
        float y[4];
        y[0] = relu_bits(__builtin_fmaf(a[0], is, bu.x * sv));
        y[1] = relu_bits(__builtin_fmaf(a[1], is, bu.y * sv));
        y[2] = relu_bits(__builtin_fmaf(a[2], is, bu.z * sv));
        y[3] = relu_bits(__builtin_fmaf(a[3], is, bu.w * sv));
        // the padding squares 30, 31 (tile X; the tail instances' half-1 tiles) store zeros: they
        // are the zero cells of the off-board taps (masked, no branch)
        if (NVB == XB ? t == 6 : CLS3 ? true : t >= 4) {
          const int keep = -(int)(p < 30);
#pragma unroll
          for (int j = 0; j < 4; ++j) y[j] = __int_as_float(__float_as_int(y[j]) & keep);
        }
        const uint32_t ym = __builtin_elementwise_max(
            __builtin_elementwise_max(__float_as_uint(y[0]), __float_as_uint(y[1])),
            __builtin_elementwise_max(__float_as_uint(y[2]), __float_as_uint(y[3])));
        ymt[t] = __builtin_elementwise_max(ymt[t], ym);
        const int ah = cell(b, p) + 256 * (co0 >> 3) + 8 * (g & 1), al = ah + PART_B;
        if constexpr (conv_a) {
          const float sd = __builtin_ldexpf(s_next, dx);
          const uint2 xh = *reinterpret_cast<const uint2*>(smem + ah);
          const uint2 xl = *reinterpret_cast<const uint2*>(smem + al);
          a[0] = ny_mix_lo(xh.x, sd, ny_mix_lo(xl.x, sd, 0.f));
          a[1] = ny_mix_hi(xh.x, sd, ny_mix_hi(xl.x, sd, 0.f));
          a[2] = ny_mix_lo(xh.y, sd, ny_mix_lo(xl.y, sd, 0.f));
          a[3] = ny_mix_hi(xh.y, sd, ny_mix_hi(xl.y, sd, 0.f));
        } else {
          a = (f32x4v){0};
        }
        f16x4 yh;
#pragma unroll
        for (int j = 0; j < 4; ++j) yh[j] = (_Float16)y[j];
        const uint2 hp = __builtin_bit_cast(uint2, yh);
        if (!D_NOE || bias == W.stem_b) {   // (diagnostic form 32: the stem's image only)
          *reinterpret_cast<uint2*>(smem + ah) = hp;
          *reinterpret_cast<uint2*>(smem + al) = make_uint2(ny_lo_pair(hp.x, y[0], y[1]), ny_lo_pair(hp.y, y[2], y[3]));
        }
      }
    }
    // per-board max of the new image (y >= 0: float bits order as values; NaN above +inf), each
    // tile's max masked into its board's
    uint32_t ymb[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if ((t & 3) >= NVB) continue;
      const int b = bp_of(t) & 3;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) ymb[bb] = __builtin_elementwise_max(ymb[bb], ymt[t] & (0u - (uint32_t)(b == bb)));
    }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const uint32_t m = wave_max_u32(ymb[bb]);
      if (lane == 63) atomicMax(&mxs[4 * slot + bb], m);
    }
    if (tid < 4) mxs[4 * (slot ^ 1) + tid] = 0u;   // every wave read it before this epilogue's first barrier
#pragma unroll
    for (int b = 0; b < 4; ++b) xs[b] = xo[b];
    __syncthreads();
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      mx_img[b] = __builtin_ldexpf(__uint_as_float(mxs[4 * slot + b]), xo[b]);   // true units
      if (b < NVB && b0 + b < nb && !__builtin_isfinite(mx_img[b])) overflow = 1;
    }
    slot ^= 1;
  };

  // ---------------- prologue: zero lines, stem input, fragment offset table ----------------
  char* simg = smem + IMG_B;
  for (int i = tid; i < 2 * XB * 2 * 32; i += NT) {   // the padding squares 30, 31 (the zero cells)
    const int q = i & 31, r = 30 + ((i >> 5) & 1), bb = (i >> 6) & 3, part = i >> 8;
    *reinterpret_cast<uint4*>(smem + cell(bb, r) + 256 * q + part * PART_B) = make_uint4(0, 0, 0, 0);
  }
  for (int i = tid; i < 2 * XB * IROWS; i += NT) *reinterpret_cast<uint4*>(simg + i * 16) = make_uint4(0, 0, 0, 0);
  if constexpr (NVB < XB) {   // board 3 (unused by the tail instances): half 0 zero, the off-board cells of every residue
    for (int i = tid; i < 2 * 32 * 16; i += NT)
      *reinterpret_cast<uint4*>(smem + 3 * BOARD_B + (i >> 9) * PART_B + 16 * (i & 511)) = make_uint4(0, 0, 0, 0);
  }
  {   // the fragment offset table [tap 9][half 2][lane 64][tile i 4]: the byte offset of chunk g of
      // the source square's cell on the board, of a zero cell (zcell) off it and for the padding
      // squares
    int* tab = reinterpret_cast<int*>(smem + IMG_B + AUXB);
    for (int e = tid; e < 9 * 2 * 64 * 4; e += NT) {
      const int i = e & 3, ln = (e >> 2) & 63, h = (e >> 8) & 1, tap = e >> 9;
      int ent = 0;
      if (i < NVB) {
        const int v = tile_bp<NVB, CLS3>(4 * h + i, ln & 15), b = v & 3, p = v >> 2, gg = ln >> 4;
        const int dh = tap / 3 - 1, dw = tap % 3 - 1, r = p / 5 + dh, c = p % 5 + dw, s = p + 5 * dh + dw;
        const bool valid = p < 30 && (unsigned)r < 6u && (unsigned)c < 5u;
        // off the board: a zero cell on the bank group the source would have had -- for the tail
        // instances any of board 3's (unused, zeroed) half 0, for 4 boards a padding square (bank
        // groups 2, 3 mod 4 only: tools/net_tiles.py)
        const int zc = (NVB < XB && !TAIL_R3) ? cell(3, (s + 4 * b + 4) & 15) : zcell(s + 4 * b);
        ent = (valid ? cell(b, s) : zc) + 256 * gg;
      }
      tab[e] = ent;
    }
  }
  __syncthreads();
  if (tid < XB * 30) {   // stem input (exp/policy.py:71-74): [part][board][row][8 ch] in simg
    const int bb = tid / 30, i = tid % 30;
    const int b = b0 + bb;
    int own = 0, opp = 0;
    if (b < nb) {
      const Pos pp = pos[b];
      const bool white = pp.info & 1u;
      const int s = white ? (5 - i / 5) * 5 + i % 5 : (i / 5) * 5 + (4 - i % 5);
      const int nib = nib_at(pp, s);
      const int t = nib & 7;
      const bool mine = t && (((nib & 8) == 0) == white);
      own = mine ? token_code(t) : 0;
      opp = (t && !mine) ? token_code(t) : 0;
    }
    f16x8 xh, xl;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float v = W.emb[(c < 4 ? own : opp) * 4 + (c & 3)];
      xh[c] = (_Float16)v;
      xl[c] = (_Float16)(v - (float)xh[c]);
    }
    *reinterpret_cast<f16x8*>(simg + (bb * IROWS + i) * 16) = xh;
    *reinterpret_cast<f16x8*>(simg + ((XB + bb) * IROWS + i) * 16) = xl;
  }
  __syncthreads();

  // ---------------- stem: conv3x3 8->256, K = 3 k-blocks of (4 taps x 8 channels) ----------
  {
    const uint4* Ws = W.stemy + (size_t)(CT * wave) * 3 * 128 + lane;
    for (int kb = 0; kb < 3; ++kb) {
      f16x8 SA[2 * CT], SH[8], SL[8];
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        SA[2 * c] = __builtin_bit_cast(f16x8, Ws[c * 3 * 128 + kb * 128]);
        SA[2 * c + 1] = __builtin_bit_cast(f16x8, Ws[c * 3 * 128 + kb * 128 + 64]);
      }
      const int tap = 4 * kb + g;
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if ((t & 3) >= NVB) continue;
        const int v = bp_of(t), b = v & 3, p = v >> 2;
        const int r = tap < 9 ? src_row(p, p / 5, p % 5, tap) : ZROW;
        SH[t] = *reinterpret_cast<const f16x8*>(simg + (b * IROWS + r) * 16);
        SL[t] = *reinterpret_cast<const f16x8*>(simg + ((XB + b) * IROWS + r) * 16);
      }
#pragma unroll
      for (int ps = 0; ps < 3; ++ps)
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            if ((t & 3) >= NVB) continue;
            acc[ct * 8 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(SA[2 * ct + (ps == 2)], ps == 1 ? SL[t] : SH[t],
                                                                     acc[ct * 8 + t], 0, 0, 0);
          }
    }
  }
  // the stem's half-0 sums (the epilogue adds the half-1 ones)
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int t = 0; t < 4; ++t) mst[ct * 8 + t] += acc[ct * 8 + t];
  {
    float bnd[4];
#pragma unroll
    for (int b = 0; b < 4; ++b)
      bnd[b] = __builtin_fmaf(W.yrange[2 * CONV_LAYERS], mx_img[b], W.yrange[2 * CONV_LAYERS + 1]) * 1.0009765625f;
    epilogue(W.stemx_inv[0], W.stem_b, std::false_type{}, 0.f, bnd);
    note_xs(0);
  }
  stamp(st_stem);

  // ---------------- residual trunk: 18 convs, activations resident in LDS ----------------
  // Per half-step (k-block u of a row, half h): the MFMAs of the active tiles of half h, pass by
  // pass, in groups of 4 fixed by sched_barrier; spread over the groups, the next half-step's
  // fragment reads (from the table entries read a half-step earlier), the table read of the
  // half-step after that, the next k-block's weight loads (buffer loads into the other slot of a
  // 2-slot register ring) and, at chunk boundaries, the chunk sums' adds into the master sums
  // (half-0 tiles in the chunk's last half-step, half-1 tiles in the next chunk's first one).  The
  // row-gated tile (T in half 0, B in half 1) runs last, behind one uniform branch.
  const int tab_l = IMG_B + AUXB + 16 * lane;
  // the weight ring: RS slots, loads PD k-blocks ahead.  A 4-board k-block runs 60-96 MFMAs, which
  // cover one k-block of load latency; a tail instance's runs 12 x NVB, so its loads go further
  // ahead into the registers its fewer fragment tiles leave free (round 3's depths 5 / 3 / 2).
  // RS divides the 24 k-blocks of a tap row, so a k-block's slot is the same in every row.
  constexpr int PD = TAIL_R3 ? 1 : NVB == 1 ? MTAZ_Y_PD1 : NVB == 2 ? MTAZ_Y_PD2 : NVB == 3 ? 2 : 1, RS = PD + 1;
  static_assert(24 % RS == 0, "weight ring");
  f16x8 A[RS][2 * CT], BH[2][8];
  uint4 tpre;     // table entries of the half-step after next (read during the current one)
  int onx[4];     // table entries (fragment bases, k-block step aside) of the next half-step
  // weights k-block-major (NetWeights::convyk): the wave's fragment (channel tile ct, part) of
  // k-block kb at 32768 kb + 8192 wave + 2048 ct + 1024 part: the lane offset and the tile-pair's
  // 4 KB step in the scalar offset, the rest an immediate
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc((void*)W.convyk, (short)0, 0x7ffffff0, 0x00020000);
  const int voy = wave * 8192 + lane * 16;
  int lofs = 0;   // the layer's byte offset in convyk
  auto wload = [&](f16x8& dst, int kb, int ct, int part) __attribute__((always_inline)) {
    dst = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rsy, voy + ((ct & 1) * 2 + part) * 1024,
                                                                           lofs + kb * 32768 + (ct >> 1) * 4096, 0));
  };
  for (int L = 0; L < CONV_LAYERS; ++L) {
    // layer prologue: k-block 0's weights, half-step (0, 0)'s fragments, the offsets of (0, 1)
#pragma unroll
    for (int kp = 0; kp < (D_NOW ? RS : PD); ++kp)
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        wload(A[kp][2 * c], kp, c, 0);
        wload(A[kp][2 * c + 1], kp, c, 1);
      }
    {
      const uint4 e0 = *reinterpret_cast<const uint4*>(smem + tab_l);
      const uint4 e1 = *reinterpret_cast<const uint4*>(smem + tab_l + 1024);
      const int o[4] = {(int)e0.x, (int)e0.y, (int)e0.z, (int)e0.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < NVB) {
          BH[0][i] = *reinterpret_cast<const f16x8*>(smem + o[i]);
          BH[0][4 + i] = *reinterpret_cast<const f16x8*>(smem + o[i] + PART_B);
        }
      onx[0] = (int)e1.x, onx[1] = (int)e1.y, onx[2] = (int)e1.z, onx[3] = (int)e1.w;
      if constexpr (D_NOF) {   // diagnostic: half 1's fragments too, reused by every k-block
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i < NVB) {
            BH[1][i] = *reinterpret_cast<const f16x8*>(smem + onx[i]);
            BH[1][4 + i] = *reinterpret_cast<const f16x8*>(smem + onx[i] + PART_B);
          }
      }
    }
    for (int j = 0; j < 3; ++j) {   // T (half 0) runs no dr = -1 taps (j = 0), B (half 1) no dr = +1 (j = 2)
      const int tab_j = tab_l + 6144 * j;
      const int tab_n = j < 2 ? tab_j + 6144 : tab_j;   // the next row's table (clamped in-bounds)
      const int kb_j = 24 * j;
      if constexpr (SKIP && NVB == XB) {
        if (j == 0) {   // T runs no k-block of row 0: its (stale) chunk sums must add zeros
#pragma unroll
          for (int ct = 0; ct < CT; ++ct) acc[ct * 8 + 3] = (f32x4v){0};
        }
      }
      sfor<0, 48>([&](auto s_c) __attribute__((always_inline)) {
        constexpr int S = decltype(s_c)::value, U = S >> 1, H = S & 1;
        // the next half-step (U1, H1) and the one after (U2, H2), within the row or the next one
        constexpr int U1 = H ? U + 1 : U, H1 = H ^ 1, U2 = U + 1, H2 = H;
        constexpr int ACTN = (act(NVB, SKIP, U, 4 * H + 0) && !gated(NVB, SKIP, U, 4 * H + 0)) +
                             (act(NVB, SKIP, U, 4 * H + 1) && !gated(NVB, SKIP, U, 4 * H + 1)) +
                             (act(NVB, SKIP, U, 4 * H + 2) && !gated(NVB, SKIP, U, 4 * H + 2)) +
                             (act(NVB, SKIP, U, 4 * H + 3) && !gated(NVB, SKIP, U, 4 * H + 3));
        constexpr int NG = 3 * ACTN;                       // groups of 4 MFMAs
        constexpr int U1r = U1 < 24 ? U1 : U1 - 24;        // the next half-step's k-block in its row
        // fragment reads of (U1, H1): tiles active there at compile time or gated
        constexpr bool need0 = act(NVB, SKIP, U1r, 4 * H1 + 0), need1 = act(NVB, SKIP, U1r, 4 * H1 + 1);
        constexpr bool need2 = act(NVB, SKIP, U1r, 4 * H1 + 2), need3 = act(NVB, SKIP, U1r, 4 * H1 + 3);
        constexpr int NFR = 2 * (need0 + need1 + need2 + need3);
        // + the table read + (half 0) all 8 weight loads of k-block U + PD: a full k-block of MFMAs
        // then covers their latency (a k-block runs 60-96 MFMAs with the tap skip)
        constexpr int NW_ = H == 0 ? 2 * CT : 0;
        constexpr int NQ = NFR + 1 + NW_;
        // memory items per group: at most 2 (3 when the half-step is short), from group 0 on
        constexpr int QPG = (NQ + NG - 1) / NG > 2 ? (NQ + NG - 1) / NG : 2;
        constexpr bool ADD0 = H == 1 && (U == 11 || U == 23);   // half-0 tiles' chunk sums
        constexpr bool ADD1 = H == 0 && (U == 0 || U == 12);    // half-1 tiles' (previous chunk)
        constexpr int NADD = (ADD0 || ADD1) ? 16 : 0;
        if constexpr (SKIP && NVB == XB && S == 1) {   // B runs no k-block of row 2: zero it after its last add
          if (j == 2) {
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) acc[ct * 8 + 7] = (f32x4v){0};
          }
        }
        int o[4] = {onx[0], onx[1], onx[2], onx[3]};
        f16x8 (&BC)[8] = BH[H];
        f16x8 (&BN)[8] = BH[H1];
        f16x8 (&AC)[2 * CT] = A[U % RS];
        f16x8 (&AN)[2 * CT] = A[(U + PD) % RS];
        // group kq issues memory items [q0, q1) and adds [a0, a1)
        sfor<0, NG>([&](auto k_c) __attribute__((always_inline)) {
          constexpr int KQ = decltype(k_c)::value;
          constexpr int q0 = KQ * QPG < NQ ? KQ * QPG : NQ, q1 = (KQ + 1) * QPG < NQ ? (KQ + 1) * QPG : NQ;
          constexpr int a0 = KQ * NADD / NG, a1 = (KQ + 1) * NADD / NG;
          __builtin_amdgcn_sched_barrier(0);
          sfor<q0, q1>([&](auto q_c) __attribute__((always_inline)) {
            constexpr int Q = decltype(q_c)::value;
            if constexpr (Q < NFR) {           // fragment read Q: the (Q / 2)-th needed tile, part Q & 1
              constexpr int nd[4] = {need0, need1, need2, need3};
              constexpr int I = [] {
                int c = 0;
                for (int i = 0; i < 4; ++i)
                  if (nd[i] && c++ == Q / 2) return i;
                return 0;
              }();
              if constexpr (!D_NOF)
                BN[(Q & 1) * 4 + I] = *reinterpret_cast<const f16x8*>(smem + o[I] + 1024 * (U1 & 7) + (Q & 1) * PART_B);
            } else if constexpr (Q == NFR) {   // the table entries of (U2, H2)
              const int ta = U2 < 24 ? tab_j + (U2 / 8) * 2048 + H2 * 1024 : tab_n + ((U2 - 24) / 8) * 2048 + H2 * 1024;
              tpre = *reinterpret_cast<const uint4*>(smem + ta);
            } else {                           // weight load: k-block U + PD, channel tile / part
              constexpr int W_ = Q - NFR - 1, ct = W_ >> 1, part = W_ & 1;
              const int kbn = kb_j + U + PD < KBY ? kb_j + U + PD : KBY - 1;   // (clamped: the layer's last k-blocks)
              if constexpr (!D_NOW) wload(AN[2 * ct + part], kbn, ct, part);
            }
          });
          sfor<a0, a1>([&](auto a_c) __attribute__((always_inline)) {
            constexpr int AI = decltype(a_c)::value, ct = AI >> 2, i = AI & 3;
            constexpr int t = (ADD0 ? 0 : 4) + i;
            if constexpr (i < NVB) ny_add4(mst[ct * 8 + t], acc[ct * 8 + t]);
          });
          __builtin_amdgcn_sched_barrier(0);
          sfor<0, 4>([&](auto m_c) __attribute__((always_inline)) {
            constexpr int M = 4 * KQ + decltype(m_c)::value;   // MFMA M of the half-step's list
            constexpr int ps = M / (4 * ACTN), ct = (M / ACTN) % 4, ii = M % ACTN;
            constexpr int i = [] {
              int c = 0;
              for (int k = 0; k < 4; ++k)
                if (act(NVB, SKIP, U, 4 * H + k) && !gated(NVB, SKIP, U, 4 * H + k) && c++ == ii) return k;
              return 0;
            }();
            constexpr int t = 4 * H + i;
            constexpr bool first = ps == 0 && U == first_u(NVB, SKIP, U, t);
            acc[ct * 8 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AC[2 * ct + (ps == 2)], BC[(ps == 1) * 4 + i],
                                                                     first ? (f32x4v){0} : acc[ct * 8 + t], 0, 0, 0);
          });
        });
        __builtin_amdgcn_sched_barrier(0);
        // the row-gated tile: 4 boards T / B (i = 3, whole rows: a chunk's chain may start here),
        // 3 boards t2 / t6 (i = 2, the dc = +1 k-blocks 16-23: never a chunk's first)
        constexpr int GI = NVB == XB ? 3 : 2;
        if constexpr (gated(NVB, SKIP, U, 4 * H + GI)) {
          constexpr int i = GI, t = 4 * H + i;
          constexpr bool fu = NVB == XB && (U == 0 || U == 12);
          if (j != (H ? 2 : 0)) {
            sfor<0, 12>([&](auto m_c) __attribute__((always_inline)) {
              constexpr int M = decltype(m_c)::value, ps = M / 4, ct = M % 4;
              acc[ct * 8 + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AC[2 * ct + (ps == 2)], BC[(ps == 1) * 4 + i],
                                                                       (fu && ps == 0) ? (f32x4v){0} : acc[ct * 8 + t], 0, 0, 0);
            });
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        onx[0] = (int)tpre.x, onx[1] = (int)tpre.y, onx[2] = (int)tpre.z, onx[3] = (int)tpre.w;
      });
    }
    stamp(st_k);
    lofs += (int)(CONVX_U4_PER_LAYER * 16);
    __syncthreads();   // every wave has finished reading this layer's input image
    // output bounds per board (the margin 1 + 2^-10 covers the rounding of the bound's own arithmetic)
    float bnd[4];
    if ((L & 1) == 0) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        bnd[b] = __builtin_fmaf(W.yrange[2 * L], mx_img[b], W.yrange[2 * L + 1]) * 1.0009765625f;
        mx_blk[b] = mx_img[b];
      }
      epilogue(W.convx_inv[L], W.conv_b + L * 256, std::true_type{}, 1.0f / W.convx_inv[L + 1], bnd);
    } else {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        bnd[b] = (__builtin_fmaf(W.yrange[2 * L], mx_img[b], W.yrange[2 * L + 1]) + mx_blk[b]) * 1.0009765625f;
      epilogue(W.convx_inv[L], W.conv_b + L * 256, std::false_type{}, 0.f, bnd);
    }
    note_xs(1 + L);
    stamp(st_epi);
  }
  if (overflow && !D_NOW && !D_NOF && !D_NOE) atomicOr(D.pr.err, ERR_F16);   // (diagnostic forms: garbage by design)

  // ---------------- heads (exp/policy.py:62-69, :76-79) ------------------------------------
  {
    float* fp = reinterpret_cast<float*>(smem + IMG_B);   // [XB][64]: pconv features (60) + clock
    float* fv = fp + XB * 64;                            // [XB][32]: vconv features (30) + clock
    float* red = fv + XB * 32;                           // [XB][256]
    for (int t = tid; t < XB * 90; t += NT) {
      const int bb = t / 90, o = (t % 90) / 30, p = t % 30;
      const float* wr = o < 2 ? W.pconv_w + o * 256 : W.vconv_w;
      const int cb = cell(bb, p);
      float s = 0.f;
      for (int c = 0; c < 32; ++c) {
        const f16x8 xh = *reinterpret_cast<const f16x8*>(smem + cb + 256 * c);
        const f16x8 xl = *reinterpret_cast<const f16x8*>(smem + cb + 256 * c + PART_B);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += wr[8 * c + j] * ((float)xh[j] + (float)xl[j]);
      }
      const float xsc = __builtin_ldexpf(1.f, sel4(bb, xs[0], xs[1], xs[2], xs[3]));
      s = fmaxf(__builtin_fmaf(s, xsc, o < 2 ? W.pconv_b[o] : W.vconv_b[0]), 0.f);
      if (o < 2) fp[bb * 64 + o * 30 + p] = s; else fv[bb * 32 + p] = s;
    }
    if (tid < XB) {
      const int b = b0 + tid;
      const float clk = b < nb ? clock_of(pos[b]) : 0.f;
      fp[tid * 64 + 60] = clk;
      fv[tid * 32 + 30] = clk;
    }
    __syncthreads();
    if (tid < 256) {
      const int j = tid;
#pragma unroll
      for (int bb = 0; bb < XB; ++bb) {
        float hsum = W.vl1_b[j];
        for (int i = 0; i < 31; ++i) hsum += W.vl1_w[j * 31 + i] * fv[bb * 32 + i];
        red[bb * 256 + j] = W.vl2_w[j] * fmaxf(hsum, 0.f);
      }
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s)
#pragma unroll
        for (int bb = 0; bb < XB; ++bb) red[bb * 256 + tid] += red[bb * 256 + tid + s];
      __syncthreads();
    }
  }
  stamp(st_heads);
  if constexpr (STAMP) {
    if (tid == 0) {
      stamps[bid * 6 + 0] = st_stem;
      stamps[bid * 6 + 1] = st_k;
      stamps[bid * 6 + 2] = st_epi;
      stamps[bid * 6 + 3] = st_heads;
      stamps[bid * 6 + 4] = __builtin_amdgcn_s_memtime() - t_start;
      stamps[bid * 6 + 5] = __builtin_amdgcn_s_memrealtime() - r_start;
    }
    if (tid < 4) stamps[(size_t)gridDim.x * 6 + bid * 4 + tid] = ((unsigned long long)xs_max[tid] << 32) | xs_mask[tid];
  }
  heads_out<true>(D, smem, b0, nb, W, mode, logits_out, values_out, wave, lane);
}

template <bool STAMP, int VAR, int NVB = XB>
__global__ __launch_bounds__(256, 1) void k_net_y(Dev D, NetWeights W, const Pos* __restrict__ pos,
                                                  const int32_t* __restrict__ count, int max_b, int mode,
                                                  float* __restrict__ logits_out, float* __restrict__ values_out,
                                                  unsigned long long* __restrict__ stamps, int ncu) {
  __shared__ __attribute__((aligned(16))) char smem[ny::SMEM_B];
  net_y_body<STAMP, VAR, NVB>(smem, blockIdx.x, D, W, pos, count, max_b, mode, logits_out, values_out, stamps, ncu);
}

// The three tail instances in one launch of 3 x ncu workgroups: workgroup i runs as the
// (1 + i / ncu)-board instance for CU slot i % ncu, and exits at once unless the remainder has that
// many boards per CU
template <int VAR>
__global__ __launch_bounds__(256, 1) void k_net_y_tail(Dev D, NetWeights W, const Pos* __restrict__ pos,
                                                       const int32_t* __restrict__ count, int max_b, int mode,
                                                       float* __restrict__ logits_out,
                                                       float* __restrict__ values_out, int ncu) {
  __shared__ __attribute__((aligned(16))) char smem[ny::SMEM_B];
  const int nvb = 1 + (int)blockIdx.x / ncu, bid = (int)blockIdx.x % ncu;
  if (nvb == 1)
    net_y_body<false, VAR, 1>(smem, bid, D, W, pos, count, max_b, mode, logits_out, values_out, nullptr, ncu);
  else if (nvb == 2)
    net_y_body<false, VAR, 2>(smem, bid, D, W, pos, count, max_b, mode, logits_out, values_out, nullptr, ncu);
  else
    net_y_body<false, VAR, 3>(smem, bid, D, W, pos, count, max_b, mode, logits_out, values_out, nullptr, ncu);
}

static int device_cus_y() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cached[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) n = 0;
    cached[dev] = n > 0 ? n : -1;
  }
  return cached[dev] > 0 ? cached[dev] : 0;
}

// variant 0: the product (full rounds of 4 boards, then the tail launch); 1: 4 boards per
// workgroup throughout (no tail); 2: class tiles without the tap skip, 4 boards throughout;
// 3: round 3's kernel (mtaz_net16_r3.hip, main + tail; diagnostic library only); 5: the product with the first round-4
// build's tail instances (VAR bit 2: off-board cells on the padding squares, 2-way bank conflicts;
// weights one k-block ahead)
void launch_net_f16x3(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                      float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                      int variant) {
  if (max_b <= 0) return;
#ifdef MTAZ_NET_DIAG
  if (variant == 3) {   // round 3's kernel: diagnostic library only
    launch_net_f16x3_r3(d, w, pos, count, max_b, mode, logits_out, values_out, s, ev_begin, ev_end, 0);
    return;
  }
#endif
  if (ev_begin) (void)hipEventRecord(ev_begin, s);
  const int ncu = device_cus_y();
  const dim3 all((max_b + XB - 1) / XB);
  if (variant == 0 && ncu > 0) {
    hipLaunchKernelGGL((k_net_y<false, 0, XB>), all, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, nullptr, ncu);
    hipLaunchKernelGGL((k_net_y_tail<0>), dim3(3 * ncu), dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, ncu);
  } else if (variant == 5 && ncu > 0) {
    hipLaunchKernelGGL((k_net_y<false, 0, XB>), all, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, nullptr, ncu);
    hipLaunchKernelGGL((k_net_y_tail<2>), dim3(3 * ncu), dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, ncu);
  } else if (variant == 2) {
    hipLaunchKernelGGL((k_net_y<false, 1, XB>), all, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, nullptr, 0);
#ifdef MTAZ_NET_DIAG
  } else if (variant == 8 || variant == 16 || variant == 32) {
    // the diagnostic forms, 4 boards per workgroup throughout (tools/bench_net.py --diag)
#define Y_DIAG(V)                                                                                                  \
  if (variant == V)                                                                                                \
    hipLaunchKernelGGL((k_net_y<false, V, XB>), all, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out, \
                       values_out, nullptr, 0);
    Y_DIAG(8) Y_DIAG(16) Y_DIAG(32)
#undef Y_DIAG
#endif
  } else {
    hipLaunchKernelGGL((k_net_y<false, 0, XB>), all, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, nullptr, 0);
  }
  if (ev_end) (void)hipEventRecord(ev_end, s);
}

void launch_net_f16x3_stamped(const Dev& d, const NetWeights& w, const Pos* pos, int n, float* logits_out,
                              float* values_out, unsigned long long* stamps, hipStream_t s, int variant) {
  if (n <= 0) return;
  const dim3 all((n + XB - 1) / XB);
  if (variant == 2)
    hipLaunchKernelGGL((k_net_y<true, 1, XB>), all, dim3(256), 0, s, d, w, pos, nullptr, n, (int)NET_FULL_LOGITS,
                       logits_out, values_out, stamps, 0);
#ifdef MTAZ_NET_DIAG
#define Y_DIAG(V)                                                                                               \
  else if (variant == V) hipLaunchKernelGGL((k_net_y<true, V, XB>), all, dim3(256), 0, s, d, w, pos, nullptr, n, \
                                            (int)NET_FULL_LOGITS, logits_out, values_out, stamps, 0);
  Y_DIAG(8) Y_DIAG(16) Y_DIAG(32)
#undef Y_DIAG
#endif
  else
    hipLaunchKernelGGL((k_net_y<true, 0, XB>), all, dim3(256), 0, s, d, w, pos, nullptr, n, (int)NET_FULL_LOGITS,
                       logits_out, values_out, stamps, 0);
}

}  // namespace mtaz
