// k_net_z: the fused policy/value network (exp/policy.py:71-80 + the leaf priors of
// exp/agent.py:67-69) with the fp16x3 split's cross terms on the block-scaled e4m3 MFMA.
//
// k_net_y computes each conv as Wh*Xh + Wh*Xl + Wl*Xh, three f16 MFMA passes.  The two cross
// terms are 2^-11 of the product, so they need ~2^-11 relative precision only: k_net_z runs
// them on v_mfma_scale_f32_16x16x128_f8f6f4 with OCP e4m3 operands (twice the f16 rate per
// clock, MI355X_MICROARCH.md matrix-core table; 1.8-2.1x the f16 loop's FLOP/s on random data
// in tools/probes/fp8_mfma_probe.hip, at a higher clock) and keeps Wh*Xh on
// v_mfma_f32_16x16x32_f16: 2/3 of k_net_y's MFMA cycles for the same LDS and L2 bytes.
// Emulated end to end (fp64 reference, 300 positions, seed-0 weights, tools/split_error.py) the
// values move by 2e-6 and priors by 2e-8, against fp32's own 4e-8 / 5e-10: inside the 1e-5
// parity bound, not bitwise k_net_y.
//
// Workgroup, tiling, stem, epilogue bound logic and heads are k_net_y's (mtaz_net16.hip).  The
// LDS image keeps 4 B per activation: part 0 = Xh (f16, as k_net_y), part 1 = [Xl8 | Xh8], two
// e4m3 copies (Xl = x - Xh and Xh itself), each in units of a per-layer power of two chosen
// per board from the epilogue's rigorous output bound.  The residual is read back as Xh + Xl8 (precision
// 2^-15 of x, part of the emulation above).
//
// K loop.  A conv's 72 steps s = (tap t, 128-channel chunk c, j): step s runs
//   phase A: f16 MFMAs of k-block s (Wh x Xh, all 8 column tiles)
//   phase B: e4m3 MFMAs (K = 128) of group G = s/2 = (t, c, term) on square tile pt = s&1:
//            term 0: Wh8 x Xl8, term 1: Wl8 x Xh8
// = 1024 MFMA cycles per step and SIMD.  Operands: Wh f16 fragments PD steps ahead, the e4m3
// weight groups GD groups ahead (half a group per step), this step's e4m3 activation
// fragments during phase A and the next step's f16 ones during phase B.
//
// Waves: 8 (2 per SIMD), 16 accumulator tiles each; the wave layouts are described at ZCfg.
#include "net_common.h"

namespace mtaz {

using namespace netc;
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
constexpr int KBZ = 72;      // steps (= f16 k-blocks) per conv
constexpr int GZ = 36;       // e4m3 groups per conv

__device__ __forceinline__ i32x8 cat8(uint4 a, uint4 b) {
  return (i32x8){(int)a.x, (int)a.y, (int)a.z, (int)a.w, (int)b.x, (int)b.y, (int)b.z, (int)b.w};
}

// f32(half of pk) * b + c in one v_fma_mix_f32 (the compiler does not form it with f32
// denormals on).  Bit-identical to the unfused form (round the product, then add) where the
// product f32(half) * b is exact and neither it, c nor the sum is an f32 denormal or overflows:
// the callers' b are powers of two and the operands are normal-range activations (a denormal
// sum would be flushed differently by the mix path); test_z_mix_epilogue_bit_identical checks
// ordinary and wide-range nets
__device__ __forceinline__ float zmix_lo(uint32_t pk, float b, float c) {
  float r;
  asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(pk), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float zmix_hi(uint32_t pk, float b, float c) {
  float r;
  asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(pk), "v"(b), "v"(c));
  return r;
}

typedef short zv2i16 __attribute__((ext_vector_type(2)));
typedef _Float16 zv2f16 __attribute__((ext_vector_type(2)));
// gfx950's scaled conversions: e4m3 of x / s (encode) and x * s (decode) for a power-of-two s,
// bitwise the unscaled conversion of the exactly scaled value (tools/probes/cvt_scale_probe.hip,
// profiles/r02_tap/cvt_scale_probe.json: 65,536 random pairs per scale 2^-24..2^24, all equal)
__device__ __forceinline__ uint32_t sc_fp8x4(float a, float b, float c, float d, float s) {
  zv2i16 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32((zv2i16){0, 0}, a, b, s, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(r, c, d, s, true);
  return __builtin_bit_cast(uint32_t, r);
}
__device__ __forceinline__ uint32_t sc_fp8x4_f16(uint32_t h01, uint32_t h23, float s) {
  zv2i16 r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16((zv2i16){0, 0}, __builtin_bit_cast(zv2f16, h01), s, false);
  r = __builtin_amdgcn_cvt_scalef32_pk_fp8_f16(r, __builtin_bit_cast(zv2f16, h23), s, true);
  return __builtin_bit_cast(uint32_t, r);
}

// max over the wave's 64 lanes, in every lane: lanes i ^ 32 and i ^ 16 by gfx950's permlane
// swaps, then row rotations by 8 and 4 and quad permutations by DPP (VALU only, instead of six
// dependent ds_bpermute rounds through the LDS: epilogue share 8.1% -> 7.8% of the cycles,
// profiles/r02_final/ab_wave_max_dpp.json); max is exact, so any order gives the same value
__device__ __forceinline__ float wave_max_dpp(float x) {
  uint32_t u = __float_as_uint(x);
  const auto r32 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  x = fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
  u = __float_as_uint(x);
  const auto r16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  x = fmaxf(x, __uint_as_float(__builtin_amdgcn_update_dpp(0, (int)__float_as_uint(x), 0x128, 0xf, 0xf, false)));
  x = fmaxf(x, __uint_as_float(__builtin_amdgcn_update_dpp(0, (int)__float_as_uint(x), 0x124, 0xf, 0xf, false)));
  x = fmaxf(x, __uint_as_float(__builtin_amdgcn_update_dpp(0, (int)__float_as_uint(x), 0x4e, 0xf, 0xf, false)));
  x = fmaxf(x, __uint_as_float(__builtin_amdgcn_update_dpp(0, (int)__float_as_uint(x), 0xb1, 0xf, 0xf, false)));
  return x;
}

// 4 e4m3 bytes of {a, b, c, d} (round to nearest even, OCP e4m3fn)
__device__ __forceinline__ uint32_t pk_fp8x4(float a, float b, float c, float d) {
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (uint32_t)r;
}

// Wave layout.  VAR 0: 8 waves, wave w owns output channels [32w, 32w + 32) (CT = 2 channel tiles)
// on all 4 boards.  Diagnostic library only: VAR 4194304 (board pairs), 8 waves as 4 channel
// groups x 2 board pairs, wave w owning channels [64(w&3), +64) (CT = 4) on boards 2(w>>2) and
// 2(w>>2) + 1: the same 16 accumulator tiles per wave with half the LDS bytes per MFMA and twice
// the weight loads; bit-identical results, 3% more cycles at a 5% lower clock.
// VAR 2048: 4 waves of 64 channels on all 4 boards.
// NVB: boards the workgroup computes (4; 1..3 in the tail launches, see k_net_z): boards
// NVB..3 of the LDS image are never computed.
template <int VAR, int NVB = XB>
struct ZCfg {
  static constexpr bool BP = (VAR & 4194304) != 0;
  static constexpr int NW = (VAR & 2048) ? 4 : 8;   // waves
  static constexpr int NBG = BP ? 2 : 1;            // board groups
  static constexpr int BPW = BP ? 2 : NVB;          // boards per wave
  static constexpr int CT = BP ? 4 : 16 / NW;       // channel tiles (of 16) per wave
  static constexpr int NCG = 16 / CT;               // channel groups
  static constexpr int TW = 2 * BPW;                // column tiles (board x square tile) per wave
  static_assert(NCG * NBG == NW && (BP ? NVB == XB : NVB >= 1 && NVB <= XB), "waves cover channel groups x board groups");
};

// element bb of a 4-board register array with a wave-uniform runtime index, without a
// dynamically indexed local array (which would live in scratch)
template <class T>
__device__ __forceinline__ T pick4(const T* a, int bb) {
  return bb == 0 ? a[0] : bb == 1 ? a[1] : bb == 2 ? a[2] : a[3];
}

// Board assignment.  One workgroup holds a CU (its LDS image), so a launch runs in rounds of ncu
// workgroups; with 4 boards each, n boards took ceil(n / 4 ncu) rounds and the last one was often
// mostly idle (3,327 leaves: 832 workgroups, a fourth round with 64 of 256 CUs busy).  With
// ncu > 0 the R = n mod 4 ncu boards beyond the full rounds need per = ceil(R / ncu) boards per
// CU; if per < 4 they go to the tail launch k_net_z<NVB = per> instead, ceil(R / per) workgroups
// that compute only their NVB boards, so the last round takes the time of its fewer boards per CU
// (launch_net_z launches NVB = 1, 2, 3 after the full-round launch; the two that do not match exit
// at once).  A board's result does not depend on the other boards of its workgroup (per-board e4m3
// scales), so the assignment changes nothing but the time.  ncu = 0: 4 boards per workgroup
// throughout (the other builds, the stamped diagnostics).
template <bool STAMP, int VAR, int NVB = XB>
__global__ __launch_bounds__(64 * ZCfg<VAR>::NW, 1) void k_net_z(Dev D, NetWeights W, const Pos* __restrict__ pos,
                                                                 const int32_t* __restrict__ count, int max_b,
                                                                 int mode, float* __restrict__ logits_out,
                                                                 float* __restrict__ values_out,
                                                                 unsigned long long* __restrict__ stamps, int ncu) {
  using C = ZCfg<VAR, NVB>;
  constexpr int NW = C::NW, NT = 64 * NW, CT = C::CT, BPW = C::BPW, TW = C::TW;
  constexpr bool F6 = (VAR & 8192) != 0;   // cross terms in e2m3 blocks (epilogue6, NetWeights::conv6)
  // 268435456 (W3): k_net_y's arithmetic (all three split products on the f16 MFMA, fp32-accurate)
  // in this kernel's structure: part 1 of the image holds Xl = f16(y - Xh) instead of the e4m3
  // copies, and each K step runs Wh*Xh and Wl*Xh on the step's Xh fragments, then Wh*Xl on its Xl
  // fragments (Wl: the lo part of convz), 48 f16 MFMAs per wave and step
  constexpr bool W3 = (VAR & 268435456) != 0;
  static_assert(!(W3 && F6), "W3 has no e2m3 form");
  // diagnostic builds (timing only, wrong results): 16384 = every layer reads layer 0's weights
  // (an L2-resident weight set), 32768 = every step reads k-block / group 0 (L1-resident)
  constexpr bool DIAG_L2 = (VAR & 16384) != 0, DIAG_L1 = (VAR & 32768) != 0;
  // 65536 = no cross-term MFMAs (phase B issues its loads only), 131072 = no activation LDS reads
  // in the K loop (the fragments of step 0 are reused)
  constexpr bool DIAG_NOB = (VAR & 65536) != 0, DIAG_NOLDS = (VAR & 131072) != 0;
  // 1048576: static issue priority 1 for the second-dispatched half of the waves (the arbitration
  // loser of each SIMD pair, MI355X_MICROARCH.md "Two waves per SIMD" item 4)
  constexpr bool PRIO = (VAR & 1048576) != 0;
  // 2097152: the e4m3 epilogue's unfused form (product: v_fma_mix for the lo part, the Xh copy and
  // the residual seed; bit-identical, test_gpu_net.py test_z_mix_epilogue_bit_identical)
  constexpr bool NOMIX = (VAR & 2097152) != 0;
  // Product epilogue: its power-of-two scalings folded into gfx950's scaled conversions (the Xl8 /
  // Xh8 copies and the residual seed's Xl8 decode; -35% epilogue VALU).  33554432 = the round-2
  // form (v_fma_mix scalings, unscaled conversions); bit-identical (test_z_mix_epilogue_bit_identical
  // against the unfused form)
  constexpr bool SCVT = (VAR & 33554432) == 0 && !NOMIX && !F6 && !W3;   // (e2m3: more spills with it)
  // K-loop form.  Product: tap-major (one tap = 8 steps per iteration; a fragment's LDS offset is a
  // per-tap base plus a step constant, selected against the zero cell by the tap's on-board mask,
  // 2-3 VALU per address) with the weight fragments by buffer loads (descriptor + per-wave lane
  // offset, the layer / step offset in an SGPR).  8388608 = the round-2 loop (the source square's
  // offset recomputed per step and fragment), 16777216 = weights by 64-bit global addresses; all
  // four forms bit-identical (test_z_loop_forms_bit_identical).  31 -> 11 VALU and 17 -> 7 SALU
  // per step: -8.5% workgroup cycles, -5.7% launch time (profiles/r02_tap/).
  // (Wh fragments 3 steps ahead instead of 1: +0.7% time, 7 spilled registers; not kept)
  // the A16 ring (PD + 1, below): 2 with 8 waves; with 4 waves 4 in the tap-major loop, 3 in the
  // round-2 one
  constexpr int RA0 = NW == 8 ? 2 : (VAR & 8388608) ? 3 : 4;
  // (The e2m3 build spills some registers in either loop, 18 in the round-2 one and 23 in the
  // tap-major one, which is still 5% faster; with buffer-loaded weights it spills 30.)
  constexpr bool TAPA = (VAR & 8388608) == 0 && !DIAG_NOLDS && 8 % RA0 == 0;
  constexpr bool WBUF = (VAR & 16777216) == 0 && !F6;
  __shared__ __attribute__((aligned(16))) char smem[ZIMGB + AUXB];
  int b0, nb;
  {
    const int n = count ? *count : max_b;
    const int r = ncu > 0 ? n % (XB * ncu) : 0, per = ncu > 0 ? (r + ncu - 1) / ncu : XB;
    if constexpr (NVB == XB) {   // the full rounds (and a tail of 4 boards per CU)
      b0 = blockIdx.x * XB;
      nb = per < XB ? n - r : n;
    } else {                     // the tail, when it has NVB boards per CU
      if (per != NVB) return;
      b0 = n - r + blockIdx.x * NVB;
      nb = b0 + NVB < n ? b0 + NVB : n;
    }
  }
  if (b0 >= nb) return;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, n = lane & 15, g = lane >> 4;
  const int wc = wave % C::NCG, wb0 = BPW * (wave / C::NCG);   // channel group, first board
  unsigned long long t_prev = 0, st_stem = 0, st_k = 0, st_epi = 0, st_heads = 0;
  unsigned long long t_start = 0, r_start = 0;
  if constexpr (STAMP) {
    t_prev = t_start = __builtin_amdgcn_s_memtime();
    r_start = __builtin_amdgcn_s_memrealtime();
  }
  auto stamp = [&](unsigned long long& acc) {
    if constexpr (STAMP) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      acc += t - t_prev;
      t_prev = t;
    }
  };

  const int p1 = 16 + n;
  const int ph0 = n / 5, pw0 = n % 5, ph1 = p1 / 5, pw1 = p1 % 5;
  // accumulator tile ct * TW + 2 j + pt: channel tile ct, board wb0 + j, square tile pt
  f32x4v acc[CT * TW];
#pragma unroll
  for (int i = 0; i < CT * TW; ++i) acc[i] = (f32x4v){0};
  int overflow = 0;

  // dynamic range (k_net_y): the image holds x * 2^-xs, one xs per workgroup (0 for any ordinary
  // net).  mxb[bb] = max of board bb's current image, measured by the epilogue that stored it.
  int xs = 0, zrange = 0;   // zrange: some layer's exponent left 0 (ERR_ZRANGE)
  float mxb[XB], mxblk[XB];
#pragma unroll
  for (int bb = 0; bb < XB; ++bb) mxb[bb] = W.yrange[2 * CONV_LAYERS + 2], mxblk[bb] = 0.f;
  unsigned* mxs = reinterpret_cast<unsigned*>(smem + ZIMGB + AUXB - 4 * 2 * XB);   // [slot 2][board]
  if (tid < 2 * XB) mxs[tid] = 0u;
  int slot = 0;
  // e4m3 exponents of board bb's current image: Xh8 = e4m3(Xh * 2^sh[bb]),
  // Xl8 = e4m3(Xl * 2^(sh[bb] + 11)).  Per board (from the board's own bound), so a board's
  // results do not depend on the boards it shares a workgroup with.
  int sh[XB] = {0, 0, 0, 0};

  // per-board maxima of the wave's new outputs -> the workgroup's per-board maxima (mxb) after the
  // epilogue's barrier; y >= 0, so float bits order as values
  auto publish_max = [&](float* ymax, int xo) {
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      ymax[j] = wave_max_dpp(ymax[j]);
    }
    if (lane < BPW) {
      float m = ymax[0];
#pragma unroll
      for (int j = 1; j < BPW; ++j) m = lane == j ? ymax[j] : m;
      atomicMax(&mxs[slot * XB + wb0 + lane], __float_as_uint(m));
    }
    if (tid < XB) mxs[(slot ^ 1) * XB + tid] = 0u;   // every wave read them before this epilogue's barrier
    xs = xo;
    zrange |= xo;
    __syncthreads();
#pragma unroll
    for (int bb = 0; bb < XB; ++bb) {
      mxb[bb] = __builtin_ldexpf(__uint_as_float(mxs[slot * XB + bb]), xo);
      if (!__builtin_isfinite(mxb[bb])) overflow = 1;
    }
    slot ^= 1;
  };

  // Epilogue: y = ReLU(acc * 2^(xs - e - xo) + bias * 2^-xo) in stored units; part 0 <- f16(y),
  // part 1 <- e4m3 copies of y - f16(y) and f16(y).  Conv A seeds conv B's accumulators with the
  // block input Xh + Xl8 (conv B's units), read before its own store.  The weights' row order
  // (NetWeights::convz) gives lane g of tile pair cp the 8 consecutive channels
  // cb = 32 (CT/2 wc + cp) + 8 g .. cb + 7 (4 in each tile): per square one 16-B f16 store and two
  // 8-B e4m3 stores.
  // boundb[bb]: rigorous bound on board bb's outputs (true units); the workgroup's xo follows
  // their max, as k_net_y's
  auto epilogue = [&](float inv, const float* bias, auto conv_a_t, float s_next, const float* boundb) {
    constexpr bool conv_a = decltype(conv_a_t)::value;
    // the lane's coordinates, opaque here: otherwise the compiler hoists the epilogue's LDS
    // addresses out of the layer loop and spills them, and every tile then waits on a scratch
    // reload
    int el = lane;
    asm volatile("" : "+v"(el));
    const int n = el & 15, g = el >> 4, p1 = 16 + n;
    const float bound = fmaxf(fmaxf(boundb[0], boundb[1]), fmaxf(boundb[2], boundb[3]));
    const int xo = bound >= 16384.f ? (int)((__float_as_uint(bound) >> 23) & 0xffu) - 127 - 14 : 0;
    const float in_scale = __builtin_ldexpf(inv, xs - xo), st = __builtin_ldexpf(1.f, -xo);
    const float sseed = __builtin_ldexpf(s_next, xs - xo);
    // board bb's stored values are <= boundb[bb] * 2^-xo =: bs; sh_new = 7 - ilogb(bs) keeps
    // e4m3(Xh * 2^sh) < 256 (clamped so that 2^(sh + 11) stays a normal float)
    int sh_new[XB];
    float hs[BPW], ls[BPW], ls_in[BPW], ihs[BPW], ils[BPW];
#pragma unroll
    for (int bb = 0; bb < XB; ++bb) {
      const float bs = __builtin_ldexpf(boundb[bb], -xo);
      const int eb = bs > 0.f ? (int)((__float_as_uint(bs) >> 23) & 0xffu) - 127 : -126;
      int e = bs < __builtin_inff() ? 7 - eb : 0;
      sh_new[bb] = e > 60 ? 60 : e < -60 ? -60 : e;
    }
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int snew = pick4(sh_new, wb0 + j), sold = pick4(sh, wb0 + j);
      hs[j] = __builtin_ldexpf(1.f, snew);
      ls[j] = __builtin_ldexpf(1.f, snew + 11);
      ihs[j] = __builtin_ldexpf(1.f, -snew);
      ils[j] = __builtin_ldexpf(1.f, -(snew + 11));
      ls_in[j] = __builtin_ldexpf(sseed, -(sold + 11));   // Xl8 units of the image being read
    }
    float ymax[BPW];
#pragma unroll
    for (int j = 0; j < BPW; ++j) ymax[j] = 0.f;
#pragma unroll
    for (int cp = 0; cp < CT / 2; ++cp) {
      const int cb = 32 * ((CT / 2) * wc + cp) + 8 * g;
      float bv[8];
      {
        const float4 b0 = *reinterpret_cast<const float4*>(bias + cb);
        const float4 b1 = *reinterpret_cast<const float4*>(bias + cb + 4);
        bv[0] = b0.x * st; bv[1] = b0.y * st; bv[2] = b0.z * st; bv[3] = b0.w * st;
        bv[4] = b1.x * st; bv[5] = b1.y * st; bv[6] = b1.z * st; bv[7] = b1.w * st;
      }
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int j = t >> 1, bb = wb0 + j, pt = t & 1;
        f32x4v& a0 = acc[(2 * cp) * TW + t];
        f32x4v& a1 = acc[(2 * cp + 1) * TW + t];
        if (pt == 0 || p1 < 30) {
          const int p = pt ? p1 : n;
          const int ah = zoff(0, bb, p, cb >> 3);                       // Xh: 16 B
          const int al8 = zoff(1, bb, p, cb >> 4) + (cb & 15);          // Xl8: 8 B
          const int ah8 = zoff(1, bb, p, 16 + (cb >> 4)) + (cb & 15);   // Xh8: 8 B
          float y[8];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            y[i] = fmaxf(__builtin_fmaf(a0[i], in_scale, bv[i]), 0.f);
            y[4 + i] = fmaxf(__builtin_fmaf(a1[i], in_scale, bv[4 + i]), 0.f);
          }
          ymax[j] = fmaxf(ymax[j], fmaxf(fmaxf(fmaxf(y[0], y[1]), fmaxf(y[2], y[3])),
                                         fmaxf(fmaxf(y[4], y[5]), fmaxf(y[6], y[7]))));
          if constexpr (conv_a && W3) {
            // seed conv B with the block input Xh + Xl (both f16, part 0 / part 1), in conv B's units
            const uint4 xp = *reinterpret_cast<const uint4*>(smem + ah);
            const uint4 xq = *reinterpret_cast<const uint4*>(smem + ah + ZPART);
            a0[0] = zmix_lo(xp.x, sseed, zmix_lo(xq.x, sseed, 0.f));
            a0[1] = zmix_hi(xp.x, sseed, zmix_hi(xq.x, sseed, 0.f));
            a0[2] = zmix_lo(xp.y, sseed, zmix_lo(xq.y, sseed, 0.f));
            a0[3] = zmix_hi(xp.y, sseed, zmix_hi(xq.y, sseed, 0.f));
            a1[0] = zmix_lo(xp.z, sseed, zmix_lo(xq.z, sseed, 0.f));
            a1[1] = zmix_hi(xp.z, sseed, zmix_hi(xq.z, sseed, 0.f));
            a1[2] = zmix_lo(xp.w, sseed, zmix_lo(xq.w, sseed, 0.f));
            a1[3] = zmix_hi(xp.w, sseed, zmix_hi(xq.w, sseed, 0.f));
          } else if constexpr (conv_a) {
            const uint2 xl = *reinterpret_cast<const uint2*>(smem + al8);
            if constexpr (NOMIX) {
              const f16x8 xh = *reinterpret_cast<const f16x8*>(smem + ah);
#define Z_SEED(A, X, I, O) A[I] = __builtin_fmaf((float)xh[(O) + (I)], sseed, __builtin_amdgcn_cvt_f32_fp8((int)X, I) * ls_in[j])
              Z_SEED(a0, xl.x, 0, 0); Z_SEED(a0, xl.x, 1, 0); Z_SEED(a0, xl.x, 2, 0); Z_SEED(a0, xl.x, 3, 0);
              Z_SEED(a1, xl.y, 0, 4); Z_SEED(a1, xl.y, 1, 4); Z_SEED(a1, xl.y, 2, 4); Z_SEED(a1, xl.y, 3, 4);
#undef Z_SEED
            } else if constexpr (SCVT) {
              const uint4 xp = *reinterpret_cast<const uint4*>(smem + ah);
              const auto d0 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(xl.x, ls_in[j], false);
              const auto d1 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(xl.x, ls_in[j], true);
              const auto d2 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(xl.y, ls_in[j], false);
              const auto d3 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(xl.y, ls_in[j], true);
              a0[0] = zmix_lo(xp.x, sseed, d0[0]);
              a0[1] = zmix_hi(xp.x, sseed, d0[1]);
              a0[2] = zmix_lo(xp.y, sseed, d1[0]);
              a0[3] = zmix_hi(xp.y, sseed, d1[1]);
              a1[0] = zmix_lo(xp.z, sseed, d2[0]);
              a1[1] = zmix_hi(xp.z, sseed, d2[1]);
              a1[2] = zmix_lo(xp.w, sseed, d3[0]);
              a1[3] = zmix_hi(xp.w, sseed, d3[1]);
            } else {
              const uint4 xp = *reinterpret_cast<const uint4*>(smem + ah);
              a0[0] = zmix_lo(xp.x, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.x, 0) * ls_in[j]);
              a0[1] = zmix_hi(xp.x, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.x, 1) * ls_in[j]);
              a0[2] = zmix_lo(xp.y, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.x, 2) * ls_in[j]);
              a0[3] = zmix_hi(xp.y, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.x, 3) * ls_in[j]);
              a1[0] = zmix_lo(xp.z, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.y, 0) * ls_in[j]);
              a1[1] = zmix_hi(xp.z, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.y, 1) * ls_in[j]);
              a1[2] = zmix_lo(xp.w, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.y, 2) * ls_in[j]);
              a1[3] = zmix_hi(xp.w, sseed, __builtin_amdgcn_cvt_f32_fp8((int)xl.y, 3) * ls_in[j]);
            }
          } else {
            a0 = (f32x4v){0};
            a1 = (f32x4v){0};
          }
          f16x8 yh;
#pragma unroll
          for (int q = 0; q < 8; ++q) yh[q] = (_Float16)y[q];
          if constexpr (W3) {
            // part 0 <- Xh = f16(y), part 1 <- Xl = f16(y - Xh) (the difference is exact)
            const uint4 yp = __builtin_bit_cast(uint4, yh);
            const uint32_t yw[4] = {yp.x, yp.y, yp.z, yp.w};
            f16x8 yl;
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
              yl[q] = (_Float16)zmix_lo(yw[q >> 1], -1.f, y[q]);
              yl[q + 1] = (_Float16)zmix_hi(yw[q >> 1], -1.f, y[q + 1]);
            }
            *reinterpret_cast<f16x8*>(smem + ah) = yh;
            *reinterpret_cast<f16x8*>(smem + ah + ZPART) = yl;
            continue;
          }
          if constexpr (SCVT) {
            // d = y - h exactly (Sterbenz), Xl8 = e4m3(d * ls), Xh8 = e4m3(h * hs) by the scaled
            // conversions (x / s: s = 1 / ls, 1 / hs, powers of two)
            const uint4 yp = __builtin_bit_cast(uint4, yh);
            const uint32_t yw[4] = {yp.x, yp.y, yp.z, yp.w};
            float d[8];
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
              d[q] = zmix_lo(yw[q >> 1], -1.f, y[q]);
              d[q + 1] = zmix_hi(yw[q >> 1], -1.f, y[q + 1]);
            }
            *reinterpret_cast<f16x8*>(smem + ah) = yh;
            *reinterpret_cast<uint2*>(smem + al8) = make_uint2(sc_fp8x4(d[0], d[1], d[2], d[3], ils[j]),
                                                               sc_fp8x4(d[4], d[5], d[6], d[7], ils[j]));
            *reinterpret_cast<uint2*>(smem + ah8) = make_uint2(sc_fp8x4_f16(yw[0], yw[1], ihs[j]),
                                                               sc_fp8x4_f16(yw[2], yw[3], ihs[j]));
            continue;
          }
          float h[8], l[8];
          if constexpr (NOMIX) {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              h[q] = (float)yh[q];
              l[q] = (y[q] - h[q]) * ls[j];   // exact difference, power-of-two scale
              h[q] *= hs[j];
            }
          } else {
            // l = y ls - h ls (= (y - h) ls, exact) and h hs straight from the packed halves
            const uint4 yp = __builtin_bit_cast(uint4, yh);
            const uint32_t yw[4] = {yp.x, yp.y, yp.z, yp.w};
            const float nl = -ls[j];
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
              l[q] = zmix_lo(yw[q >> 1], nl, y[q] * ls[j]);
              l[q + 1] = zmix_hi(yw[q >> 1], nl, y[q + 1] * ls[j]);
              h[q] = zmix_lo(yw[q >> 1], hs[j], 0.f);
              h[q + 1] = zmix_hi(yw[q >> 1], hs[j], 0.f);
            }
          }
          *reinterpret_cast<f16x8*>(smem + ah) = yh;
          *reinterpret_cast<uint2*>(smem + al8) = make_uint2(pk_fp8x4(l[0], l[1], l[2], l[3]), pk_fp8x4(l[4], l[5], l[6], l[7]));
          *reinterpret_cast<uint2*>(smem + ah8) = make_uint2(pk_fp8x4(h[0], h[1], h[2], h[3]), pk_fp8x4(h[4], h[5], h[6], h[7]));
        } else {
          a0 = (f32x4v){0};
          a1 = (f32x4v){0};
        }
      }
    }
#pragma unroll
    for (int bb = 0; bb < XB; ++bb) sh[bb] = sh_new[bb];
    publish_max(ymax, xo);
  };

  // VAR 8192 epilogue: the cross-term copies in e2m3 (fp6) blocks instead of e4m3 bytes.  The
  // wave's channel tiles pair up into 32-channel blocks blk = (CT/2) wc + bi (= K block 4c + g of
  // the next conv's 128-channel chunk c), and per square its lane g holds channels 8 g + 4 ct + i
  // (ct < 2, i < 4) of the block (NetWeights::convz row order): values 8 g + 4 ct + i of the
  // block's 32-value fp6 vector, bits 48 g .. 48 g + 47 = bytes 6 g .. 6 g + 5
  // of the 32-B block slot (term 0: Xl, chunks 2 blk, 2 blk + 1 of part 1; term 1: Xh, chunks
  // 16 + 2 blk, 17 + 2 blk), its e8m0 scale at byte 24.  The scale covers the block's largest
  // |value| (a rounded-up 16-bit key, max over the 4 lanes g), so that every value is <= 7.5 in
  // scaled units; codes by e4m3 RNE of v * 2^(-s-6) (fp6_scale_probe).
  auto epilogue6 = [&](float inv, const float* bias, auto conv_a_t, float s_next, const float* boundb) {
    constexpr bool conv_a = decltype(conv_a_t)::value;
    int el = lane;
    asm volatile("" : "+v"(el));
    const int n = el & 15, g = el >> 4, p1 = 16 + n;
    const float bound = fmaxf(fmaxf(boundb[0], boundb[1]), fmaxf(boundb[2], boundb[3]));
    const int xo = bound >= 16384.f ? (int)((__float_as_uint(bound) >> 23) & 0xffu) - 127 - 14 : 0;
    const float in_scale = __builtin_ldexpf(inv, xs - xo), st = __builtin_ldexpf(1.f, -xo);
    const float sseed = __builtin_ldexpf(s_next, xs - xo);
    float ymax[BPW];
#pragma unroll
    for (int j = 0; j < BPW; ++j) ymax[j] = 0.f;
#pragma unroll
    for (int bi = 0; bi < CT / 2; ++bi) {
      const int blk = (CT / 2) * wc + bi;
      const int o32 = (g & 1) ? 6 * g + 2 : 6 * g, o16 = (g & 1) ? 6 * g : 6 * g + 4, osc = 24;
      float4 bv[2];
  #pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const float4 bu = *reinterpret_cast<const float4*>(bias + 32 * blk + 8 * g + 4 * ct);
        bv[ct] = make_float4(bu.x * st, bu.y * st, bu.z * st, bu.w * st);
      }
      // byte address of byte `b` of block blk's slot of term `term` on row p of board bb
      auto baddr = [&](int term, int bb, int p, int b) { return zoff(1, bb, p, 16 * term + 2 * blk + (b >> 4)) + (b & 15); };
  #pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int j = t >> 1, bb = wb0 + j, pt = t & 1;
        const bool valid = pt == 0 || p1 < 30;
        const int p = pt ? (valid ? p1 : ZROW) : n;
        float y[8];
  #pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const f32x4v& a = acc[(2 * bi + ct) * TW + t];
          y[4 * ct + 0] = fmaxf(__builtin_fmaf(a[0], in_scale, bv[ct].x), 0.f);
          y[4 * ct + 1] = fmaxf(__builtin_fmaf(a[1], in_scale, bv[ct].y), 0.f);
          y[4 * ct + 2] = fmaxf(__builtin_fmaf(a[2], in_scale, bv[ct].z), 0.f);
          y[4 * ct + 3] = fmaxf(__builtin_fmaf(a[3], in_scale, bv[ct].w), 0.f);
        }
        if (!valid) {
  #pragma unroll
          for (int k = 0; k < 8; ++k) y[k] = 0.f;
        }
  #pragma unroll
        for (int k = 0; k < 8; ++k) ymax[j] = fmaxf(ymax[j], y[k]);
        if constexpr (conv_a) {
          // seed conv B with the block input Xh + Xl (conv B's units)
          float xin[8];
          if (valid) {
            const uint32_t r32 = *reinterpret_cast<const uint32_t*>(smem + baddr(0, bb, p, o32));
            const uint32_t r16 = *reinterpret_cast<const uint16_t*>(smem + baddr(0, bb, p, o16));
            const int sb = *reinterpret_cast<const uint8_t*>(smem + baddr(0, bb, p, osc));
            const uint32_t P0 = (g & 1) ? (r16 | (r32 << 16)) : r32, P1 = (g & 1) ? (r32 >> 16) : r16;
            const uint32_t A24 = P0 & 0xffffffu, B24 = (P0 >> 24) | (P1 << 8);
            const float lsc = __builtin_ldexpf(sseed, sb - 127 + 6);
  #pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
              const uint32_t c = ct ? B24 : A24;
              uint32_t e = (c & 0x3fu) | ((c << 2) & 0x3f00u) | ((c << 4) & 0x3f0000u) | ((c << 6) & 0x3f000000u);
              e = (e & 0x1f1f1f1fu) | ((e & 0x20202020u) << 2);
              const f16x4 xh = *reinterpret_cast<const f16x4*>(smem + zoff(0, bb, p, 4 * blk + g) + 8 * ct);
              xin[4 * ct + 0] = __builtin_fmaf((float)xh[0], sseed, __builtin_amdgcn_cvt_f32_fp8((int)e, 0) * lsc);
              xin[4 * ct + 1] = __builtin_fmaf((float)xh[1], sseed, __builtin_amdgcn_cvt_f32_fp8((int)e, 1) * lsc);
              xin[4 * ct + 2] = __builtin_fmaf((float)xh[2], sseed, __builtin_amdgcn_cvt_f32_fp8((int)e, 2) * lsc);
              xin[4 * ct + 3] = __builtin_fmaf((float)xh[3], sseed, __builtin_amdgcn_cvt_f32_fp8((int)e, 3) * lsc);
            }
          } else {
  #pragma unroll
            for (int k = 0; k < 8; ++k) xin[k] = 0.f;
          }
  #pragma unroll
          for (int ct = 0; ct < 2; ++ct)
            acc[(2 * bi + ct) * TW + t] = (f32x4v){xin[4 * ct], xin[4 * ct + 1], xin[4 * ct + 2], xin[4 * ct + 3]};
        } else {
  #pragma unroll
          for (int ct = 0; ct < 2; ++ct) acc[(2 * bi + ct) * TW + t] = (f32x4v){0};
        }
        // hi / lo split, block keys: bf16 bits rounded up (>= the value) of max h, max |l|
        float h[8], l[8], mh = 0.f, ml = 0.f;
        f16x4 yh[2];
  #pragma unroll
        for (int k = 0; k < 8; ++k) {
          const _Float16 hh = (_Float16)y[k];
          yh[k >> 2][k & 3] = hh;
          h[k] = (float)hh;
          l[k] = y[k] - h[k];
          mh = fmaxf(mh, h[k]);
          ml = fmaxf(ml, fabsf(l[k]));
        }
        uint32_t key = (((__float_as_uint(mh) + 0xffffu) >> 16) << 16) | ((__float_as_uint(ml) + 0xffffu) >> 16);
        {
          // max over the 4 lanes g of square n (lanes n + 16 g): v_permlane32_swap (lane i <->
          // i + 32) then v_permlane16_swap (odd <-> even 16-lane rows), VALU ops instead of two
          // dependent ds_bpermute round trips
          const auto r32 = __builtin_amdgcn_permlane32_swap(key, key, false, false);
          key = (max(r32[0] >> 16, r32[1] >> 16) << 16) | max(r32[0] & 0xffffu, r32[1] & 0xffffu);
          const auto r16 = __builtin_amdgcn_permlane16_swap(key, key, false, false);
          key = (max(r16[0] >> 16, r16[1] >> 16) << 16) | max(r16[0] & 0xffffu, r16[1] & 0xffffu);
        }
        if (valid) {
  #pragma unroll
          for (int ct = 0; ct < 2; ++ct)
            *reinterpret_cast<f16x4*>(smem + zoff(0, bb, p, 4 * blk + g) + 8 * ct) = yh[ct];
        }
  #pragma unroll
        for (int term = 0; term < 2; ++term) {
          const uint32_t K = term ? key >> 16 : key & 0xffffu;
          int s = (int)((K >> 7) & 0xffu) - 129 + ((K & 0x7fu) > 112u ? 1 : 0);
          s = s < -120 ? -120 : s > 120 ? 120 : s;
          const float f = __builtin_ldexpf(1.f, -s - 6);
          const float* v = term ? h : l;
          uint32_t c24[2];
  #pragma unroll
          for (int ct = 0; ct < 2; ++ct) {
            uint32_t d = pk_fp8x4(v[4 * ct] * f, v[4 * ct + 1] * f, v[4 * ct + 2] * f, v[4 * ct + 3] * f);
            d = (d & 0x1f1f1f1fu) | ((d >> 2) & 0x20202020u);
            c24[ct] = (d & 0x3fu) | ((d >> 2) & 0xfc0u) | ((d >> 4) & 0x3f000u) | ((d >> 6) & 0xfc0000u);
          }
          const uint32_t P0 = c24[0] | (c24[1] << 24), P1 = c24[1] >> 8;
          const uint32_t w32 = (g & 1) ? ((P0 >> 16) | (P1 << 16)) : P0;
          const uint32_t w16 = (g & 1) ? (P0 & 0xffffu) : P1;
          if (valid) {
            *reinterpret_cast<uint32_t*>(smem + baddr(term, bb, p, o32)) = w32;
            *reinterpret_cast<uint16_t*>(smem + baddr(term, bb, p, o16)) = (uint16_t)w16;
            if (g == 0) *reinterpret_cast<uint8_t*>(smem + baddr(term, bb, p, osc)) = (uint8_t)(127 + s);
          }
        }
      }
    }
    publish_max(ymax, xo);
  };

  // ---------------- stem: conv3x3 8->256 in f16x3 (k_net_y's), K = 3 k-blocks -------------
  // (stem_input zeroes both parts' zero lines, which covers [Xl8 | Xh8] of off-board taps)
  char* simg = smem + ZIMGB;
  stem_input<NT, true>(smem, simg, pos, b0, nb, W, tid);
  __syncthreads();
  {
    const uint4* Ws = W.stemz + (size_t)(CT * wc) * 3 * 128 + lane;
    for (int kb = 0; kb < 3; ++kb) {
      f16x8 SA[2 * CT], SB[2 * TW];
#pragma unroll
      for (int c = 0; c < CT; ++c) {
        SA[2 * c] = __builtin_bit_cast(f16x8, Ws[c * 3 * 128 + kb * 128]);
        SA[2 * c + 1] = __builtin_bit_cast(f16x8, Ws[c * 3 * 128 + kb * 128 + 64]);
      }
      const int tap = 4 * kb + g;
      const int r0 = tap < 9 ? src_row(n, ph0, pw0, tap) : ZROW;
      const int r1 = tap < 9 ? src_row(p1, ph1, pw1, tap) : ZROW;
#pragma unroll
      for (int part = 0; part < 2; ++part)
#pragma unroll
        for (int j = 0; j < BPW; ++j) {
          const int bb = wb0 + j;
          SB[part * TW + 2 * j] = *reinterpret_cast<const f16x8*>(simg + ((part * XB + bb) * IROWS + r0) * 16);
          SB[part * TW + 2 * j + 1] = *reinterpret_cast<const f16x8*>(simg + ((part * XB + bb) * IROWS + r1) * 16);
        }
#pragma unroll
      for (int ps = 0; ps < 3; ++ps) {
        const int wp = ps == 2 ? 1 : 0, xp = ps == 1 ? 1 : 0;
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int t = 0; t < TW; ++t)
            acc[ct * TW + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(SA[2 * ct + wp], SB[xp * TW + t], acc[ct * TW + t], 0, 0, 0);
      }
    }
  }
  {
    float bnd[XB];
#pragma unroll
    for (int bb = 0; bb < XB; ++bb)
      bnd[bb] = __builtin_fmaf(W.yrange[2 * CONV_LAYERS], mxb[bb], W.yrange[2 * CONV_LAYERS + 1]) * 1.0009765625f;
    if constexpr (F6)
      epilogue6(W.stemx_inv[0], W.stem_b, std::false_type{}, 0.f, bnd);
    else
      epilogue(W.stemx_inv[0], W.stem_b, std::false_type{}, 0.f, bnd);
  }
  stamp(st_stem);

  // ---------------- residual trunk ----------------------------------------------------------
  if constexpr (PRIO) {
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  constexpr int PD = RA0 - 1, RA = PD + 1, GD = 1, RG = GD + 1;
  constexpr int U = (RA == 2 && RG == 2) ? 4 : 12;
  static_assert(KBZ % U == 0 && U % RA == 0 && (U / 2) % RG == 0 && RG > GD, "rings");
  f16x8 A16[RA][CT], B16[TW];
  i32x8 A8[RG][CT], B8[BPW];
  f16x8 AL16[RA][CT], BL16[TW];   // W3: the Wl fragments and the step's Xl fragments
  static_assert(!W3 || TAPA, "W3 runs the tap-major loop");
  const int n_ = n, p1_ = p1, ph0_ = ph0, pw0_ = pw0, ph1_ = ph1, pw1_ = pw1, g_ = g;
  const uint4* Wh = W.convz + (size_t)(CT * wc) * KBZ * 128 + lane;   // hi parts
  const uint4* W8 = W.conv8 + (size_t)(CT * wc) * GZ * 128 + lane;
  const uint4* W6 = W.conv6 + (size_t)(CT * wc) * GZ * 112;
  const int32_t* sc8 = W.conv8_sc;
  const int bofs = wb0 * ZBOARD;   // the wave's first board in each image part
  // WBUF: buffer descriptors of the f16 and e4m3 weight sets, the wave's lane offsets and the
  // layer's byte offsets (both sets < 2 GB)
  const __amdgpu_buffer_rsrc_t rs_h = __builtin_amdgcn_make_buffer_rsrc((void*)W.convz, (short)0, 0x7ffffff0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_8 = __builtin_amdgcn_make_buffer_rsrc((void*)W.conv8, (short)0, 0x7ffffff0, 0x00020000);
  const int vo_h = (CT * wc * KBZ * 128 + lane) * 16, vo_8 = (CT * wc * GZ * 128 + lane) * 16;
  int lo_h = 0, lo_8 = 0;

  // Wh fragments of step (k-block) KB, the wave's channel tiles
#define Z_LOAD_A16(S, KB)                                                             \
  {                                                                                   \
    const int kk_ = DIAG_L1 ? 0 : (KB) < KBZ ? (KB) : KBZ - 1;                        \
    _Pragma("unroll") for (int c_ = 0; c_ < CT; ++c_) {                               \
      if constexpr (WBUF)                                                             \
        S[c_] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(       \
                    rs_h, vo_h, lo_h + (c_ * KBZ + kk_) * 2048, 0));                  \
      else                                                                            \
        S[c_] = __builtin_bit_cast(f16x8, Wh[((size_t)c_ * KBZ + kk_) * 128]);        \
    }                                                                                 \
  }
  // W3: Wl (lo part) fragments of step KB: the hi part's + 1 KB
#define Z_LOAD_AL16(S, KB)                                                            \
  {                                                                                   \
    const int kk_ = DIAG_L1 ? 0 : (KB) < KBZ ? (KB) : KBZ - 1;                        \
    _Pragma("unroll") for (int c_ = 0; c_ < CT; ++c_) {                               \
      if constexpr (WBUF)                                                             \
        S[c_] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(       \
                    rs_h, vo_h, lo_h + (c_ * KBZ + kk_) * 2048 + 1024, 0));           \
      else                                                                            \
        S[c_] = __builtin_bit_cast(f16x8, Wh[((size_t)c_ * KBZ + kk_) * 128 + 64]);   \
    }                                                                                 \
  }
  // e4m3 weight fragments of group GR (tap, chunk, term), channel tiles [C0, C0 + CT/2); with
  // F6 the e2m3 vector in dwords 0..5 and the lane's e8m0 scale in dword 6
#define Z_LOAD_A8(S, GR, C0)                                                          \
  {                                                                                   \
    const int gg_ = DIAG_L1 ? 0 : (GR) < GZ ? (GR) : GZ - 1;                          \
    _Pragma("unroll") for (int c_ = (C0); c_ < (C0) + CT / 2; ++c_) {                 \
      if constexpr (F6) {                                                             \
        const uint4* p_ = W6 + ((size_t)c_ * GZ + gg_) * 112;                         \
        const uint4 d0_ = p_[lane];                                                   \
        const uint2 d1_ = reinterpret_cast<const uint2*>(p_ + 64)[lane];              \
        const uint32_t sc_ = reinterpret_cast<const uint32_t*>(p_ + 96)[lane];        \
        S[c_] = (i32x8){(int)d0_.x, (int)d0_.y, (int)d0_.z, (int)d0_.w,               \
                        (int)d1_.x, (int)d1_.y, (int)sc_, 0};                         \
      } else if constexpr (WBUF) {                                                    \
        const int so_ = lo_8 + (c_ * GZ + gg_) * 2048;                                \
        const auto a_ = __builtin_amdgcn_raw_buffer_load_b128(rs_8, vo_8, so_, 0);    \
        const auto b_ = __builtin_amdgcn_raw_buffer_load_b128(rs_8, vo_8 + 1024, so_, 0); \
        S[c_] = (i32x8){(int)a_[0], (int)a_[1], (int)a_[2], (int)a_[3],               \
                        (int)b_[0], (int)b_[1], (int)b_[2], (int)b_[3]};              \
      } else {                                                                        \
        const uint4* p_ = W8 + ((size_t)c_ * GZ + gg_) * 128;                         \
        S[c_] = cat8(p_[0], p_[64]);                                                  \
      }                                                                               \
    }                                                                                 \
  }
  // Xh (f16) fragments of step KB for both square tiles of the wave's boards: S16[2 j + tile]
#define Z_LOAD_B16(S16, KB)                                                           \
  {                                                                                   \
    const int kk_ = (KB) < KBZ ? (KB) : KBZ - 1;                                      \
    const int tap_ = kk_ >> 3, ch_ = 4 * (kk_ & 7) + g;                               \
    const int o0_ = zsrc(n, ph0, pw0, tap_, ch_), o1_ = zsrc(p1, ph1, pw1, tap_, ch_); \
    _Pragma("unroll") for (int j_ = 0; j_ < BPW; ++j_) {                              \
      const char* base_ = smem + bofs + j_ * ZBOARD;                                  \
      S16[2 * j_] = *reinterpret_cast<const f16x8*>(base_ + o0_);                     \
      S16[2 * j_ + 1] = *reinterpret_cast<const f16x8*>(base_ + o1_);                 \
    }                                                                                 \
  }
  // e4m3 fragments of step KB's group on square tile KB & 1 (Xl8 for term 0, Xh8 for term 1):
  // lane (g, n) takes the 32 channels [128 c + 32 g, +32) of its source square
#define Z_LOAD_B8(S8, KB)                                                             \
  {                                                                                   \
    const int kk_ = (KB) < KBZ ? (KB) : KBZ - 1;                                      \
    const int tap_ = kk_ >> 3, term_ = (kk_ >> 1) & 1, cc_ = (kk_ >> 2) & 1;          \
    const int q0_ = 16 * term_ + 8 * cc_ + 2 * g;                                     \
    /* part-1 row base once, so that the boards' offsets (< 64 KB) fit the ds_read immediate; */ \
    /* chunk q0 + 1 is 256 B after chunk q0 (zero-line cells: the same cell) */    \
    const int z0_ = (kk_ & 1) ? zsrc(p1, ph1, pw1, tap_, q0_) : zsrc(n, ph0, pw0, tap_, q0_); \
    const char* p0_ = smem + ZPART + bofs + z0_;                                      \
    const char* p1_ = p0_ + (z0_ < ZROWS_B ? 256 : 0);                                \
    _Pragma("unroll") for (int j_ = 0; j_ < BPW; ++j_)                                \
      S8[j_] = cat8(*reinterpret_cast<const uint4*>(p0_ + j_ * ZBOARD),               \
                    *reinterpret_cast<const uint4*>(p1_ + j_ * ZBOARD));              \
  }

  for (int L = 0; L < CONV_LAYERS; ++L) {
    // the lane's square coordinates, opaque to the compiler per layer: the LDS offsets of the
    // 72 steps are recomputed in the loop (a few VALU each) instead of being hoisted out of the
    // layer loop into ~150 VGPRs
    int n = n_, p1 = p1_, ph0 = ph0_, pw0 = pw0_, ph1 = ph1_, pw1 = pw1_, g = g_;
    asm volatile("" : "+v"(n), "+v"(p1), "+v"(ph0), "+v"(pw0), "+v"(ph1), "+v"(pw1), "+v"(g));
    const int sa_h = sc8[2 * L], sa_l = sc8[2 * L + 1];
    int sb_l[BPW], sb_h[BPW];   // the input image's e4m3 units, per board of the wave
#pragma unroll
    for (int j = 0; j < BPW; ++j) {
      const int shj = pick4(sh, wb0 + j);
      sb_l[j] = 127 - (shj + 11), sb_h[j] = 127 - shj;
    }
#pragma unroll
    for (int p = 0; p < PD; ++p) {
      Z_LOAD_A16(A16[p], p);
      if constexpr (W3) Z_LOAD_AL16(AL16[p], p);
    }
    if constexpr (!W3) {
#pragma unroll
      for (int p = 0; p < GD; ++p) {
        Z_LOAD_A8(A8[p], p, 0)
        Z_LOAD_A8(A8[p], p, CT / 2)
      }
    }
    if constexpr (TAPA) {
      static_assert(8 % RA == 0 && RG == 2 && !DIAG_NOLDS, "tap-major loop: 8 steps per iteration");
      // per tap and square tile: the source square's chunk-0 row offset, its zero cell and the
      // on-board mask (as zsrc); a fragment's offset = mask ? row + chunk offset : zero cell
      const int g256 = g << 8, g512 = g << 9;
      auto zsel = [](int m, int on, int off) { return (on & m) | (off & ~m); };
      auto tap_addr = [&](int t, int* row, int* off, int* m) {
        const int dh = t / 3 - 1, dw = t - 3 * (t / 3) - 1;
        const int pp[2] = {n, p1}, hh[2] = {ph0, ph1}, ww[2] = {pw0, pw1};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int r = hh[i] + dh, c = ww[i] + dw, s = pp[i] + 5 * dh + dw;
          const bool valid = (pp[i] < 30) & ((unsigned)r < 6u) & ((unsigned)c < 5u);
          row[i] = 8192 * (s >> 4) + 16 * (s & 15);
          off[i] = ZROWS_B + 16 * (s & 15);
          m[i] = valid ? -1 : 0;
        }
      };
      int crow[2], coff[2], cm[2];
      tap_addr(0, crow, coff, cm);
      // Xh fragments of chunk-step CS (0..7) of a tap: channels 4 CS + g of 32-channel block
#define Z_LOAD_B16T(S16, ROW, OFF, M, CS)                                                  \
  {                                                                                       \
    const int o0_ = zsel(M[0], ROW[0] + g256 + 1024 * (CS), OFF[0]);                      \
    const int o1_ = zsel(M[1], ROW[1] + g256 + 1024 * (CS), OFF[1]);                      \
    _Pragma("unroll") for (int j_ = 0; j_ < BPW; ++j_) {                                  \
      const char* base_ = smem + bofs + j_ * ZBOARD;                                      \
      S16[2 * j_] = *reinterpret_cast<const f16x8*>(base_ + o0_);                         \
      S16[2 * j_ + 1] = *reinterpret_cast<const f16x8*>(base_ + o1_);                     \
    }                                                                                     \
  }
      Z_LOAD_B16T(B16, crow, coff, cm, 0);
      // W3: the Xl fragments (part 1), same offsets as Z_LOAD_B16T
#define Z_LOAD_BL16T(S16, ROW, OFF, M, CS)                                                 \
  {                                                                                       \
    const int o0_ = zsel(M[0], ROW[0] + g256 + 1024 * (CS), OFF[0]);                      \
    const int o1_ = zsel(M[1], ROW[1] + g256 + 1024 * (CS), OFF[1]);                      \
    _Pragma("unroll") for (int j_ = 0; j_ < BPW; ++j_) {                                  \
      const char* base_ = smem + ZPART + bofs + j_ * ZBOARD;                              \
      S16[2 * j_] = *reinterpret_cast<const f16x8*>(base_ + o0_);                         \
      S16[2 * j_ + 1] = *reinterpret_cast<const f16x8*>(base_ + o1_);                     \
    }                                                                                     \
  }
#pragma unroll 1
      for (int t = 0; t < 9; ++t) {
        int nrow[2], noff[2], nm[2];
        tap_addr(t < 8 ? t + 1 : 8, nrow, noff, nm);
        if constexpr (W3) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const int s = 8 * t + u;
            // Wh*Xh and Wl*Xh on the step's Xh fragments; meanwhile its Xl fragments and the
            // weight fragments PD steps ahead
            __builtin_amdgcn_sched_barrier(0);
            Z_LOAD_BL16T(BL16, crow, coff, cm, u);
            Z_LOAD_A16(A16[(u + PD) % RA], s + PD);
            Z_LOAD_AL16(AL16[(u + PD) % RA], s + PD);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
              for (int tt = 0; tt < TW; ++tt)
                acc[ct * TW + tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A16[u % RA][ct], B16[tt], acc[ct * TW + tt], 0, 0, 0);
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
              for (int tt = 0; tt < TW; ++tt)
                acc[ct * TW + tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(AL16[u % RA][ct], B16[tt], acc[ct * TW + tt], 0, 0, 0);
            // Wh*Xl; meanwhile the next step's Xh fragments
            __builtin_amdgcn_sched_barrier(0);
            if (u < 7)
              Z_LOAD_B16T(B16, crow, coff, cm, u + 1)
            else
              Z_LOAD_B16T(B16, nrow, noff, nm, 0)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
              for (int tt = 0; tt < TW; ++tt)
                acc[ct * TW + tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A16[u % RA][ct], BL16[tt], acc[ct * TW + tt], 0, 0, 0);
          }
#pragma unroll
          for (int i = 0; i < 2; ++i) crow[i] = nrow[i], coff[i] = noff[i], cm[i] = nm[i];
          continue;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int s = 8 * t + u;
          __builtin_amdgcn_sched_barrier(0);
          {
            // e4m3 fragments of step s (group s/2 = term (u>>1)&1, chunk (u>>2)&1, tile u&1):
            // channels [128 cc + 32 g, +32) of part 1's Xl8 (term 0) or Xh8 (term 1) block
            const int tl = u & 1;
            const int z0 = zsel(cm[tl], crow[tl] + g512 + 4096 * ((u >> 1) & 1) + 2048 * ((u >> 2) & 1), coff[tl]);
            const char* p0 = smem + ZPART + bofs + z0;
#pragma unroll
            for (int j = 0; j < BPW; ++j)
              B8[j] = cat8(*reinterpret_cast<const uint4*>(p0 + j * ZBOARD),
                           *reinterpret_cast<const uint4*>(p0 + j * ZBOARD + 256));
          }
          Z_LOAD_A16(A16[(u + PD) % RA], s + PD);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int tt = 0; tt < TW; ++tt)
              acc[ct * TW + tt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A16[u % RA][ct], B16[tt], acc[ct * TW + tt], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if (u < 7)
            Z_LOAD_B16T(B16, crow, coff, cm, u + 1)
          else
            Z_LOAD_B16T(B16, nrow, noff, nm, 0)
          Z_LOAD_A8(A8[((u >> 1) + GD) % RG], (s >> 1) + GD, (CT / 2) * (u & 1));
          const int pt = u & 1;
          const bool term = (u >> 1) & 1;
          const int sa = term ? sa_l : sa_h;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int j = 0; j < BPW; ++j) {
              if constexpr (DIAG_NOB)
                ;
              else if constexpr (F6)
                acc[ct * TW + 2 * j + pt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                    A8[(u >> 1) % RG][ct], B8[j], acc[ct * TW + 2 * j + pt], 2, 2, 0, A8[(u >> 1) % RG][ct][6], 0,
                    B8[j][6]);
              else
                acc[ct * TW + 2 * j + pt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                    A8[(u >> 1) % RG][ct], B8[j], acc[ct * TW + 2 * j + pt], 0, 0, 0, sa, 0,
                    term ? sb_h[j] : sb_l[j]);
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) crow[i] = nrow[i], coff[i] = noff[i], cm[i] = nm[i];
      }
#undef Z_LOAD_B16T
#undef Z_LOAD_BL16T
    } else {
    Z_LOAD_B16(B16, 0);
    if constexpr (DIAG_NOLDS) Z_LOAD_B8(B8, 0);
    {
#pragma unroll 1
      for (int s0 = 0; s0 < KBZ; s0 += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int s = s0 + u;
          // phase A: Wh x Xh of k-block s on every column tile; meanwhile this step's e4m3
          // activation fragments and the Wh fragments PD steps ahead.  Phase B: group s/2 on
          // square tile s&1; meanwhile the next step's Xh fragments and half of the e4m3 weight
          // group GD groups ahead
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (!DIAG_NOLDS) Z_LOAD_B8(B8, s);
          Z_LOAD_A16(A16[(u + PD) % RA], s + PD);
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int t = 0; t < TW; ++t)
              acc[ct * TW + t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A16[u % RA][ct], B16[t], acc[ct * TW + t], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (!DIAG_NOLDS) Z_LOAD_B16(B16, s + 1);
          Z_LOAD_A8(A8[((u >> 1) + GD) % RG], (s >> 1) + GD, (CT / 2) * (u & 1));
          const int pt = u & 1;
          const bool term = (u >> 1) & 1;
          const int sa = term ? sa_l : sa_h;
#pragma unroll
          for (int ct = 0; ct < CT; ++ct)
#pragma unroll
            for (int j = 0; j < BPW; ++j) {
              if constexpr (DIAG_NOB)
                ;
              else if constexpr (F6)
                acc[ct * TW + 2 * j + pt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                    A8[(u >> 1) % RG][ct], B8[j], acc[ct * TW + 2 * j + pt], 2, 2, 0, A8[(u >> 1) % RG][ct][6], 0,
                    B8[j][6]);
              else
                acc[ct * TW + 2 * j + pt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
                    A8[(u >> 1) % RG][ct], B8[j], acc[ct * TW + 2 * j + pt], 0, 0, 0, sa, 0,
                    term ? sb_h[j] : sb_l[j]);
            }
        }
      }
    }
    }
    if constexpr (!DIAG_L2 && !DIAG_L1) {
      Wh += CONVX_U4_PER_LAYER;
      W8 += CONV8_U4_PER_LAYER;
      lo_h += (int)(CONVX_U4_PER_LAYER * 16);
      lo_8 += (int)(CONV8_U4_PER_LAYER * 16);
      W6 += CONV6_U4_PER_LAYER;
    }
    __syncthreads();
    stamp(st_k);   // (k_net_z: the K-loop share includes the wait for the workgroup's slowest wave)
    float bnd[XB];
    if ((L & 1) == 0) {
#pragma unroll
      for (int bb = 0; bb < XB; ++bb) {
        bnd[bb] = __builtin_fmaf(W.yrange[2 * L], mxb[bb], W.yrange[2 * L + 1]) * 1.0009765625f;
        mxblk[bb] = mxb[bb];
      }
      if constexpr (F6)
        epilogue6(W.convx_inv[L], W.conv_b + L * 256, std::true_type{}, 1.0f / W.convx_inv[L + 1], bnd);
      else
        epilogue(W.convx_inv[L], W.conv_b + L * 256, std::true_type{}, 1.0f / W.convx_inv[L + 1], bnd);
    } else {
#pragma unroll
      for (int bb = 0; bb < XB; ++bb)
        bnd[bb] = (__builtin_fmaf(W.yrange[2 * L], mxb[bb], W.yrange[2 * L + 1]) + mxblk[bb]) * 1.0009765625f;
      // (F6: the last conv stores e4m3 bytes, the image heads_reduce reads)
      if (F6 && L < CONV_LAYERS - 1)
        epilogue6(W.convx_inv[L], W.conv_b + L * 256, std::false_type{}, 0.f, bnd);
      else
        epilogue(W.convx_inv[L], W.conv_b + L * 256, std::false_type{}, 0.f, bnd);
    }
    stamp(st_epi);
  }
#undef Z_LOAD_A16
#undef Z_LOAD_AL16
#undef Z_LOAD_A8
#undef Z_LOAD_B16
#undef Z_LOAD_B8
  if (overflow && !DIAG_L2 && !DIAG_L1 && !DIAG_NOB && !DIAG_NOLDS) atomicOr(D.pr.err, ERR_F16);
  if (zrange && tid == 0 && !DIAG_L2 && !DIAG_L1 && !DIAG_NOB && !DIAG_NOLDS) atomicOr(D.pr.err, ERR_ZRANGE);

  heads_reduce<NT, !W3, true>(smem, pos, b0, nb, W, tid, __builtin_ldexpf(1.f, xs),
                         make_float4(__builtin_ldexpf(1.f, -(sh[0] + 11)), __builtin_ldexpf(1.f, -(sh[1] + 11)),
                                     __builtin_ldexpf(1.f, -(sh[2] + 11)), __builtin_ldexpf(1.f, -(sh[3] + 11))));
  stamp(st_heads);
  if constexpr (STAMP) {
    if (tid == 0) {
      stamps[blockIdx.x * 6 + 0] = st_stem;
      stamps[blockIdx.x * 6 + 1] = st_k;
      stamps[blockIdx.x * 6 + 2] = st_epi;
      stamps[blockIdx.x * 6 + 3] = st_heads;
      stamps[blockIdx.x * 6 + 4] = __builtin_amdgcn_s_memtime() - t_start;
      stamps[blockIdx.x * 6 + 5] = __builtin_amdgcn_s_memrealtime() - r_start;
    }
  }
  heads_out<true>(D, smem, b0, nb, W, mode, logits_out, values_out, wave, lane);
}

template <bool S>
static void launch_z(int var, dim3 grid, hipStream_t s, const Dev& d, const NetWeights& w, const Pos* pos,
                     const int32_t* count, int max_b, int mode, float* logits, float* values,
                     unsigned long long* stamps) {
#define Z_LAUNCH(V, T)                                                                                       \
  hipLaunchKernelGGL((k_net_z<S, V>), grid, dim3(T), 0, s, d, w, pos, count, max_b, mode, logits, values, stamps, 0)
  // product builds (mtaz_set_net_variant accepts these): 0, the unfused epilogue, e2m3 cross terms,
  // the round-2 K loop (per-step addresses, global-address weights)
  if (var == 2097152) Z_LAUNCH(2097152, 512);
  else if (var == 8192) Z_LAUNCH(8192, 512);
  else if (var == 268435456) Z_LAUNCH(268435456, 512);
  else if (var == 33554432) Z_LAUNCH(33554432, 512);
  else if (var == 8388608 + 16777216 + 33554432) Z_LAUNCH(8388608 + 16777216 + 33554432, 512);
  else if (var == 8388608 + 16777216) Z_LAUNCH(8388608 + 16777216, 512);
#ifdef MTAZ_NET_DIAG
  else if (var == 8388608) Z_LAUNCH(8388608, 512);
  else if (var == 16777216) Z_LAUNCH(16777216, 512);
  else if (var == 4194304) Z_LAUNCH(4194304, 512);
  else if (var == 4194304 + 8192) Z_LAUNCH(4194304 + 8192, 512);
  // A/B and timing-only builds: the diagnostic library only (tools/bench_net.py --diag)
  else if (var == 1048576) Z_LAUNCH(1048576, 512);
  else if (var == 1048576 + 2048 + 8192) Z_LAUNCH(1048576 + 2048 + 8192, 256);
  else if (var == 16384) Z_LAUNCH(16384, 512);
  else if (var == 32768) Z_LAUNCH(32768, 512);
  else if (var == 65536) Z_LAUNCH(65536, 512);
  else if (var == 131072) Z_LAUNCH(131072, 512);
  else if (var == 65536 + 131072) Z_LAUNCH(65536 + 131072, 512);
  else if (var == 8192 + 131072) Z_LAUNCH(8192 + 131072, 512);
  else if (var == 2048 + 8192) Z_LAUNCH(2048 + 8192, 256);
  else if (var == 2048) Z_LAUNCH(2048, 256);
  else if (var == 4194304 + 16384) Z_LAUNCH(4194304 + 16384, 512);
  else if (var == 4194304 + 65536) Z_LAUNCH(4194304 + 65536, 512);
  else if (var == 4194304 + 131072) Z_LAUNCH(4194304 + 131072, 512);
#endif
  else Z_LAUNCH(0, 512);
#undef Z_LAUNCH
}

// compute units of the current device (the size of a launch's round)
static int device_cus() {
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

void launch_net_z(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                  float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                  int variant) {
  if (max_b <= 0) return;
  if (ev_begin) (void)hipEventRecord(ev_begin, s);
  const int ncu = device_cus();
  // the product (and its f16x3 form W3): full rounds, then the tail launches (k_net_z above)
  auto tailed = [&](auto var_t) {
    constexpr int V = decltype(var_t)::value;
    const dim3 blk(64 * ZCfg<V>::NW);
    hipLaunchKernelGGL((k_net_z<false, V, XB>), dim3((max_b + XB - 1) / XB), blk, 0, s, d, w, pos, count, max_b, mode,
                       logits_out, values_out, nullptr, ncu);
    hipLaunchKernelGGL((k_net_z<false, V, 1>), dim3(ncu), blk, 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, nullptr, ncu);
    hipLaunchKernelGGL((k_net_z<false, V, 2>), dim3(ncu), blk, 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, nullptr, ncu);
    hipLaunchKernelGGL((k_net_z<false, V, 3>), dim3(ncu), blk, 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, nullptr, ncu);
  };
  if (variant == 0 && ncu > 0) {
    tailed(std::integral_constant<int, 0>{});
  } else if (variant == 268435456 && ncu > 0) {
    tailed(std::integral_constant<int, 268435456>{});
  } else {   // variant 1: the product kernel with 4 boards per workgroup throughout (the round-2 assignment)
    launch_z<false>(variant == 1 ? 0 : variant, dim3((max_b + XB - 1) / XB), s, d, w, pos, count, max_b, mode,
                    logits_out, values_out, nullptr);
  }
  if (ev_end) (void)hipEventRecord(ev_end, s);
}

void launch_net_z_stamped(const Dev& d, const NetWeights& w, const Pos* pos, int n, float* logits_out,
                          float* values_out, unsigned long long* stamps, hipStream_t s, int variant) {
  if (n <= 0) return;
  launch_z<true>(variant, dim3((n + XB - 1) / XB), s, d, w, pos, nullptr, n, (int)NET_FULL_LOGITS, logits_out,
                 values_out, stamps);
}

}  // namespace mtaz
