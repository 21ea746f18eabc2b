// k_net_y3: ROUND 3's k_net_y, kept as f16x3 variant 3 (a bit-identity reference for the round-4
// k_net_y on nets whose activations stay below 2^14, and its A/B baseline).  Its stored-units
// exponent is one per WORKGROUP (below), so beyond 2^14 a board's results depend on its workgroup's
// other boards; round 4's k_net_y (mtaz_net16.hip) keeps one per board.
//
// k_net_y: the fused fp16x3 policy/value network (exp/policy.py:71-80 + the leaf priors of
// exp/agent.py:67-69) on v_mfma_f32_16x16x32_f16.  Under the chip's power limit the 16x16x32
// shape holds a higher clock than 32x32x16 at equal cycles per FLOP (MI355X_MICROARCH.md, DVFS
// item 7; round 1 measured the 32x32x16 form of this kernel 11% slower), and this kernel is
// MFMA-bound.
//
// Workgroup = 4 boards, 256 threads.  Wave w owns output channels [64w, 64w+64) as 4 channel
// tiles of 16, times 4 boards x 2 square tiles of 16 (squares 0..15, 16..31; 30, 31 pad):
// 32 accumulator tiles of 16x16 (128 AGPRs).  A conv's K = 2304 runs as 72 k-blocks of 32
// contiguous k = tap*256 + ci, so a k-block is one tap and 32 input channels: lane l holds
// A = W[co = 16ct + (l&15)][k = 32kb + 8(l>>4) + j] and B = X[k][square 16pt + (l&15)],
// i.e. the 16-B chunk 4(kb&7) + (l>>4) of the source square's image row.
#include <type_traits>

#include "net_common.h"

namespace mtaz {

using namespace netc;
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int KBY = 72;   // k-blocks of 32 per conv

// Mixed-precision FMAs (v_fma_mix*: each source f16 or f32).  The compiler does not form them
// while f32 denormals are enabled, so they are written out.  Used only where the fused
// result is exact in f32, hence bit-identical to the unfused expression:
//  lo_pair: {f16(y0 - f32(h0)), f16(y1 - f32(h1))} packed, h = hi_pk (y - hi is exact in f32)
//  mix_lo / mix_hi: fma(f32(f16 half of pk), b, c)
__device__ __forceinline__ uint32_t lo_pair(uint32_t hi_pk, float y0, float y1) {
  uint32_t r;
  asm volatile(
      "v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(r)
      : "v"(hi_pk), "v"(y0), "v"(y1));
  return r;
}
__device__ __forceinline__ float mix_lo(uint32_t pk, float b, float c) {
  float r;
  asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(pk), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float mix_hi(uint32_t pk, float b, float c) {
  float r;
  asm volatile("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(pk), "v"(b), "v"(c));
  return r;
}

// a * b + c on v_mad_i32_i24 (b uniform; operands within 24 bits signed)
__device__ __forceinline__ int mad_i24(int a, int b, int c) {
  int r;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}

// fp32 add as one v_add_f32 (the compiler would pair adds into v_pk_add_f32, which costs ~13
// cycles beside MFMAs instead of hiding in their issue gaps: MI355X_MICROARCH.md, cycle constants)
__device__ __forceinline__ float add_f32(float a, float b) {
  float r;
  asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ void add4(f32x4v& m, const f32x4v& a) {
  m[0] = add_f32(m[0], a[0]);
  m[1] = add_f32(m[1], a[1]);
  m[2] = add_f32(m[2], a[2]);
  m[3] = add_f32(m[3], a[3]);
}

// one split pass over the wave's 32 tiles: W part WP (0 hi / 1 lo) x X part XP.
// SA[2*ct + part], SB[part*8 + t] with t = 2*board + square tile.
#define YMMA(SA, SB, WP, XP)                                                                          \
  {                                                                                                   \
    _Pragma("unroll") for (int ct_ = 0; ct_ < CT; ++ct_)                                              \
    _Pragma("unroll") for (int t_ = 0; t_ < 2 * NVB; ++t_)                                            \
      acc[ct_ * 8 + t_] = __builtin_amdgcn_mfma_f32_16x16x32_f16(SA[2 * ct_ + (WP)], SB[(XP) * 8 + t_], \
                                                                 acc[ct_ * 8 + t_], 0, 0, 0);         \
  }
// Wh*Xh + Wh*Xl + Wl*Xh: 96 MFMAs, 31 independent ones between two updates of one accumulator
#define YMMA3(SA, SB) YMMA(SA, SB, 0, 0) YMMA(SA, SB, 0, 1) YMMA(SA, SB, 1, 0)

// VAR: 0 = product; 1024 = the epilogue in unfused form (bit-identity reference for the
// product's v_fma_mix epilogue, test_gpu_net.py); 114688 = the K loop without the offset table,
// the buffer loads and the 2-slot weight ring (bitwise equal, test_y_loop_forms_bit_identical);
// 16777216 = the row-major swizzled LDS image instead of the chunk-major one (ZL below; bitwise
// equal, test_y_loop_forms_bit_identical);
// 4096 (diagnostic library) = one accumulation chain per layer (round 2's k_net_y, see CH below).  Round 1's schedule A/B variants (whole-k-block
// steps, sched_group_barrier interleaves, 8 waves of 32 channels) measured within 1% of the
// pinned half-steps and were retired.
// NVB / ncu: the tail-balanced board assignment of k_net_z (mtaz_net8.hip): with ncu > 0 the
// NVB = 4 launch computes the full rounds of 4 boards per workgroup and the NVB = 1..3 launches
// the remaining boards, at most NVB per workgroup, computing only those (boards NVB..3 of the
// image are never computed).  The workgroup's stored-units exponent xs follows the bound of its
// own boards, so the assignment is exact for any net whose activations stay below 2^14 (xs = 0).
// LDS bytes of a VAR build: the image, the aux region, the fragment offset table
constexpr int net_y3_smem(int var) {
  return ((var & (1 << 24)) ? IMGB : ZIMGB) + AUXB + ((var & 32768) ? 0 : 9 * 2 * 64 * 4);
}

// the network on workgroup `bid`'s boards (k_net_y, k_net_y3_tail below), in the kernel's LDS `smem`
template <bool STAMP, int VAR, int NVB = XB>
__device__ __forceinline__ void net_y3_body(char* smem, const int bid, const Dev& D, const NetWeights& W,
                                           const Pos* __restrict__ pos, const int32_t* __restrict__ count,
                                           int max_b, int mode, float* __restrict__ logits_out,
                                           float* __restrict__ values_out, unsigned long long* __restrict__ stamps,
                                           int ncu) {
  static_assert(NVB >= 1 && NVB <= XB, "boards per workgroup");
  // OT (product; VAR 32768 = off): the K loop's fragment offsets come from a per-lane LDS table of
  // the source rows [tap 9][square tile 2][lane 64] (one ds_read_b32 per half-step, issued a
  // half-step ahead) instead of recomputing src_row (~20 VALU / SALU per half-step)
  constexpr bool OT = (VAR & 32768) == 0;
  constexpr int OTB = OT ? 9 * 2 * 64 * 4 : 0;
  // ZL (product; VAR 1 << 24 = round 2's row-major swizzled image): k_net_z's chunk-major image
  // (net_common.h zrow / zoff): the bank group of a 16-B cell is its row's, so a 16-lane read group
  // (16 consecutive output squares, any chunk per lane) is conflict-free, off-board taps included
  // (a per-lane cell of the board's zero line on the bank the on-board source would have had)
  constexpr bool ZL = (VAR & (1 << 24)) == 0;
  constexpr int IMG = ZL ? ZIMGB : IMGB, PART = ZL ? ZPART : PARTB, BSTR = ZL ? ZBOARD : IROWS * RB;
  static_assert(IMG + AUXB + OTB == net_y3_smem(VAR), "LDS layout");
  int b0, nb;
  {
    const int n = count ? *count : max_b;
    const int r = ncu > 0 ? n % (XB * ncu) : 0, per = ncu > 0 ? (r + ncu - 1) / ncu : XB;
    if constexpr (NVB == XB) {   // the full rounds (and a tail of 4 boards per CU)
      b0 = bid * XB;
      nb = per < XB ? n - r : n;
    } else {                     // the tail, when it has NVB boards per CU
      if (per != NVB) return;
      b0 = n - r + bid * NVB;
      nb = b0 + NVB < n ? b0 + NVB : n;
    }
  }
  if (b0 >= nb) return;
  constexpr int NW = 4, NT = 64 * NW, CT = 16 / NW;   // waves, threads, channel tiles per wave
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, n = lane & 15, g = lane >> 4;
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

  // the lane's output squares: n (tile 0) and p1 = 16 + n (tile 1; 30, 31 are padding)
  const int p1 = 16 + n;
  const int ph0 = n / 5, pw0 = n % 5, ph1 = p1 / 5, pw1 = p1 % 5;
  // Chunked accumulation (CH; VAR 4096 = round 2's single chain, for A/B only).  The MFMAs of
  // every U = 12 k-blocks (a chunk) accumulate from zero into acc, and each tile's chunk sum is
  // added into the master sums mst (fp32, round to nearest).  Each output then takes 6 roundings at
  // its full magnitude per layer instead of one per MFMA (216: a 16x16x32 f16 MFMA rounds C + its
  // 32 products once), and the residual (seeded into mst) no longer sits under every MFMA's
  // rounding.  On the stress net (trunk activations ~3300) this takes the priors' error from
  // 1.5e-5 to 2.7e-6 of an fp64 forward (tools/stress_error.py, tools/dump_net.py) for +3% time.
  // The adds are staggered so that they issue between MFMAs on other tiles: the square-tile-0
  // tiles' during the chunk's last half-step (square tile 1), the square-tile-1 tiles' during the
  // next chunk's first half-step (square tile 0), whose MFMAs start from C = 0.  After a layer's
  // K loop the square-tile-1 tiles are still pending: the epilogue reads mst (+ acc for those).
  // (Measured and dropped: chunks of 6 k-blocks, 1.2e-6 for +7.4%; the residual alone kept out of
  // the chain, 9.7e-6 for +7.5%.)
  constexpr bool CH = (VAR & 4096) == 0, MS = CH;
  f32x4v acc[CT * 8], mst[MS ? CT * 8 : 1];
#pragma unroll
  for (int i = 0; i < CT * 8; ++i) acc[i] = (f32x4v){0};
#pragma unroll
  for (int i = 0; i < (MS ? CT * 8 : 1); ++i) mst[i] = (f32x4v){0};
  int overflow = 0;

  // Dynamic range.  The image holds x * 2^-xs in f16 hi/lo with one exponent xs per workgroup
  // (uniform), so activations keep fp32's range (a freshly trained net in eval mode can grow
  // far beyond f16's 65504) at f16x3 precision.  xs is chosen BEFORE a layer's outputs are
  // stored, from a rigorous bound on them: |z| <= G_L * max(input) + B_L (+ max(residual) for
  // conv B), G_L = max over output channels of the L1 norm of the folded weights, B_L = max
  // |folded bias| (host, NetWeights::yrange), and max(input) measured by the previous epilogue
  // (workgroup max of its outputs through one LDS word).  xo = max(0, ilogb(bound) - 14) keeps
  // every stored value below 2^15; rescaling is by powers of two, hence exact, and ordinary nets
  // stay at xs = 0 (the results are then bit-identical to an unscaled kernel).
  int xs = 0;
  float mx_img = W.yrange[2 * CONV_LAYERS + 2];   // max |embedding| = max of the stem input
  float mx_blk = 0.f;                             // max of the current residual block's input
  unsigned* mxs = reinterpret_cast<unsigned*>(smem + IMG + AUXB - 16);
  if (tid == 0) mxs[0] = mxs[1] = 0u;
  int slot = 0;

  // Epilogue (stem and every conv): y = ReLU(acc * 2^(xs - e) + bias) stored in place as f16
  // hi/lo of y * 2^-xo (the scale folded into the fma); conv A seeds the accumulators with conv B's residual in conv B's units
  // (x_stored * 2^(e_B + xs - xo)), otherwise resets them.  Lane l holds channels
  // 16ct + 4(l>>4) + r of square 16pt + (l&15): 8 B per image part.  The lo parts and the
  // residual seed use v_fma_mix (bit-identical to the unfused forms, variant 1024;
  // test_mix_epilogue_bit_identical).  Ends with a barrier, after which mx_img holds the
  // workgroup max of the new image (true units).
  auto epilogue = [&](float inv, const float* bias, auto conv_a_t, float s_next, float bound) {
    constexpr bool conv_a = decltype(conv_a_t)::value;
    // floor(log2(bound)) - 14 for bound >= 2^14 (exponent field of a normal float); inf -> 114
    const int xo = bound >= 16384.f ? (int)((__float_as_uint(bound) >> 23) & 0xffu) - 127 - 14 : 0;
    // stored y = ReLU(acc * 2^(xs - e - xo) + bias * 2^-xo): the power-of-two output scale folded
    // into the fma (exact, so the same bits as scaling y afterwards)
    const float in_scale = __builtin_ldexpf(inv, xs - xo), st = __builtin_ldexpf(1.f, -xo);
    const float sseed = __builtin_ldexpf(s_next, xs - xo);
    float ymax = 0.f;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int co0 = 16 * CT * wave + 16 * ct + 4 * g;
      const float4 bu = *reinterpret_cast<const float4*>(bias + co0);
      const float4 bv = make_float4(bu.x * st, bu.y * st, bu.z * st, bu.w * st);
#pragma unroll
      for (int t = 0; t < 2 * NVB; ++t) {
        const int bb = t >> 1, pt = t & 1;
        f32x4v& acc_t = acc[ct * 8 + t];
        f32x4v& a = MS ? mst[MS ? ct * 8 + t : 0] : acc_t;   // the sum; the next layer's seed goes here
        if constexpr (CH) {
          if (pt == 1) {   // pending (square tile 1); zeroed for the next layer's first add
            a += acc_t;
            acc_t = (f32x4v){0};
          }
        }
        // ZL: the padding squares 30, 31 of square tile 1 are computed and stored like the others,
        // without a lane-divergent branch: their cells (rows 30, 31 of the chunk-major image) are
        // never a fragment source (off-board taps read the zero line), nor read by the heads, and
        // their values stay out of the workgroup max
        const bool real = pt == 0 || p1 < 30;
        if (ZL || real) {
          const int p = pt ? p1 : n;
          const int ah = (ZL ? zoff(0, bb, p, co0 >> 3) : ioff(0, bb, p, co0 >> 3)) + 8 * (g & 1), al = ah + PART;
          float y[4];
          y[0] = fmaxf(__builtin_fmaf(a[0], in_scale, bv.x), 0.f);
          y[1] = fmaxf(__builtin_fmaf(a[1], in_scale, bv.y), 0.f);
          y[2] = fmaxf(__builtin_fmaf(a[2], in_scale, bv.z), 0.f);
          y[3] = fmaxf(__builtin_fmaf(a[3], in_scale, bv.w), 0.f);
          const float ym = fmaxf(fmaxf(y[0], y[1]), fmaxf(y[2], y[3]));
          ymax = real ? fmaxf(ymax, ym) : ymax;   // stored units
          if constexpr (VAR & 1024) {   // reference form of the same epilogue (unfused)
            if constexpr (conv_a) {
              const f16x4 xh = *reinterpret_cast<const f16x4*>(smem + ah);
              const f16x4 xl = *reinterpret_cast<const f16x4*>(smem + al);
#pragma unroll
              for (int j = 0; j < 4; ++j) a[j] = __builtin_fmaf((float)xh[j], sseed, (float)xl[j] * sseed);
            } else {
              a = (f32x4v){0};
            }
            f16x4 yh, yl;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              yh[j] = (_Float16)y[j];
              yl[j] = (_Float16)(y[j] - (float)yh[j]);
            }
            *reinterpret_cast<f16x4*>(smem + ah) = yh;
            *reinterpret_cast<f16x4*>(smem + al) = yl;
            continue;
          }
          if constexpr (conv_a) {
            const uint2 xh = *reinterpret_cast<const uint2*>(smem + ah);
            const uint2 xl = *reinterpret_cast<const uint2*>(smem + al);
            a[0] = mix_lo(xh.x, sseed, mix_lo(xl.x, sseed, 0.f));
            a[1] = mix_hi(xh.x, sseed, mix_hi(xl.x, sseed, 0.f));
            a[2] = mix_lo(xh.y, sseed, mix_lo(xl.y, sseed, 0.f));
            a[3] = mix_hi(xh.y, sseed, mix_hi(xl.y, sseed, 0.f));
          } else {
            a = (f32x4v){0};
          }
          f16x4 yh;
#pragma unroll
          for (int j = 0; j < 4; ++j) yh[j] = (_Float16)y[j];
          const uint2 hp = __builtin_bit_cast(uint2, yh);
          *reinterpret_cast<uint2*>(smem + ah) = hp;
          *reinterpret_cast<uint2*>(smem + al) = make_uint2(lo_pair(hp.x, y[0], y[1]), lo_pair(hp.y, y[2], y[3]));
        } else {
          a = (f32x4v){0};
        }
      }
    }
    // workgroup max of the new image (y >= 0: float bits order as values; NaN above +inf)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ymax = fmaxf(ymax, __shfl_xor(ymax, o, 64));
    if (lane == 0) atomicMax(&mxs[slot], __float_as_uint(ymax));
    if (tid == 0) mxs[slot ^ 1] = 0u;   // every wave read it before this epilogue's first barrier
    xs = xo;
    __syncthreads();
    mx_img = __builtin_ldexpf(__uint_as_float(mxs[slot]), xo);   // true units
    slot ^= 1;
    if (!__builtin_isfinite(mx_img)) overflow = 1;   // fp32 overflow / NaN, as fp32 would produce
  };

  // ---------------- stem: conv3x3 8->256, K = 3 k-blocks of (4 taps x 8 channels) ----------
  char* simg = smem + IMG;
  stem_input<NT, ZL>(smem, simg, pos, b0, nb, W, tid);
  if constexpr (OT) {   // entry: row * RB | (g ^ (row & 15)) for square n (tile 0) or 16 + n (tile 1)
    if (wave == 0) {
      int* ot = reinterpret_cast<int*>(smem + IMG + AUXB);
      for (int e = 0; e < 18; ++e) {
        const int tap = e >> 1, pt = e & 1;
        if constexpr (ZL) {   // chunk g's cell | 1 on the board, the zero-line cell (bit 0 clear) off it
          const int p = pt ? p1 : n, ph = pt ? ph1 : ph0, pw = pt ? pw1 : pw0;
          const int dh = tap / 3 - 1, dw = tap % 3 - 1, sq = p + 5 * dh + dw;
          const bool valid = (p < 30) & ((unsigned)(ph + dh) < 6u) & ((unsigned)(pw + dw) < 5u);
          ot[e * 64 + lane] = valid ? (zrow(sq, g) | 1) : ZROWS_B + 16 * (sq & 15);
        } else {
          const int r = pt ? src_row(p1, ph1, pw1, tap) : src_row(n, ph0, pw0, tap);
          ot[e * 64 + lane] = r * RB | (g ^ (r & 15));
        }
      }
    }
  }
  __syncthreads();
  {
    const uint4* Ws = W.stemy + (size_t)(CT * wave) * 3 * 128 + lane;
    for (int kb = 0; kb < 3; ++kb) {
      f16x8 SA[2 * CT], SB[16];
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
        for (int bb = 0; bb < NVB; ++bb) {
          SB[part * 8 + 2 * bb] = *reinterpret_cast<const f16x8*>(simg + ((part * XB + bb) * IROWS + r0) * 16);
          SB[part * 8 + 2 * bb + 1] = *reinterpret_cast<const f16x8*>(simg + ((part * XB + bb) * IROWS + r1) * 16);
        }
      YMMA3(SA, SB);
    }
  }
  if constexpr (CH) {   // the stem's square-tile-0 sums (the epilogue adds the square-tile-1 ones)
#pragma unroll
    for (int i = 0; i < CT * 8; i += 2) mst[CH ? i : 0] += acc[i];
  }
  epilogue(W.stemx_inv[0], W.stem_b, std::false_type{}, 0.f,
           __builtin_fmaf(W.yrange[2 * CONV_LAYERS], mx_img, W.yrange[2 * CONV_LAYERS + 1]) * 1.0009765625f);
  stamp(st_stem);

  // ---------------- residual trunk: 18 convs, activations resident in LDS ----------------
  // Weights stream from L2 through a 3-slot register ring two k-blocks ahead.  Product
  // schedule: each k-block step runs as two half-steps, one per square tile, so only the 8
  // activation fragments of one tile are live (a 2 x 8-fragment ring): the next half's are read
  // from LDS during the current half, in 12 chunks of 4 MFMAs whose order sched_barrier pins
  // (HALF_PINNED: no accumulator copies, no spills).
  // the weight ring: 2 slots, one k-block ahead (VAR 16384: 3 slots, two ahead, round 2's; tail
  // instances: below)
  // Tail instances prefetch deeper: with 1, 2 or 3 boards a k-block is 384, 768 or 1,152 MFMA
  // cycles, less than an L2 round trip under load, and they have registers to spare (1 board: 200
  // of 512 with the 2-slot ring)
  constexpr int PD = (VAR & 16384) ? 2 : NVB == 1 ? 5 : NVB == 2 ? 3 : NVB == 3 ? 2 : 1, RS = PD + 1, U = CH ? 12 : 6;
  const char* otab = smem + IMG + AUXB + 4 * lane;   // OT: this lane's column of the table
  int tpre = 0;                                        // OT: the next half-step's table entry
  static_assert(KBY % U == 0 && U % RS == 0 && RS > PD, "ring");
  f16x8 A[RS][2 * CT], BH[2][8];
  const uint4* Wl = W.convy + (size_t)(CT * wave) * KBY * 128 + lane;
  // WB (product; VAR 65536 = off): weight fragments by buffer loads (descriptor over convy, the
  // wave's lane offset in a VGPR, layer / k-block / tile offsets in an SGPR) instead of 64-bit
  // global addresses
  constexpr bool WB = (VAR & 65536) == 0;
  // timing-only diagnostic forms (diagnostic library; wrong results by construction): the K loop
  // without its weight loads (DX_NOW, 1 << 20), without its fragment LDS reads (DX_NOB, 1 << 21),
  // without the chunk adds into the master sums (DX_NOADD, 1 << 22)
  // EL (1 << 23): every weight load of the next k-block issued in the first half-step of the
  // current one (the ring slot is free from its start), so a load has ~1.5 k-blocks of latency
  // instead of ~0.4 for the second half's loads; the same values, so bitwise the same results
  constexpr bool EL = (VAR & (1 << 23)) != 0;
  constexpr bool DX_NOW = (VAR & (1 << 20)) != 0, DX_NOB = (VAR & (1 << 21)) != 0, DX_NOADD = (VAR & (1 << 22)) != 0;
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc((void*)W.convy, (short)0, 0x7ffffff0, 0x00020000);
  const int voy = ((CT * wave) * KBY * 128 + lane) * 16;
  int lofs = 0;   // WB: the layer's byte offset in convy
  // byte offset (board 0, part 0) of the 16-B chunk ch of the source square of output square p
  // (row ph, file pw) for tap; off-board / padding: the zero row (ZL: the zero-line cell)
  auto frag_off = [](int p, int ph, int pw, int tap, int ch) {
    if constexpr (ZL) {
      return zsrc(p, ph, pw, tap, ch);
    } else {
      const int r = src_row(p, ph, pw, tap);
      return r * RB + ((ch ^ (r & 15)) << 4);
    }
  };
#define LOAD_A(S, KB)                                                                 \
  {                                                                                   \
    const int kk_ = (KB) < KBY ? (KB) : KBY - 1;                                      \
    const uint4* p_ = Wl + (size_t)kk_ * 128;                                         \
    _Pragma("unroll") for (int c_ = 0; c_ < CT; ++c_) {                               \
      if constexpr (WB) {                                                             \
        S[2 * c_] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(   \
            rsy, voy, lofs + (c_ * KBY + kk_) * 2048, 0));                            \
        S[2 * c_ + 1] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128( \
            rsy, voy, lofs + (c_ * KBY + kk_) * 2048 + 1024, 0));                     \
      } else {                                                                        \
        S[2 * c_] = __builtin_bit_cast(f16x8, p_[c_ * KBY * 128]);                    \
        S[2 * c_ + 1] = __builtin_bit_cast(f16x8, p_[c_ * KBY * 128 + 64]);           \
      }                                                                               \
    }                                                                                 \
  }
// one square tile's fragments of k-block KB: S[part*4 + board]
#define LOAD_BH(S, KB, PT)                                                            \
  {                                                                                   \
    const int kk_ = (KB) < KBY ? (KB) : KBY - 1;                                      \
    const int tap_ = kk_ >> 3, ch_ = 4 * (kk_ & 7) + g;                               \
    const int o_ = frag_off((PT) ? p1 : n, (PT) ? ph1 : ph0, (PT) ? pw1 : pw0, tap_, ch_); \
    _Pragma("unroll") for (int part_ = 0; part_ < 2; ++part_)                         \
    _Pragma("unroll") for (int bb_ = 0; bb_ < NVB; ++bb_)                             \
      S[part_ * 4 + bb_] = *reinterpret_cast<const f16x8*>(smem + part_ * PART + bb_ * BSTR + o_); \
  }
// product half-step: 12 chunks of 4 MFMAs in fixed program order (sched_barrier between
// chunks), LDS reads 2 per chunk in chunks 0-3, weight loads 1 per chunk in chunks 4-7
#define HALF_PINNED(KB, PT, AC, AP, BC, BN, KBN, PTN, FIRST, ADDT)                    \
  {                                                                                   \
    const int kk_ = (KBN) < KBY ? (KBN) : KBY - 1;                                    \
    int o_;                                                                           \
    if constexpr (OT) {                                                               \
      /* tpre holds the entry of (KBN, PTN); load the one of (KB + 1, PT) for the next half */ \
      if constexpr (ZL) {                                                             \
        /* on the board: entry = cell | 1, + 1024 (kk & 7) - 1; off: the entry (bit 0 clear) */ \
        o_ = mad_i24(tpre & 1, 1024 * (kk_ & 7) - 1, tpre);                             \
      } else {                                                                        \
        const int t_ = tpre, x_ = t_ ^ (4 * (kk_ & 7));                               \
        o_ = (t_ & ~31) | ((x_ & 31) << 4);                                           \
      }                                                                               \
      const int kq_ = ((KB) + 1) < KBY ? ((KB) + 1) : KBY - 1;                        \
      tpre = *reinterpret_cast<const int*>(otab + ((kq_ >> 3) * 2 + (PT)) * 256);     \
    } else {                                                                          \
      const int tap_ = kk_ >> 3, ch_ = 4 * (kk_ & 7) + g;                             \
      o_ = frag_off((PTN) ? p1 : n, (PTN) ? ph1 : ph0, (PTN) ? pw1 : pw0, tap_, ch_);  \
    }                                                                                 \
    const int o1_ = o_ + PART;                                                        \
    const int ka_ = ((KB) + PD) < KBY ? ((KB) + PD) : KBY - 1;                        \
    const uint4* pa_ = Wl + (size_t)ka_ * 128;                                        \
    _Pragma("unroll") for (int i_ = 0; i_ < 12 * CT; ++i_) {                          \
      if (i_ % 4 == 0) {                                                              \
        const int c_ = i_ / 4;                                                        \
        __builtin_amdgcn_sched_barrier(0);                                            \
        /* chunk c_ issues LDS reads [l0_, l1_) and weight loads [g0_, g1_) of the next half */ \
        /* 2 LDS reads per chunk 0-3, 1 load per chunk 4-7 */                        \
        const int l0_ = c_ < 4 ? 2 * c_ : 0, l1_ = c_ < 4 ? 2 * c_ + 2 : 0;           \
        /* EL: all 2 CT loads of the next k-block in the first half-step, chunks 1..2CT */ \
        const int g0_ = EL ? (((PT) == 0 && c_ >= 1 && c_ <= 2 * CT) ? c_ - 1 : 0)     \
                           : ((c_ >= 4 && c_ < 4 + CT) ? c_ - 4 : 0);                 \
        const int g1_ = EL ? (((PT) == 0 && c_ >= 1 && c_ <= 2 * CT) ? c_ : 0)         \
                           : ((c_ >= 4 && c_ < 4 + CT) ? c_ - 3 : 0);                 \
        /* part 1 from its own base (o_ + PART): the board offsets stay 16-bit immediates */ \
        _Pragma("unroll") for (int q_ = 0; q_ < 8; ++q_)                              \
          if (!DX_NOB && q_ >= l0_ && q_ < l1_ && (q_ & 3) < NVB)                     \
            BN[q_] = *reinterpret_cast<const f16x8*>(smem + ((q_ >> 2) ? o1_ : o_) + (q_ & 3) * BSTR); \
        _Pragma("unroll") for (int q_ = 0; q_ < 2 * CT; ++q_)                         \
          if (!DX_NOW && q_ >= g0_ && q_ < g1_) {                                     \
            const int ct_ = (EL ? 0 : (CT / 2) * (PT)) + (q_ >> 1), pp_ = q_ & 1;     \
            if constexpr (WB)                                                         \
              AP[2 * ct_ + pp_] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128( \
                  rsy, voy, lofs + (ct_ * KBY + ka_) * 2048 + pp_ * 1024, 0));        \
            else                                                                      \
              AP[2 * ct_ + pp_] = __builtin_bit_cast(f16x8, pa_[ct_ * KBY * 128 + pp_ * 64]); \
          }                                                                           \
        /* CH: the chunk sums of square tile ADDT into mst, 1-2 tiles per chunk */      \
        /* (tile j = 4 ct + board goes with chunk floor(3j / 4)) */                    \
        if (CH && !DX_NOADD && (ADDT) >= 0) {                                         \
          const int ja_ = (4 * c_ + 2) / 3, jb_ = ja_ + 1;                            \
          if ((ja_ & 3) < NVB) {                                                      \
            const int ix_ = (ja_ >> 2) * 8 + (ja_ & 3) * 2 + ((ADDT) > 0);            \
            add4(mst[CH ? ix_ : 0], acc[ix_]);                                        \
          }                                                                           \
          if (jb_ < 16 && (3 * jb_) / 4 == c_ && (jb_ & 3) < NVB) {                   \
            const int ix_ = (jb_ >> 2) * 8 + (jb_ & 3) * 2 + ((ADDT) > 0);            \
            add4(mst[CH ? ix_ : 0], acc[ix_]);                                        \
          }                                                                           \
        }                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                            \
      }                                                                               \
      const int ps_ = i_ / (4 * CT), ct_ = (i_ >> 2) % CT, bb_ = i_ & 3;              \
      const int wp_ = ps_ == 2 ? 1 : 0, xp_ = ps_ == 1 ? 1 : 0;                       \
      if (bb_ < NVB)                                                                  \
        acc[ct_ * 8 + bb_ * 2 + (PT)] = __builtin_amdgcn_mfma_f32_16x16x32_f16(       \
            AC[2 * ct_ + wp_], BC[xp_ * 4 + bb_],                                     \
            (CH && (FIRST) && ps_ == 0) ? (f32x4v){0} : acc[ct_ * 8 + bb_ * 2 + (PT)], 0, 0, 0); \
    }                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                \
  }
  for (int L = 0; L < CONV_LAYERS; ++L) {
#pragma unroll
    for (int p = 0; p < (DX_NOW ? RS : PD); ++p) LOAD_A(A[p], p);   // (DX_NOW: every slot defined once)
    LOAD_BH(BH[0], 0, 0);
    if constexpr (DX_NOB) LOAD_BH(BH[1], 0, 1);
    if constexpr (OT) tpre = *reinterpret_cast<const int*>(otab + 1 * 256);   // (k-block 0, tile 1)
    for (int kb = 0; kb < KBY; kb += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        HALF_PINNED(kb + u, 0, A[u % RS], A[(u + PD) % RS], BH[0], BH[1], kb + u, 1, u == 0, u == 0 ? 1 : -1);
        HALF_PINNED(kb + u, 1, A[u % RS], A[(u + PD) % RS], BH[1], BH[0], kb + u + 1, 0, u == 0,
                    u == U - 1 ? 0 : -1);
      }
    }
    stamp(st_k);
    Wl += CONVX_U4_PER_LAYER;
    lofs += (int)(CONVX_U4_PER_LAYER * 16);
    __syncthreads();   // every wave has finished reading this layer's input image
    // output bound (the margin 1 + 2^-10 covers the rounding of the bound's own arithmetic)
    if ((L & 1) == 0) {
      const float bound = __builtin_fmaf(W.yrange[2 * L], mx_img, W.yrange[2 * L + 1]) * 1.0009765625f;
      mx_blk = mx_img;
      epilogue(W.convx_inv[L], W.conv_b + L * 256, std::true_type{}, 1.0f / W.convx_inv[L + 1], bound);
    } else {
      const float bound = (__builtin_fmaf(W.yrange[2 * L], mx_img, W.yrange[2 * L + 1]) + mx_blk) * 1.0009765625f;
      epilogue(W.convx_inv[L], W.conv_b + L * 256, std::false_type{}, 0.f, bound);
    }
    stamp(st_epi);
  }
#undef HALF_PINNED
#undef LOAD_BH
#undef LOAD_A
  // (the timing-only forms compute garbage that may overflow: no flag from them)
  if (overflow && !(DX_NOW || DX_NOB || DX_NOADD)) atomicOr(D.pr.err, ERR_F16);

  // ---------------- heads (exp/policy.py:62-69, :76-79) ------------------------------------
  heads_reduce<NT, false, ZL>(smem, pos, b0, nb, W, tid, __builtin_ldexpf(1.f, xs));
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
  }
  heads_out<ZL>(D, smem, b0, nb, W, mode, logits_out, values_out, wave, lane);
}

template <bool STAMP, int VAR, int NVB = XB>
__global__ __launch_bounds__(256, 1) void k_net_y3(Dev D, NetWeights W, const Pos* __restrict__ pos,
                                                  const int32_t* __restrict__ count, int max_b, int mode,
                                                  float* __restrict__ logits_out, float* __restrict__ values_out,
                                                  unsigned long long* __restrict__ stamps, int ncu) {
  __shared__ __attribute__((aligned(16))) char smem[net_y3_smem(VAR)];
  net_y3_body<STAMP, VAR, NVB>(smem, blockIdx.x, D, W, pos, count, max_b, mode, logits_out, values_out, stamps, ncu);
}

// The three tail instances in one launch of 3 x ncu workgroups: workgroup i runs as the
// (1 + i / ncu)-board instance for CU slot i % ncu, and exits at once unless the remainder has that
// many boards per CU (one launch instead of three, two of which were always empty)
template <int VAR>
__global__ __launch_bounds__(256, 1) void k_net_y3_tail(Dev D, NetWeights W, const Pos* __restrict__ pos,
                                                       const int32_t* __restrict__ count, int max_b, int mode,
                                                       float* __restrict__ logits_out,
                                                       float* __restrict__ values_out, int ncu) {
  __shared__ __attribute__((aligned(16))) char smem[net_y3_smem(VAR)];
  const int nvb = 1 + (int)blockIdx.x / ncu, bid = (int)blockIdx.x % ncu;
  if (nvb == 1)
    net_y3_body<false, VAR, 1>(smem, bid, D, W, pos, count, max_b, mode, logits_out, values_out, nullptr, ncu);
  else if (nvb == 2)
    net_y3_body<false, VAR, 2>(smem, bid, D, W, pos, count, max_b, mode, logits_out, values_out, nullptr, ncu);
  else
    net_y3_body<false, VAR, 3>(smem, bid, D, W, pos, count, max_b, mode, logits_out, values_out, nullptr, ncu);
}

template <bool S>
static void launch_y3(int var, dim3 grid, hipStream_t s, const Dev& d, const NetWeights& w, const Pos* pos,
                      const int32_t* count, int max_b, int mode, float* logits, float* values,
                      unsigned long long* stamps) {
#ifdef MTAZ_NET_DIAG
  if (var == 1024)
    hipLaunchKernelGGL((k_net_y3<S, 1024>), grid, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits, values, stamps, 0);
  else if (var == 4096)
    hipLaunchKernelGGL((k_net_y3<S, 4096>), grid, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits, values, stamps, 0);
  else
#endif
    hipLaunchKernelGGL((k_net_y3<S, 0>), grid, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits, values, stamps, 0);
}

static int device_cus_y3() {
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

void launch_net_f16x3_r3(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                  float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                  int variant) {
  if (max_b <= 0) return;
  if (ev_begin) (void)hipEventRecord(ev_begin, s);
  const int ncu = device_cus_y3();
  if (variant == 0 && ncu > 0) {   // the product: full rounds, then the tail launches (k_net_y above)
    hipLaunchKernelGGL((k_net_y3<false, 0, XB>), dim3((max_b + XB - 1) / XB), dim3(256), 0, s, d, w, pos, count, max_b,
                       mode, logits_out, values_out, nullptr, ncu);
    hipLaunchKernelGGL((k_net_y3_tail<0>), dim3(3 * ncu), dim3(256), 0, s, d, w, pos, count, max_b, mode, logits_out,
                       values_out, ncu);
  } else {   // variant 1: 4 boards per workgroup throughout
    launch_y3<false>(variant == 1 ? 0 : variant, dim3((max_b + XB - 1) / XB), s, d, w, pos, count, max_b, mode,
                    logits_out, values_out, nullptr);
  }
  if (ev_end) (void)hipEventRecord(ev_end, s);
}

#ifdef MTAZ_NET_DIAG
void launch_net_f16x3_r3_stamped(const Dev& d, const NetWeights& w, const Pos* pos, int n, float* logits_out,
                          float* values_out, unsigned long long* stamps, hipStream_t s, int variant) {
  if (n <= 0) return;
  launch_y3<true>(variant, dim3((n + XB - 1) / XB), s, d, w, pos, nullptr, n, (int)NET_FULL_LOGITS, logits_out,
                 values_out, stamps);
}

#endif

}  // namespace mtaz
