// Fused policy/value network for MCTS leaf evaluation (exp/policy.py:71-80 + the
// leaf prior extraction of exp/agent.py:67-69) in ONE launch per simulation wave.
//
// Workgroup = 4 boards, 256 threads (4 waves, one per SIMD).  The boards'
// activations never leave the CU: they live in LDS as fp16 hi/lo images
// (x = hi + lo, hi = f16(x), lo = f16(x - hi)) of [board][square][channel],
// 2 x 63,488 B, rewritten in place after every convolution.  Each 3x3 conv is an
// implicit GEMM  Y[co][sq] = sum_k W[co][k] X[k][sq], k = tap*256 + ci (K = 2304),
// on v_mfma_f32_32x32x16_f16 with three passes  Wh*Xh + Wh*Xl + Wl*Xh  accumulated
// in fp32 (weights pre-scaled by 2^e so their lo parts stay normal).  That is
// fp32-accurate (CPU emulation: same 1e-7 logit error as fp32 vs fp64) at 16/3 of
// the fp32 MFMA rate.  Wave w owns output channels [64w, 64w+64) x all 4 boards:
// 8 accumulator tiles of 32 channels x 32 squares (squares 30, 31 are padding).
// Weights stream from L2 (2.36 MB per layer, shared by every workgroup) into
// registers two k-blocks ahead; activation fragments are read from LDS one k-block
// ahead with ds_read_b128 on an XOR-swizzled image (conflict-free).  Residual
// blocks: the conv-A epilogue reads the block input x and seeds the conv-B
// accumulators with 2^e_B * x, so no extra residual buffer exists.
#include "engine.h"

namespace mtaz {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16x __attribute__((ext_vector_type(16)));

constexpr int XB = 4;                     // boards per workgroup
constexpr int IROWS = 31;                 // image rows: squares 0..29 + zero row
constexpr int ZROW = 30;
constexpr int RB = 512;                   // bytes per row: 256 channels x f16
constexpr int PARTB = XB * IROWS * RB;    // 63,488 B per part
constexpr int IMGB = 2 * PARTB;           // 126,976 B
constexpr int AUXB = XB * 8 * 56 * 4;     // 7,168 B: stem input / head features
constexpr int KBLK = 144;                 // 2304 / 16

__device__ __forceinline__ int ioff(int part, int bb, int row, int chunk) {
  return part * PARTB + (bb * IROWS + row) * RB + ((chunk ^ (row & 15)) << 4);
}

// image row holding the source square of output square `col` for tap (dh, dw), or the zero row
__device__ __forceinline__ int src_row(int col, int ph, int pw, int tap) {
  const int dh = tap / 3 - 1, dw = tap - 3 * (tap / 3) - 1;
  const int r = ph + dh, c = pw + dw;
  return (col < 30 && r >= 0 && r < 6 && c >= 0 && c < 5) ? col + 5 * dh + dw : ZROW;
}

__device__ __forceinline__ int padpos_x(int p) { return (p / 5 + 1) * 7 + (p % 5 + 1); }

// Three split passes Wh*Xh + Wh*Xl + Wl*Xh over the wave's 8 tiles (2 channel tiles x
// XB boards); SA = {ct0 hi, ct0 lo, ct1 hi, ct1 lo}, SB = {bb0 hi, bb0 lo, ...}.  Pass-major
// order keeps 7 independent MFMAs between two updates of one accumulator.
#define MMA3(SA, SB)                                                                                  \
  {                                                                                                   \
    _Pragma("unroll") for (int ct_ = 0; ct_ < 2; ++ct_)                                               \
    _Pragma("unroll") for (int bb_ = 0; bb_ < XB; ++bb_)                                              \
      acc[ct_ * 4 + bb_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(SA[2 * ct_], SB[2 * bb_], acc[ct_ * 4 + bb_], 0, 0, 0); \
    _Pragma("unroll") for (int ct_ = 0; ct_ < 2; ++ct_)                                               \
    _Pragma("unroll") for (int bb_ = 0; bb_ < XB; ++bb_)                                              \
      acc[ct_ * 4 + bb_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(SA[2 * ct_], SB[2 * bb_ + 1], acc[ct_ * 4 + bb_], 0, 0, 0); \
    _Pragma("unroll") for (int ct_ = 0; ct_ < 2; ++ct_)                                               \
    _Pragma("unroll") for (int bb_ = 0; bb_ < XB; ++bb_)                                              \
      acc[ct_ * 4 + bb_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(SA[2 * ct_ + 1], SB[2 * bb_], acc[ct_ * 4 + bb_], 0, 0, 0); \
  }

// one split pass (8 MFMAs): W part WP (0 hi / 1 lo) x X part XP
#define MMA_PASS(SA, SB, WP, XP)                                                                      \
  {                                                                                                   \
    _Pragma("unroll") for (int ct_ = 0; ct_ < 2; ++ct_)                                               \
    _Pragma("unroll") for (int bb_ = 0; bb_ < XB; ++bb_)                                              \
      acc[ct_ * 4 + bb_] = __builtin_amdgcn_mfma_f32_32x32x16_f16(SA[2 * ct_ + (WP)], SB[2 * bb_ + (XP)], acc[ct_ * 4 + bb_], 0, 0, 0); \
  }

// STAMP = diagnostic build only: thread 0 accumulates s_memtime deltas per phase
// (stem, conv K loops, conv epilogues, heads) into stamps[block*4 + phase].
// VAR: variant bits for in-process A/B timing (tools/bench_net.py); 0 = the product kernel.
//   bit 0: stem on the VALU in fp32 instead of the f16 MFMA split
template <bool STAMP, int VAR>
__global__ __launch_bounds__(256, 1) void k_net_x(Dev D, NetWeights W, const Pos* __restrict__ pos,
                                                  const int32_t* __restrict__ count, int max_b, int mode,
                                                  float* __restrict__ logits_out, float* __restrict__ values_out,
                                                  unsigned long long* __restrict__ stamps) {
  __shared__ __attribute__((aligned(16))) char smem[IMGB + AUXB];
  const int nb = count ? *count : max_b;
  const int b0 = blockIdx.x * XB;
  if (b0 >= nb) return;
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, col = lane & 31, h = lane >> 5;
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

  const int ph = col / 5, pw = col % 5;
  f32x16x acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = (f32x16x){0};
  int overflow = 0;

  // Epilogue of every conv (and the stem): y = ReLU(acc * 2^-e + bias) written in place as
  // f16 hi/lo.  conv_a: the image still holds the block input x -> seed the next conv's
  // accumulators with 2^e_next * x (the residual of conv B); otherwise reset them.
  auto epilogue = [&](float inv, const float* bias, bool conv_a, float s_next) {
    if (col < 30) {
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co0 = (2 * wave + ct) * 32 + 8 * g + 4 * h;
          const float4 bv = *reinterpret_cast<const float4*>(bias + co0);
#pragma unroll
          for (int bb = 0; bb < XB; ++bb) {
            f32x16x& a = acc[ct * 4 + bb];
            const int ah = ioff(0, bb, col, co0 >> 3) + 8 * h, al = ioff(1, bb, col, co0 >> 3) + 8 * h;
            float y[4];
            y[0] = fmaxf(a[4 * g + 0] * inv + bv.x, 0.f);
            y[1] = fmaxf(a[4 * g + 1] * inv + bv.y, 0.f);
            y[2] = fmaxf(a[4 * g + 2] * inv + bv.z, 0.f);
            y[3] = fmaxf(a[4 * g + 3] * inv + bv.w, 0.f);
            if (conv_a) {
              const f16x4 xh = *reinterpret_cast<const f16x4*>(smem + ah);
              const f16x4 xl = *reinterpret_cast<const f16x4*>(smem + al);
#pragma unroll
              for (int j = 0; j < 4; ++j) a[4 * g + j] = ((float)xh[j] + (float)xl[j]) * s_next;
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) a[4 * g + j] = 0.f;
            }
            f16x4 yh, yl;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              overflow |= y[j] >= 65504.f;
              yh[j] = (_Float16)y[j];
              yl[j] = (_Float16)(y[j] - (float)yh[j]);
            }
            *reinterpret_cast<f16x4*>(smem + ah) = yh;
            *reinterpret_cast<f16x4*>(smem + al) = yl;
          }
        }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = (f32x16x){0};
    }
  };

  // ---------------- stem: tokens -> Embedding(7,4) -> conv3x3 8->256 + BN + ReLU ----------
  // Same implicit GEMM on f16 MFMA with K = 5 k-blocks of (2 taps x 8 channels); the input
  // image [part][board][row][8 ch] f16 (rows = squares in the mover's view + zero row)
  // sits in the aux region.
  char* simg = smem + IMGB;
  for (int i = tid; i < 2 * XB * 32; i += 256) {
    const int part = i / (XB * 32), bb = (i / 32) % XB, ch = i & 31;
    *reinterpret_cast<uint4*>(smem + ioff(part, bb, ZROW, ch)) = make_uint4(0, 0, 0, 0);
  }
  if constexpr (VAR & 1) {
    // A/B variant: fp32 VALU stem, thread = output channel
    float* xin = reinterpret_cast<float*>(simg);          // [bb][8][56] fp32, zero padded
    for (int i = tid; i < XB * 8 * 56; i += 256) xin[i] = 0.f;
    __syncthreads();
    if (tid < XB * 30) {
      const int bb = tid / 30, i = tid % 30;
      const int b = b0 + bb;
      int own = 0, opp = 0;
      if (b < nb) {
        const BB bd = unpack(pos[b]);
        const int s = bd.white ? (5 - i / 5) * 5 + i % 5 : (i / 5) * 5 + (4 - i % 5);
        const int t = piece_type_at(bd, s);
        const bool mine = ((bd.white ? bd.w : bd.b) >> s) & 1u;
        own = mine ? token_code(t) : 0;
        opp = (t && !mine) ? token_code(t) : 0;
      }
      const int pp = padpos_x(i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xin[bb * 448 + e * 56 + pp] = W.emb[own * 4 + e];
        xin[bb * 448 + (4 + e) * 56 + pp] = W.emb[opp * 4 + e];
      }
    }
    __syncthreads();
    const int co = tid;
    float w[72];
#pragma unroll
    for (int j = 0; j < 72; ++j) w[j] = W.stem_w[co * 72 + j];
    const float bias = W.stem_b[co];
    for (int bb = 0; bb < XB; ++bb) {
      const float* xb = xin + bb * 448;
      for (int p = 0; p < 30; ++p) {
        const int pp = padpos_x(p);
        float a = bias;
#pragma unroll
        for (int ci = 0; ci < 8; ++ci)
#pragma unroll
          for (int tap = 0; tap < 9; ++tap) a += w[ci * 9 + tap] * xb[ci * 56 + pp + (tap / 3 - 1) * 7 + (tap % 3 - 1)];
        const float y = fmaxf(a, 0.f);
        const _Float16 hi = (_Float16)y;
        const _Float16 lo = (_Float16)(y - (float)hi);
        *reinterpret_cast<_Float16*>(smem + ioff(0, bb, p, co >> 3) + (co & 7) * 2) = hi;
        *reinterpret_cast<_Float16*>(smem + ioff(1, bb, p, co >> 3) + (co & 7) * 2) = lo;
      }
    }
    __syncthreads();
  } else {
  for (int i = tid; i < 2 * XB * IROWS; i += 256) *reinterpret_cast<uint4*>(simg + i * 16) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  if (tid < XB * 30) {
    const int bb = tid / 30, i = tid % 30;          // i = square index in the mover's view
    const int b = b0 + bb;
    int own = 0, opp = 0;
    if (b < nb) {
      const BB bd = unpack(pos[b]);
      const int s = bd.white ? (5 - i / 5) * 5 + i % 5 : (i / 5) * 5 + (4 - i % 5);
      const int t = piece_type_at(bd, s);
      const bool mine = ((bd.white ? bd.w : bd.b) >> s) & 1u;
      own = mine ? token_code(t) : 0;
      opp = (t && !mine) ? token_code(t) : 0;
    }
    f16x8 xh, xl;
#pragma unroll
    for (int c = 0; c < 8; ++c) {                   // channel c = plane*4 + e (exp/policy.py:73-74)
      const float v = W.emb[(c < 4 ? own : opp) * 4 + (c & 3)];
      xh[c] = (_Float16)v;
      xl[c] = (_Float16)(v - (float)xh[c]);
    }
    *reinterpret_cast<f16x8*>(simg + (bb * IROWS + i) * 16) = xh;
    *reinterpret_cast<f16x8*>(simg + ((XB + bb) * IROWS + i) * 16) = xl;
  }
  __syncthreads();
  {
    const uint4* Ws = W.stemx + (size_t)(2 * wave) * 5 * 128 + lane;
    for (int kb = 0; kb < 5; ++kb) {
      f16x8 SA[4], SB[8];
      const uint4* p = Ws + kb * 128;
      SA[0] = __builtin_bit_cast(f16x8, p[0]);
      SA[1] = __builtin_bit_cast(f16x8, p[64]);
      SA[2] = __builtin_bit_cast(f16x8, p[5 * 128]);
      SA[3] = __builtin_bit_cast(f16x8, p[5 * 128 + 64]);
      const int tap = 2 * kb + h;
      const int src = tap < 9 ? src_row(col, ph, pw, tap) : ZROW;
#pragma unroll
      for (int bb = 0; bb < XB; ++bb) {
        SB[2 * bb] = *reinterpret_cast<const f16x8*>(simg + (bb * IROWS + src) * 16);
        SB[2 * bb + 1] = *reinterpret_cast<const f16x8*>(simg + ((XB + bb) * IROWS + src) * 16);
      }
      MMA3(SA, SB);
    }
  }
  epilogue(W.stemx_inv[0], W.stem_b, false, 0.f);
  __syncthreads();
  }

  stamp(st_stem);
  // ---------------- residual trunk: 18 convs, activations resident in LDS ----------------

  for (int L = 0; L < CONV_LAYERS; ++L) {
    const uint4* Wl = W.convx + (size_t)L * CONVX_U4_PER_LAYER + (size_t)(2 * wave) * KBLK * 2 * 64 + lane;
    f16x8 A0[4], A1[4], A2[4], B0[8], B1[8];
#define LOAD_A(S, KB)                                                                 \
    {                                                                                 \
      const int kk_ = (KB) < KBLK ? (KB) : KBLK - 1;                                  \
      const uint4* p_ = Wl + (size_t)kk_ * 128;                                       \
      S[0] = __builtin_bit_cast(f16x8, p_[0]);                                        \
      S[1] = __builtin_bit_cast(f16x8, p_[64]);                                       \
      S[2] = __builtin_bit_cast(f16x8, p_[KBLK * 128]);                               \
      S[3] = __builtin_bit_cast(f16x8, p_[KBLK * 128 + 64]);                          \
    }
#define LOAD_B(S, KB)                                                                 \
    {                                                                                 \
      const int kk_ = (KB) < KBLK ? (KB) : KBLK - 1;                                  \
      const int src_ = src_row(col, ph, pw, kk_ >> 4);                                \
      const int off_ = src_ * RB + (((2 * (kk_ & 15) + h) ^ (src_ & 15)) << 4);       \
      _Pragma("unroll") for (int bb_ = 0; bb_ < XB; ++bb_) {                          \
        S[2 * bb_] = *reinterpret_cast<const f16x8*>(smem + bb_ * IROWS * RB + off_); \
        S[2 * bb_ + 1] = *reinterpret_cast<const f16x8*>(smem + PARTB + bb_ * IROWS * RB + off_); \
      }                                                                               \
    }
#define STEP(KB, AC, AP, BC, BP)                  \
    if constexpr (VAR & 8) {                      \
      LOAD_A(AP, (KB) + 2);                       \
      LOAD_B(BP, (KB) + 1);                       \
      MMA3(AC, BC);                               \
      _Pragma("unroll") for (int g_ = 0; g_ < 4; ++g_) {           \
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);         \
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);         \
      }                                                            \
      _Pragma("unroll") for (int g_ = 0; g_ < 8; ++g_) {           \
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);         \
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);         \
      }                                                            \
      __builtin_amdgcn_sched_barrier(0);          \
    } else if constexpr (VAR & 2) {               \
      MMA_PASS(AC, BC, 0, 0);                     \
      __builtin_amdgcn_sched_barrier(0);          \
      LOAD_A(AP, (KB) + 2);                       \
      __builtin_amdgcn_sched_barrier(0);          \
      MMA_PASS(AC, BC, 0, 1);                     \
      __builtin_amdgcn_sched_barrier(0);          \
      LOAD_B(BP, (KB) + 1);                       \
      __builtin_amdgcn_sched_barrier(0);          \
      MMA_PASS(AC, BC, 1, 0);                     \
      __builtin_amdgcn_sched_barrier(0);          \
    } else {                                      \
      LOAD_A(AP, (KB) + 2);                       \
      LOAD_B(BP, (KB) + 1);                       \
      __builtin_amdgcn_sched_barrier(0);          \
      MMA3(AC, BC);                               \
      __builtin_amdgcn_sched_barrier(0);          \
    }
    LOAD_A(A0, 0);
    LOAD_A(A1, 1);
    LOAD_B(B0, 0);
    for (int kb = 0; kb < KBLK; kb += 6) {
      STEP(kb + 0, A0, A2, B0, B1);
      STEP(kb + 1, A1, A0, B1, B0);
      STEP(kb + 2, A2, A1, B0, B1);
      STEP(kb + 3, A0, A2, B1, B0);
      STEP(kb + 4, A1, A0, B0, B1);
      STEP(kb + 5, A2, A1, B1, B0);
    }
#undef STEP
#undef LOAD_B
#undef LOAD_A
    stamp(st_k);
    __syncthreads();   // every wave has finished reading this layer's input image

    // epilogue: y = ReLU(acc * 2^-e + bias) (conv B: acc already holds 2^e * x, the residual)
    const bool conv_a = (L & 1) == 0;
    epilogue(W.convx_inv[L], W.conv_b + L * 256, conv_a, conv_a ? 1.0f / W.convx_inv[L + 1] : 0.f);
    __syncthreads();
    stamp(st_epi);
  }
  if (overflow) atomicOr(D.pr.err, ERR_F16);

  // ---------------- heads (exp/policy.py:62-69, :76-79) ------------------------------------
  float* fp = reinterpret_cast<float*>(smem + IMGB);   // [XB][64]: pconv features (60) + clock
  float* fv = fp + XB * 64;                            // [XB][32]: vconv features (30) + clock
  float* red = fv + XB * 32;                           // [XB][256]
  for (int t = tid; t < XB * 90; t += 256) {
    const int bb = t / 90, o = (t % 90) / 30, p = t % 30;
    const float* wr = o < 2 ? W.pconv_w + o * 256 : W.vconv_w;
    float s = 0.f;
    for (int c = 0; c < 32; ++c) {
      const f16x8 xh = *reinterpret_cast<const f16x8*>(smem + ioff(0, bb, p, c));
      const f16x8 xl = *reinterpret_cast<const f16x8*>(smem + ioff(1, bb, p, c));
#pragma unroll
      for (int j = 0; j < 8; ++j) s += wr[8 * c + j] * ((float)xh[j] + (float)xl[j]);
    }
    s = fmaxf(s + (o < 2 ? W.pconv_b[o] : W.vconv_b[0]), 0.f);
    if (o < 2) fp[bb * 64 + o * 30 + p] = s; else fv[bb * 32 + p] = s;
  }
  if (tid < XB) {
    const int b = b0 + tid;
    const float clk = b < nb ? encode_clock(unpack(pos[b])) : 0.f;
    fp[tid * 64 + 60] = clk;
    fv[tid * 32 + 30] = clk;
  }
  __syncthreads();
  {
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
  stamp(st_heads);
  if constexpr (STAMP) {
    if (tid == 0) {
      stamps[blockIdx.x * 6 + 0] = st_stem;
      stamps[blockIdx.x * 6 + 1] = st_k;
      stamps[blockIdx.x * 6 + 2] = st_epi;
      stamps[blockIdx.x * 6 + 3] = st_heads;
      stamps[blockIdx.x * 6 + 4] = __builtin_amdgcn_s_memtime() - t_start;      // shader cycles
      stamps[blockIdx.x * 6 + 5] = __builtin_amdgcn_s_memrealtime() - r_start;  // 100 MHz ticks
    }
  }
  // wave bb finishes board bb: value, then policy logits / legal softmax
  const int bb = wave;
  const int b = b0 + bb;
  if (b >= nb) return;
  const float v = tanhf(red[bb * 256] + W.vl2_b[0]);
  const float* f = fp + bb * 64;
  if (mode == NET_FULL_LOGITS) {
    if (lane == 0) values_out[b] = v;
    for (int a = lane; a < NUM_ACTIONS; a += 64) {
      float l = W.plin_b[a];
      for (int j = 0; j < 61; ++j) l += W.plin_w[a * 61 + j] * f[j];
      logits_out[(size_t)b * NUM_ACTIONS + a] = l;
    }
    return;
  }
  if (lane == 0) D.lf.v[b] = v;
  const int t = D.lf.tree[b];
  const uint32_t n = D.lf.node[b];
  const int k = D.tr.node_k[(size_t)t * D.tr.NC + n];
  const uint32_t e0 = D.tr.node_e0[(size_t)t * D.tr.NC + n];
  const uint16_t* codes = D.tr.e_code + (size_t)t * D.tr.EC + e0;
  float lg[KMAX / 64];
  float mx = -__builtin_inff();
#pragma unroll
  for (int r = 0; r < KMAX / 64; ++r) {
    const int c = lane + 64 * r;
    float l = -__builtin_inff();
    if (c < k) {
      const int a = codes[c];
      l = W.plin_b[a];
      for (int j = 0; j < 61; ++j) l += W.plin_w[a * 61 + j] * f[j];
    }
    lg[r] = l;
    mx = fmaxf(mx, l);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
#pragma unroll
  for (int r = 0; r < KMAX / 64; ++r) {
    lg[r] = (lane + 64 * r < k) ? expf(lg[r] - mx) : 0.f;
    sum += lg[r];
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
#pragma unroll
  for (int r = 0; r < KMAX / 64; ++r) {
    const int c = lane + 64 * r;
    if (c < k) D.lf.P[(size_t)b * KMAX + c] = lg[r] / sum;
  }
}

template <bool S>
static void launch_variant(int var, dim3 grid, hipStream_t s, const Dev& d, const NetWeights& w, const Pos* pos,
                           const int32_t* count, int max_b, int mode, float* logits, float* values,
                           unsigned long long* stamps) {
  switch (var) {
#define MTAZ_VAR_CASE(V)                                                                                    \
    case V:                                                                                                   \
      hipLaunchKernelGGL((k_net_x<S, V>), grid, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits, values, \
                         stamps);                                                                             \
      break;
    MTAZ_VAR_CASE(1)
    MTAZ_VAR_CASE(2)
    MTAZ_VAR_CASE(8)
#undef MTAZ_VAR_CASE
    default:
      hipLaunchKernelGGL((k_net_x<S, 0>), grid, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits, values, stamps);
  }
}

void launch_net_x(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                  float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                  int variant) {
  if (max_b <= 0) return;
  if (ev_begin) (void)hipEventRecord(ev_begin, s);
  launch_variant<false>(variant, dim3((max_b + XB - 1) / XB), s, d, w, pos, count, max_b, mode, logits_out, values_out,
                        nullptr);
  if (ev_end) (void)hipEventRecord(ev_end, s);
}

void launch_net_x_stamped(const Dev& d, const NetWeights& w, const Pos* pos, int n, float* logits_out,
                          float* values_out, unsigned long long* stamps, hipStream_t s, int variant) {
  if (n <= 0) return;
  launch_variant<true>(variant, dim3((n + XB - 1) / XB), s, d, w, pos, nullptr, n, (int)NET_FULL_LOGITS, logits_out,
                       values_out, stamps);
}

}  // namespace mtaz
