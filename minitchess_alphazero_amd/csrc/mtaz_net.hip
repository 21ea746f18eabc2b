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
#include <type_traits>

#include "net_common.h"

namespace mtaz {

using namespace netc;
typedef float f32x16x __attribute__((ext_vector_type(16)));
constexpr int KBLK = 144;                 // 2304 / 16

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

// STAMP = diagnostic build only: thread 0 accumulates s_memtime deltas per phase
// (stem, conv K loops, conv epilogues, heads) into stamps[block*4 + phase].
// VAR: variant bits for in-process A/B timing (tools/bench_net.py); 0 = its best schedule.
// k_net_x is the A/B reference for the product kernel k_net_y (mtaz_net16.hip): same
// algorithm on v_mfma_f32_32x32x16_f16, selected by variant bit NET_VAR_X.
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
  // conv_a is a compile-time flag (std::true_type / false_type) so the conv-A and conv-B
  // epilogues are two straight-line bodies.  The residual seed xh*s + xl*s and the lo part
  // fma(hi, -1, y) are exact in fp32 (s is a power of two; y - hi is representable), so
  // the stored values are the same bits as the unfused expressions.
  auto epilogue = [&](float inv, const float* bias, auto conv_a_t, float s_next) {
    constexpr bool conv_a = decltype(conv_a_t)::value;
    if (col < 30) {
      float ymax = 0.f;
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
            y[0] = fmaxf(__builtin_fmaf(a[4 * g + 0], inv, bv.x), 0.f);
            y[1] = fmaxf(__builtin_fmaf(a[4 * g + 1], inv, bv.y), 0.f);
            y[2] = fmaxf(__builtin_fmaf(a[4 * g + 2], inv, bv.z), 0.f);
            y[3] = fmaxf(__builtin_fmaf(a[4 * g + 3], inv, bv.w), 0.f);
            if constexpr (conv_a) {
              const f16x4 xh = *reinterpret_cast<const f16x4*>(smem + ah);
              const f16x4 xl = *reinterpret_cast<const f16x4*>(smem + al);
#pragma unroll
              for (int j = 0; j < 4; ++j) a[4 * g + j] = __builtin_fmaf((float)xh[j], s_next, (float)xl[j] * s_next);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j) a[4 * g + j] = 0.f;
            }
            f16x4 yh, yl;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              ymax = fmaxf(ymax, y[j]);
              yh[j] = (_Float16)y[j];
              yl[j] = (_Float16)__builtin_fmaf((float)yh[j], -1.f, y[j]);
            }
            *reinterpret_cast<f16x4*>(smem + ah) = yh;
            *reinterpret_cast<f16x4*>(smem + al) = yl;
          }
        }
      overflow |= ymax >= 65504.f;
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
  stem_input(smem, simg, pos, b0, nb, W, tid);
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
  epilogue(W.stemx_inv[0], W.stem_b, std::false_type{}, 0.f);
  __syncthreads();

  stamp(st_stem);
  // ---------------- residual trunk: 18 convs, activations resident in LDS ----------------

  // Weights stream from L2 through a ring of RS register slots PD k-blocks ahead of their
  // use; activation fragments come from LDS one k-block ahead.
  constexpr int PD = 2, RS = 3, U = 6;                   // U: unroll, a multiple of RS and of 2
  static_assert(KBLK % U == 0 && U % RS == 0 && RS > PD, "ring");
  f16x8 A[RS][4], B[2][8];
  const uint4* Wl = W.convx + (size_t)(2 * wave) * KBLK * 2 * 64 + lane;
#define LOAD_A(S, KB)                                                                 \
  {                                                                                   \
    const int kk_ = (KB) < KBLK ? (KB) : KBLK - 1;                                    \
    const uint4* p_ = Wl + (size_t)kk_ * 128;                                         \
    S[0] = __builtin_bit_cast(f16x8, p_[0]);                                          \
    S[1] = __builtin_bit_cast(f16x8, p_[64]);                                         \
    S[2] = __builtin_bit_cast(f16x8, p_[KBLK * 128]);                                 \
    S[3] = __builtin_bit_cast(f16x8, p_[KBLK * 128 + 64]);                            \
  }
#define LOAD_B(S, KB)                                                                 \
  {                                                                                   \
    const int kk_ = (KB) < KBLK ? (KB) : KBLK - 1;                                    \
    const int src_ = src_row(col, ph, pw, kk_ >> 4);                                  \
    const int off_ = src_ * RB + (((2 * (kk_ & 15) + h) ^ (src_ & 15)) << 4);         \
    _Pragma("unroll") for (int bb_ = 0; bb_ < XB; ++bb_)                              \
      S[2 * bb_] = *reinterpret_cast<const f16x8*>(smem + bb_ * IROWS * RB + off_);   \
    _Pragma("unroll") for (int bb_ = 0; bb_ < XB; ++bb_)                              \
      S[2 * bb_ + 1] = *reinterpret_cast<const f16x8*>(smem + PARTB + bb_ * IROWS * RB + off_); \
  }
// Product schedule: the 24 MFMAs of a step interleaved with its loads by
// sched_group_barrier (2 MFMA : 1 global load x4, then 2 MFMA : 1 ds_read x8), so the
// loads issue in the MFMA shadow.  Variants: 128 = the next k-block's LDS reads first, in
// consumption order, one per MFMA; 4 = all loads first, then the 24 MFMAs (first schedule).
#define STEP(KB, AC, AP, BC, BP)                  \
  if constexpr (VAR & 128) {                      \
    LOAD_B(BP, (KB) + 1);                         \
    LOAD_A(AP, (KB) + PD);                        \
    MMA3(AC, BC);                                 \
    _Pragma("unroll") for (int g_ = 0; g_ < 8; ++g_) {           \
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);         \
    }                                                            \
    _Pragma("unroll") for (int g_ = 0; g_ < 4; ++g_) {           \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);         \
    }                                                            \
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);           \
    __builtin_amdgcn_sched_barrier(0);            \
  } else if constexpr (VAR & 4) {                 \
    LOAD_A(AP, (KB) + PD);                        \
    LOAD_B(BP, (KB) + 1);                         \
    __builtin_amdgcn_sched_barrier(0);            \
    MMA3(AC, BC);                                 \
    __builtin_amdgcn_sched_barrier(0);            \
  } else {                                        \
    LOAD_A(AP, (KB) + PD);                        \
    LOAD_B(BP, (KB) + 1);                         \
    MMA3(AC, BC);                                 \
    _Pragma("unroll") for (int g_ = 0; g_ < 4; ++g_) {           \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);         \
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);         \
    }                                                            \
    _Pragma("unroll") for (int g_ = 0; g_ < 8; ++g_) {           \
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);         \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);         \
    }                                                            \
    __builtin_amdgcn_sched_barrier(0);            \
  }
  for (int L = 0; L < CONV_LAYERS; ++L) {
#pragma unroll
    for (int p = 0; p < PD; ++p) LOAD_A(A[p], p);
    LOAD_B(B[0], 0);
    for (int kb = 0; kb < KBLK; kb += U) {
#pragma unroll
      for (int u = 0; u < U; ++u) STEP(kb + u, A[u % RS], A[(u + PD) % RS], B[u & 1], B[(u + 1) & 1]);
    }
    stamp(st_k);
    Wl += CONVX_U4_PER_LAYER;
    __syncthreads();   // every wave has finished reading this layer's input image

    // epilogue: y = ReLU(acc * 2^-e + bias) (conv B: acc already holds 2^e * x, the residual)
    if ((L & 1) == 0)
      epilogue(W.convx_inv[L], W.conv_b + L * 256, std::true_type{}, 1.0f / W.convx_inv[L + 1]);
    else
      epilogue(W.convx_inv[L], W.conv_b + L * 256, std::false_type{}, 0.f);
    __syncthreads();
    stamp(st_epi);
  }
#undef STEP
#undef LOAD_B
#undef LOAD_A
  if (overflow) atomicOr(D.pr.err, ERR_F16);

  // ---------------- heads (exp/policy.py:62-69, :76-79) ------------------------------------
  heads_reduce(smem, pos, b0, nb, W, tid);
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
  heads_out(D, smem, b0, nb, W, mode, logits_out, values_out, wave, lane);
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
    MTAZ_VAR_CASE(4)
    MTAZ_VAR_CASE(128)
#undef MTAZ_VAR_CASE
    default:
      hipLaunchKernelGGL((k_net_x<S, 0>), grid, dim3(256), 0, s, d, w, pos, count, max_b, mode, logits, values, stamps);
  }
}

void launch_net_f16x3(const Dev& d, const NetWeights& w, const Pos* pos, const int32_t* count, int max_b, int mode,
                      float* logits_out, float* values_out, hipStream_t s, hipEvent_t ev_begin, hipEvent_t ev_end,
                      int variant) {
  if (!(variant & NET_VAR_X))
    return launch_net_y(d, w, pos, count, max_b, mode, logits_out, values_out, s, ev_begin, ev_end, variant);
  if (max_b <= 0) return;
  if (ev_begin) (void)hipEventRecord(ev_begin, s);
  launch_variant<false>(variant & ~NET_VAR_X, dim3((max_b + XB - 1) / XB), s, d, w, pos, count, max_b, mode,
                        logits_out, values_out, nullptr);
  if (ev_end) (void)hipEventRecord(ev_end, s);
}

void launch_net_f16x3_stamped(const Dev& d, const NetWeights& w, const Pos* pos, int n, float* logits_out,
                              float* values_out, unsigned long long* stamps, hipStream_t s, int variant) {
  if (!(variant & NET_VAR_X)) return launch_net_y_stamped(d, w, pos, n, logits_out, values_out, stamps, s, variant);
  if (n <= 0) return;
  launch_variant<true>(variant & ~NET_VAR_X, dim3((n + XB - 1) / XB), s, d, w, pos, nullptr, n, (int)NET_FULL_LOGITS,
                       logits_out, values_out, stamps);
}

}  // namespace mtaz
