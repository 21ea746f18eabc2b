// Pieces shared by the fused network kernels (k_net_y: fp16x3 on v_mfma_f32_16x16x32_f16,
// mtaz_net16.hip; k_net_z: f16 + e4m3 cross terms, mtaz_net8.hip): the LDS activation image, the
// stem input, and the policy/value heads (exp/policy.py:62-80, exp/agent.py:67-69).
#pragma once
#include "engine.h"

namespace mtaz {
namespace netc {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

constexpr int XB = 4;                     // boards per workgroup
constexpr int IROWS = 31;                 // image rows: squares 0..29 + zero row
constexpr int ZROW = 30;
constexpr int RB = 512;                   // bytes per row: 256 channels x f16
constexpr int PARTB = XB * IROWS * RB;    // 63,488 B per part (hi / lo)
constexpr int IMGB = 2 * PARTB;           // 126,976 B
constexpr int AUXB = XB * 8 * 56 * 4;     // 7,168 B: stem input / head features

// byte offset of 16-B channel chunk `chunk` (8 channels) of image row `row`; the chunk index
// is XOR-swizzled with the row so that a wave's 16-B reads of one chunk over consecutive rows
// land in distinct bank groups
__device__ __forceinline__ int ioff(int part, int bb, int row, int chunk) {
  return part * PARTB + (bb * IROWS + row) * RB + ((chunk ^ (row & 15)) << 4);
}

// k_net_z's image layout.  Per part and board, rows 0..31 x 32 chunks of 16 B, stored chunk-major
// within 16-row halves: (row r, chunk q) at 256 (q + 32 (r >> 4)) + 16 (r & 15).  The bank group
// of a 16-B chunk then depends on its row alone, and a K-loop fragment read (each 16-lane read
// group = the 16 consecutive output squares of a tile, any chunk per lane) touches 16 distinct
// rows: conflict-free.  Off-board taps read a per-lane cell of the board's zero line (after the
// rows), on the bank the on-board source would have had (tools/lds_conflicts.py: 4.0 LDS
// cycles per ds_read_b128 against 6.9 / 7.6 for the row-major swizzled image).  The zero line is
// two chunks wide (512 B), so that an e4m3 fragment's second 16-B read is always its first read's
// address + 256, on-board (the next chunk) or off (the second zero cell).
constexpr int ZROWS_B = 16384;                 // bytes of rows per board and part
constexpr int ZBOARD = ZROWS_B + 512;          // + the zero line
constexpr int ZPART = XB * ZBOARD;             // 67,584 B per part
constexpr int ZIMGB = 2 * ZPART;               // 135,168 B
__device__ __forceinline__ int zrow(int row, int chunk) { return 256 * (chunk + 32 * (row >> 4)) + 16 * (row & 15); }
__device__ __forceinline__ int zoff(int part, int bb, int row, int chunk) {
  return part * ZPART + bb * ZBOARD + zrow(row, chunk);
}
// byte offset within a board of the 16-B chunk `chunk` of the source square of output square p
// (row ph, file pw) for tap (dh, dw), or of p's cell in the zero line when the tap is off-board
__device__ __forceinline__ int zsrc(int p, int ph, int pw, int tap, int chunk) {
  const int dh = tap / 3 - 1, dw = tap - 3 * (tap / 3) - 1;
  const int r = ph + dh, c = pw + dw, s = p + 5 * dh + dw;
  // bitwise, not short-circuit: a select (v_cndmask), not exec-masked branches
  const bool valid = (p < 30) & ((unsigned)r < 6u) & ((unsigned)c < 5u);
  const int on = zrow(s, chunk), off = ZROWS_B + 16 * (s & 15);
  return valid ? on : off;
}

// image row holding the source square of output square `p` (row ph, file pw) for tap
// (dh, dw) = (tap/3 - 1, tap%3 - 1), or the zero row (off-board / padding square)
__device__ __forceinline__ int src_row(int p, int ph, int pw, int tap) {
  const int dh = tap / 3 - 1, dw = tap - 3 * (tap / 3) - 1;
  const int r = ph + dh, c = pw + dw;
  return (p < 30 && r >= 0 && r < 6 && c >= 0 && c < 5) ? p + 5 * dh + dw : ZROW;
}

// piece nibble of square s (rules.h Pos layout) without a dynamically indexed local array
__device__ __forceinline__ int nib_at(const Pos& p, int s) {
  const int w = s >> 3;
  const uint32_t word = w == 0 ? p.sq[0] : w == 1 ? p.sq[1] : w == 2 ? p.sq[2] : p.sq[3];
  return (word >> (4 * (s & 7))) & 15;
}

// encode_clock (rules.h) straight from the packed info word
__device__ __forceinline__ float clock_of(const Pos& p) {
  const double c = (double)(p.info >> 16) + ((p.info & 1u) ? 0.0 : 0.5);
  return (float)(c / 30.0);
}

// Zero the image's zero rows and build the stem input image in `simg` (aux region):
// [part][board][row 31][8 ch f16], channel c = plane*4 + e of Embedding(7,4) applied to the
// own / opponent token planes (exp/policy.py:71-74, encoder exp/environment.py:63-75).
// Caller: __syncthreads() before reading.
template <int NT = 256, bool ZL = false>
__device__ __forceinline__ void stem_input(char* smem, char* simg, const Pos* pos, int b0, int nb,
                                           const NetWeights& W, int tid) {
  if constexpr (ZL) {   // the zero lines
    for (int i = tid; i < 2 * XB * 32; i += NT) {
      const int part = i / (XB * 32), bb = (i / 32) % XB, c = i & 31;
      *reinterpret_cast<uint4*>(smem + part * ZPART + bb * ZBOARD + ZROWS_B + 16 * c) = make_uint4(0, 0, 0, 0);
    }
  } else {
    for (int i = tid; i < 2 * XB * 32; i += NT) {
      const int part = i / (XB * 32), bb = (i / 32) % XB, ch = i & 31;
      *reinterpret_cast<uint4*>(smem + ioff(part, bb, ZROW, ch)) = make_uint4(0, 0, 0, 0);
    }
  }
  for (int i = tid; i < 2 * XB * IROWS; i += NT) *reinterpret_cast<uint4*>(simg + i * 16) = make_uint4(0, 0, 0, 0);
  __syncthreads();
  if (tid < XB * 30) {
    const int bb = tid / 30, i = tid % 30;          // i = square index in the mover's view
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
}

// Heads, part 1 (all NT >= 256 threads of the workgroup): policy conv 256->2 and value conv
// 256->1 (1x1, BN folded, ReLU) from the final image, the clock feature, the value MLP hidden
// layer and its reduction.  Leaves fp [XB][64] (60 policy features + clock), red[bb*256] = value
// pre-tanh.  xscale: the image holds x / xscale (a power of two; k_net_y's dynamic range).
// F8LO (k_net_z's image): part 1 holds e4m3 bytes, the lo part of channel c at byte c of the
// row's first 256 B (16-B chunks swizzled as ioff), board bb's in units of lo_scale[bb] (powers
// of two).
template <int NT = 256, bool F8LO = false, bool ZL = false>
__device__ __forceinline__ void heads_reduce(char* smem, const Pos* pos, int b0, int nb, const NetWeights& W,
                                             int tid, float xscale = 1.f, float4 lo_scale = {1.f, 1.f, 1.f, 1.f}) {
  auto off = [](int part, int bb, int row, int chunk) { return ZL ? zoff(part, bb, row, chunk) : ioff(part, bb, row, chunk); };
  float* fp = reinterpret_cast<float*>(smem + (ZL ? ZIMGB : IMGB));   // [XB][64]: pconv features (60) + clock
  float* fv = fp + XB * 64;                            // [XB][32]: vconv features (30) + clock
  float* red = fv + XB * 32;                           // [XB][256]
  for (int t = tid; t < XB * 90; t += NT) {
    const int bb = t / 90, o = (t % 90) / 30, p = t % 30;
    const float* wr = o < 2 ? W.pconv_w + o * 256 : W.vconv_w;
    float s = 0.f;
    for (int c = 0; c < 32; ++c) {
      const f16x8 xh = *reinterpret_cast<const f16x8*>(smem + off(0, bb, p, c));
      if constexpr (F8LO) {
        const float lsc = bb == 0 ? lo_scale.x : bb == 1 ? lo_scale.y : bb == 2 ? lo_scale.z : lo_scale.w;
        const uint2 q = *reinterpret_cast<const uint2*>(smem + off(1, bb, p, c >> 1) + 8 * (c & 1));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float lo = __builtin_amdgcn_cvt_f32_fp8((int)((j < 4 ? q.x : q.y) >> (8 * (j & 3))), 0) * lsc;
          s += wr[8 * c + j] * ((float)xh[j] + lo);
        }
      } else {
        const f16x8 xl = *reinterpret_cast<const f16x8*>(smem + off(1, bb, p, c));
#pragma unroll
        for (int j = 0; j < 8; ++j) s += wr[8 * c + j] * ((float)xh[j] + (float)xl[j]);
      }
    }
    s = fmaxf(__builtin_fmaf(s, xscale, o < 2 ? W.pconv_b[o] : W.vconv_b[0]), 0.f);
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

// Heads, part 2 (wave bb finishes board bb): value = tanh, then either the full 554 logits
// (evaluate mode) or the leaf priors = softmax over the legal moves' logits in the node's
// legal-list order (exp/agent.py:67-69), written to D.lf.
template <bool ZL = false>
__device__ __forceinline__ void heads_out(const Dev& D, char* smem, int b0, int nb, const NetWeights& W, int mode,
                                          float* logits_out, float* values_out, int wave, int lane) {
  const float* fp = reinterpret_cast<const float*>(smem + (ZL ? ZIMGB : IMGB));
  const float* red = fp + XB * 64 + XB * 32;
  if (wave >= XB) return;
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
  const NodeHdr hd = D.tr.node_hdr[(size_t)t * D.tr.NC + n];
  const int k = hdr_k(hd);
  const uint32_t e0 = hd.e0;
  const uint16_t* codes = D.tr.e_code + e0;
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

}  // namespace netc
}  // namespace mtaz
