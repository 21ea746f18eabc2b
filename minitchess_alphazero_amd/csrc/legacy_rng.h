// numpy's legacy RandomState for one game per wavefront (device code shared by mtaz_rng.hip and the
// free-running move transitions of mtaz_device.hip; see mtaz_rng.hip for the algorithm notes).
#pragma once
#include "engine.h"

#define MTAZ_GLIBC_FN static __device__ __forceinline__
#define MTAZ_GLIBC_CONST static __device__ const
#include "glibc_math.h"

namespace mtaz {
namespace rng {
namespace {   // internal linkage: included by more than one translation unit

constexpr int MT_N = 624, MT_M = 397;
constexpr uint32_t MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu, MT_MATRIX_A = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t a1, uint32_t x) {
  const uint32_t y = (a & MT_UPPER) | (a1 & MT_LOWER);
  return x ^ (y >> 1) ^ ((0u - (y & 1u)) & MT_MATRIX_A);
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// B = the block mt19937_gen makes from A (lane-parallel in the recurrence's three dependency ranges:
// words [0, 227) read A only, [227, 454) and [454, 623) the new words 227 back, 623 wraps to B[0]).
__device__ void mt_twist(const uint32_t* A, uint32_t* B, int lane) {
  for (int i = lane; i < MT_N - MT_M; i += 64) B[i] = mt_mix(A[i], A[i + 1], A[i + MT_M]);
  __syncthreads();
  for (int i = MT_N - MT_M + lane; i < 2 * (MT_N - MT_M); i += 64) B[i] = mt_mix(A[i], A[i + 1], B[i - (MT_N - MT_M)]);
  __syncthreads();
  for (int i = 2 * (MT_N - MT_M) + lane; i < MT_N - 1; i += 64) B[i] = mt_mix(A[i], A[i + 1], B[i - (MT_N - MT_M)]);
  __syncthreads();
  if (lane == 0) B[MT_N - 1] = mt_mix(A[MT_N - 1], B[0], B[MT_M - 1]);
  __syncthreads();
}

// One game's stream in a wavefront: blocks buf[cur] (the current block, words [0, 624) from it) and
// buf[cur ^ 1] (the next, valid once `next_ok`); pos = the next word's index in the current block.
struct WaveMT {
  uint32_t (*buf)[MT_N];
  int cur, pos;
  bool next_ok;

  __device__ void load(const uint32_t* key, int p, int lane) {
    cur = 0;
    next_ok = false;
    for (int i = lane; i < MT_N; i += 64) buf[0][i] = key[i];
    pos = p;
    __syncthreads();
  }
  // make words [pos, pos + n) available (n <= 624), and the next block whenever an advance of up to
  // n words can reach the end of the current one (an advance to exactly 624 makes the next block
  // current, so it must exist even when no word of it was read)
  __device__ void reserve(int n, int lane) {
    if (pos + n >= MT_N && !next_ok) {
      mt_twist(buf[cur], buf[cur ^ 1], lane);
      next_ok = true;
    }
  }
  __device__ uint32_t word(int idx) const {   // idx relative to the current block, < 2 * 624
    return mt_temper(idx < MT_N ? buf[cur][idx] : buf[cur ^ 1][idx - MT_N]);
  }
  __device__ void advance(int n, int lane) {
    reserve(n, lane);   // (a no-op after the caller's reserve of at least n words)
    pos += n;
    if (pos >= MT_N) {   // the next block becomes current
      pos -= MT_N;
      cur ^= 1;
      next_ok = false;
    }
  }
  __device__ void store(uint32_t* key, int32_t* p, int lane) {
    __syncthreads();
    for (int i = lane; i < MT_N; i += 64) key[i] = buf[cur][i];
    if (lane == 0) *p = pos;
  }
};

__device__ __forceinline__ double legacy_double_w(uint32_t w0, uint32_t w1) {
#pragma clang fp contract(off)
  const int32_t a = (int32_t)(w0 >> 5), b = (int32_t)(w1 >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

constexpr int GAMMA_BUF = 1024;   // gammas per chunk (LDS), >= 4 vectors of KMAX

// n_vec Dirichlet(alpha x k) vectors (alpha < 1) of one game's stream into out[j * js + c].
__device__ void wave_dirichlet(WaveMT& mt, double alpha, int k, int n_vec, double* __restrict__ out, int64_t js,
                               double* s_g, double* s_inv, int lane) {
#pragma clang fp contract(off)
  const double one_m = 1.0 - alpha, inv_shape = 1. / alpha;
  const int J = min(GAMMA_BUF / k, 64);
  for (int j0 = 0; j0 < n_vec; j0 += J) {
    const int nj = min(J, n_vec - j0), need = nj * k;
    int got = 0;
    while (got < need) {
      mt.reserve(256, lane);
      const int w = mt.pos + 4 * lane;
      const double U = legacy_double_w(mt.word(w), mt.word(w + 1));
      const double V = -glibc_log(1.0 - legacy_double_w(mt.word(w + 2), mt.word(w + 3)));
      const bool low = U <= one_m;
      double Y = 0.0, xb = U;
      if (!low) {
        Y = -glibc_log((1 - U) / alpha);
        xb = one_m + alpha * Y;
      }
      const double X = glibc_pow(xb, inv_shape);
      const bool acc = low ? X <= V : X <= (V + Y);
      const uint64_t m = __ballot(acc);
      const int total = __popcll(m), rem = need - got;
      const int rank = __popcll(m & ((1ull << lane) - 1ull));
      int take = total, used = 64;
      if (total >= rem) {
        take = rem;
        used = __ffsll((unsigned long long)__ballot(acc && rank == rem - 1));   // lane of the last kept + 1
      }
      if (acc && rank < take) s_g[got + rank] = X;
      got += take;
      mt.advance(4 * used, lane);
    }
    __syncthreads();
    if (lane < nj) {
      double a = 0.0;
      for (int c = 0; c < k; ++c) a = a + s_g[lane * k + c];
      s_inv[lane] = 1 / a;
    }
    __syncthreads();
    for (int i = lane; i < need; i += 64) {
      const int j = i / k, c = i - j * k;
      out[(int64_t)(j0 + j) * js + c] = s_g[i] * s_inv[j];
    }
    __syncthreads();
  }
}

// Action choice of one game (exp/agent.py:110-119) from its root visit counts v[0..k): pi = N / N.sum()
// (exp/policy.py:119-121); fullmove < tau: RandomState.choice(legal, p=pi) = searchsorted(cdf, u,
// 'right') with cdf = cumsum(pi) / its last element; else a uniform choice among the maxima of pi
// (randint(0, m): masked rejection on 32-bit words).  Returns the chosen index (all lanes), or -1.
// s_pi: KMAX doubles of LDS; s_u: one LDS word.  Called by all 64 lanes.
__device__ int wave_choose(WaveMT& mt, const uint32_t* __restrict__ v, int k, int fullmove, int tau, double* s_pi,
                           unsigned long long* s_u, int32_t* err, int lane) {
#pragma clang fp contract(off)
  if (lane == 0) *s_u = 0;
  __syncthreads();
  unsigned long long part = 0;
  for (int i = lane; i < k; i += 64) part += v[i];
  atomicAdd(s_u, part);   // LDS
  __syncthreads();
  // the visit counts are integers below 2^53: numpy's float sum of them is exact, = the integer sum
  const double sum = (double)*s_u;
  for (int i = lane; i < k; i += 64) s_pi[i] = (double)v[i] / sum;
  mt.reserve(64, lane);   // a choice takes 2 words (p) or 1 per randint rejection
  __syncthreads();
  if (lane == 0) {
    int idx = 0, w = mt.pos;
    if (fullmove < tau) {
      double acc = 0.0;
      for (int i = 0; i < k; ++i) {   // cdf = pi.cumsum() (in place)
        acc = acc + s_pi[i];
        s_pi[i] = acc;
      }
      const double last = s_pi[k - 1];
      const double u = legacy_double_w(mt.word(w), mt.word(w + 1));
      w += 2;
      while (idx < k && s_pi[idx] / last <= u) ++idx;
    } else {
      double mx = s_pi[0];
      for (int i = 1; i < k; ++i) mx = fmax(mx, s_pi[i]);
      int m = 0;
      for (int i = 0; i < k; ++i) m += s_pi[i] == mx;
      const uint32_t rng = (uint32_t)(m - 1);
      uint32_t r = 0;
      if (rng != 0) {
        uint32_t mask = rng;
        mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
        do {
          if (w >= mt.pos + 64) {   // 64 rejections in a row (p < 2^-64): the reserved words ran out
            atomicOr(err, ERR_RNG);
            break;
          }
          r = mt.word(w++) & mask;
        } while (r > rng);
      }
      for (int i = 0; i < k; ++i)
        if (s_pi[i] == mx && r-- == 0) { idx = i; break; }
    }
    *s_u = ((unsigned long long)(w - mt.pos) << 32) | (uint32_t)(idx < k ? idx : -1);   // words used | index
  }
  __syncthreads();
  const unsigned long long r = *s_u;
  mt.advance((int)(r >> 32), lane);
  return (int)(uint32_t)r;
}

}  // namespace
}  // namespace rng
}  // namespace mtaz
