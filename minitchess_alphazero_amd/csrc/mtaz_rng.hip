// numpy's legacy RandomState on the device (SURVEY a-14): per-game MT19937
// state in HBM, the Dirichlet root noise of exp/agent.py:82 and the action choice of
// exp/agent.py:114-118, bit-exact with numpy.random.RandomState(seed) per game.
//
//   MT19937       numpy/random/src/mt19937/mt19937.c: mt19937_seed (init_genrand), mt19937_gen (the
//                 twist of 624 words), tempering; the state of game g is key[g*624 .. +624] + pos[g]
//   legacy double (a >> 5) * 2^26 + (b >> 6), / 2^53 (random_sample / legacy_double)
//   gamma(shape < 1)  legacy_standard_gamma's rejection loop: U = double, V = -log(1 - double),
//                 U <= 1 - shape: X = pow(U, 1/shape), accept X <= V; else Y = -log((1 - U)/shape),
//                 X = pow(1 - shape + shape*Y, 1/shape), accept X <= V + Y.  One attempt always takes
//                 exactly 4 words, so a wavefront runs 64 consecutive attempts of one game at once
//                 (lane i takes words 4i .. 4i+3 from the stream position) and keeps, in order, the
//                 accepted ones the game's draws still need; the stream advances to just past the
//                 attempt that produced the last gamma it kept.  log / pow are glibc's (glibc_math.h).
//   dirichlet     RandomState.dirichlet (mtrand.pyx): k gammas, acc = their sum in order,
//                 invacc = 1 / acc, each gamma * invacc
//   choice        RandomState.choice(a, p=pi): cdf = cumsum(p), cdf /= cdf[-1], u = random_sample(),
//                 searchsorted(cdf, u, 'right'); choice(maxima) = randint(0, m): masked rejection on
//                 32-bit words (_bounded_integers, buffered_bounded_masked_uint32)
//
// One wavefront per game.  The game's current 624-word block (A) and the next one (B, twisted on
// demand) sit in LDS; the state is read from HBM at kernel start and written back at its end.
#include "engine.h"

#define MTAZ_GLIBC_FN static __device__ __forceinline__
#define MTAZ_GLIBC_CONST static __device__ const
#include "glibc_math.h"

namespace mtaz {
namespace {

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

__global__ void k_rng_seed(uint32_t* __restrict__ key, int32_t* __restrict__ pos, uint64_t seed_base, int G) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= G) return;
  uint32_t s = (uint32_t)(seed_base + (uint64_t)g);
  uint32_t* k = key + (size_t)g * MT_N;
  for (int i = 0; i < MT_N; ++i) {   // mt19937_seed
    k[i] = s;
    s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
  }
  pos[g] = MT_N;
}

// This move's Dirichlet vectors (exp/agent.py:81-82): sims - root_new draws of size k = the root's
// legal count per active game, in order, at noise[noise_off[g] + j * noise_js[g] + c] (k_select
// reads draw `sim - root_new`).
__global__ __launch_bounds__(64) void k_noise(Dev D) {
  __shared__ uint32_t s_mt[2][MT_N];
  __shared__ double s_g[GAMMA_BUF];
  __shared__ double s_inv[64];
  const int g = blockIdx.x, lane = threadIdx.x;
  if (!D.gm.active[g]) return;
  const int k = D.gm.root_k[g], nd = D.pr.sims - D.gm.root_new[g];
  if (nd <= 0 || k <= 0 || k > KMAX) return;
  WaveMT mt{s_mt};
  mt.load(D.gm.mt_key + (size_t)g * MT_N, D.gm.mt_pos[g], lane);
  wave_dirichlet(mt, D.pr.alpha, k, nd, D.gm.noise + D.gm.noise_off[g], D.gm.noise_js[g], s_g, s_inv, lane);
  mt.store(D.gm.mt_key + (size_t)g * MT_N, D.gm.mt_pos + g, lane);
}

// Action selection after the search (exp/agent.py:110-119): pi = N / N.sum() (exp/policy.py:119-121);
// fullmove < tau: choice(legal, p=pi), else a uniform choice among the maxima of pi.  codes / visits:
// the root rows k_move_end wrote (row length kout).
__global__ __launch_bounds__(64) void k_choose(Dev D, const uint16_t* __restrict__ codes,
                                               const uint32_t* __restrict__ visits, int kout,
                                               int32_t* __restrict__ actions) {
#pragma clang fp contract(off)
  __shared__ uint32_t s_mt[2][MT_N];
  __shared__ double s_pi[KMAX];
  __shared__ unsigned long long s_sum;
  const int g = blockIdx.x, lane = threadIdx.x;
  if (!D.gm.active[g]) return;
  const int k = D.gm.root_k[g];
  if (k <= 0 || k > kout) return;   // (k_move_end flagged it)
  WaveMT mt{s_mt};
  mt.load(D.gm.mt_key + (size_t)g * MT_N, D.gm.mt_pos[g], lane);
  if (lane == 0) s_sum = 0;
  __syncthreads();
  const uint32_t* v = visits + (size_t)g * kout;
  unsigned long long part = 0;
  for (int i = lane; i < k; i += 64) part += v[i];
  atomicAdd(&s_sum, part);   // LDS
  __syncthreads();
  // the visit counts are integers below 2^53: numpy's float sum of them is exact, = the integer sum
  const double sum = (double)s_sum;
  for (int i = lane; i < k; i += 64) s_pi[i] = (double)v[i] / sum;
  mt.reserve(64, lane);   // a choice takes 2 words (p) or 1 per randint rejection
  __syncthreads();
  if (lane == 0) {
    const int fullmove = (int)(D.gm.root[g].info >> 16);
    int idx = 0, w = mt.pos;
    if (fullmove < D.pr.tau) {
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
            atomicOr(D.pr.err, ERR_RNG);
            break;
          }
          r = mt.word(w++) & mask;
        } while (r > rng);
      }
      for (int i = 0; i < k; ++i)
        if (s_pi[i] == mx && r-- == 0) { idx = i; break; }
    }
    actions[g] = idx < k ? codes[(size_t)g * kout + idx] : -1;
    s_sum = (unsigned long long)(w - mt.pos);   // words used
  }
  __syncthreads();
  mt.advance((int)s_sum, lane);
  mt.store(D.gm.mt_key + (size_t)g * MT_N, D.gm.mt_pos + g, lane);
}

// Test entry (mtaz_rng_dirichlet_device): stream s = RandomState(seeds[s]) draws n_vec Dirichlet(alpha
// x ks[s]) vectors into out + offs[s] (row-major) and then one random_sample() into tail[s], so that
// the stream position after the draws is checked too.
__global__ __launch_bounds__(64) void k_rng_dirichlet_test(const uint32_t* __restrict__ seeds, const int32_t* __restrict__ ks,
                                                           const int64_t* __restrict__ offs, int n_vec, double alpha,
                                                           double* __restrict__ out, double* __restrict__ tail,
                                                           uint32_t* __restrict__ scratch) {
  __shared__ uint32_t s_mt[2][MT_N];
  __shared__ double s_g[GAMMA_BUF];
  __shared__ double s_inv[64];
  const int s = blockIdx.x, lane = threadIdx.x;
  uint32_t* key = scratch + (size_t)s * MT_N;
  if (lane == 0) {
    uint32_t x = seeds[s];
    for (int i = 0; i < MT_N; ++i) {
      key[i] = x;
      x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
    }
  }
  __syncthreads();
  WaveMT mt{s_mt};
  mt.load(key, MT_N, lane);
  const int k = ks[s];
  if (k > 0 && k <= KMAX) wave_dirichlet(mt, alpha, k, n_vec, out + offs[s], k, s_g, s_inv, lane);
  mt.reserve(2, lane);
  if (lane == 0) tail[s] = legacy_double_w(mt.word(mt.pos), mt.word(mt.pos + 1));
}

}  // namespace

void launch_rng_seed(const Dev& d, uint64_t seed_base, hipStream_t s) {
  hipLaunchKernelGGL(k_rng_seed, dim3((d.pr.G + 63) / 64), dim3(64), 0, s, d.gm.mt_key, d.gm.mt_pos, seed_base, d.pr.G);
}

void launch_noise(const Dev& d, hipStream_t s) { hipLaunchKernelGGL(k_noise, dim3(d.pr.G), dim3(64), 0, s, d); }

void launch_choose(const Dev& d, const uint16_t* codes, const uint32_t* visits, int kout, int32_t* actions, hipStream_t s) {
  hipLaunchKernelGGL(k_choose, dim3(d.pr.G), dim3(64), 0, s, d, codes, visits, kout, actions);
}

void launch_rng_dirichlet_test(const uint32_t* seeds, const int32_t* ks, const int64_t* offs, int n_streams, int n_vec,
                               double alpha, double* out, double* tail, uint32_t* scratch, hipStream_t s) {
  hipLaunchKernelGGL(k_rng_dirichlet_test, dim3(n_streams), dim3(64), 0, s, seeds, ks, offs, n_vec, alpha, out, tail,
                     scratch);
}

}  // namespace mtaz
