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
#include "legacy_rng.h"

namespace mtaz {
namespace {

using namespace rng;

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

// Action selection after the search (exp/agent.py:110-119) from the root rows k_move_end wrote (row
// length kout).
__global__ __launch_bounds__(64) void k_choose(Dev D, const uint16_t* __restrict__ codes,
                                               const uint32_t* __restrict__ visits, int kout,
                                               int32_t* __restrict__ actions) {
  __shared__ uint32_t s_mt[2][MT_N];
  __shared__ double s_pi[KMAX];
  __shared__ unsigned long long s_u;
  const int g = blockIdx.x, lane = threadIdx.x;
  if (!D.gm.active[g]) return;
  const int k = D.gm.root_k[g];
  if (k <= 0 || k > kout) return;   // (k_move_end flagged it)
  WaveMT mt{s_mt};
  mt.load(D.gm.mt_key + (size_t)g * MT_N, D.gm.mt_pos[g], lane);
  const int idx = wave_choose(mt, visits + (size_t)g * kout, k, (int)(D.gm.root[g].info >> 16), D.pr.tau, s_pi, &s_u,
                              D.pr.err, lane);
  if (lane == 0) actions[g] = idx >= 0 ? codes[(size_t)g * kout + idx] : -1;
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
