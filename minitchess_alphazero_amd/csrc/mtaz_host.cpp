// Host side of the mtaz engine: the C ABI of include/mtaz.h.
//
//   * codec loader        exp/moves_dict.json format (exp/environment.py:15-20)
//   * host rules / FEN    single-position MinitChessEpisode support (exp/environment.py:22-85)
//   * numpy legacy RNG    MT19937 + legacy gamma / dirichlet / choice, bit-exact with
//                         numpy.random.RandomState (exp/agent.py:82,115,118); compiled
//                         without FP contraction and calling the same libm log/pow
//   * engine              HBM allocation, BN folding + MFMA weight swizzle, and the
//                         batched self-play driver that replaces erlyx.run_episodes
//                         under SimulatePuppet.run_episodes (app/base.py:108-124)
#pragma STDC FP_CONTRACT OFF
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <sched.h>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/mtaz.h"
#include "engine.h"

using namespace mtaz;

// ---------------------------------------------------------------------------------------
// errors
static thread_local std::string g_err;
static int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}
#define HIPCHK(x)                                                                            \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) return set_err(MTAZ_E_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

extern "C" int mtaz_abi_version(void) { return MTAZ_ABI_VERSION; }
#ifndef MTAZ_SRC_SHA256
#define MTAZ_SRC_SHA256 "unknown"
#endif
// the build fingerprint (build.py source_hash: csrc/*, include/mtaz.h, compile flags)
extern "C" const char* mtaz_version(void) { return "mtaz 0.3 (gfx950) mtaz-src-sha256=" MTAZ_SRC_SHA256; }
extern "C" const char* mtaz_last_error(void) { return g_err.c_str(); }

// ---------------------------------------------------------------------------------------
// codec
static Codec h_codec;
static bool h_codec_ok = false;

static int sq_from_name(const char* s) {
  if (s[0] < 'a' || s[0] > 'e' || s[1] < '1' || s[1] > '6') return -1;
  return (s[1] - '1') * 5 + (s[0] - 'a');
}

// Parses {"w": {"a1b2": 0, ...}, "b": {...}} (json.dump default formatting, or any
// whitespace).  Every code must appear exactly once per side.
extern "C" int mtaz_load_codec(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return set_err(MTAZ_E_FAIL, "cannot open %s", path);
  std::string s;
  char buf[4096];
  size_t r;
  while ((r = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, r);
  fclose(f);
  Codec c;
  memset(c.enc, 0xff, sizeof(c.enc));
  memset(c.dec, 0xff, sizeof(c.dec));
  int side = -1, seen[2] = {0, 0};
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] != '"') { ++i; continue; }
    const size_t j = s.find('"', i + 1);
    if (j == std::string::npos) break;
    const std::string key = s.substr(i + 1, j - i - 1);
    i = j + 1;
    if (key == "w" || key == "b") { side = key == "w" ? 0 : 1; continue; }
    if (key.size() != 4 || side < 0) return set_err(MTAZ_E_FAIL, "codec: unexpected key '%s'", key.c_str());
    while (i < s.size() && (s[i] == ':' || s[i] == ' ')) ++i;
    int code = 0, nd = 0;
    while (i < s.size() && s[i] >= '0' && s[i] <= '9') { code = code * 10 + (s[i] - '0'); ++i; ++nd; }
    const int from = sq_from_name(key.c_str()), to = sq_from_name(key.c_str() + 2);
    if (!nd || from < 0 || to < 0 || code >= NUM_ACTIONS) return set_err(MTAZ_E_FAIL, "codec: bad entry '%s'", key.c_str());
    if (c.dec[side][code] != 0xffff) return set_err(MTAZ_E_FAIL, "codec: duplicate code %d", code);
    c.enc[side][from * 30 + to] = (int16_t)code;
    c.dec[side][code] = (uint16_t)(from | (to << 8));
    ++seen[side];
  }
  if (seen[0] != NUM_ACTIONS || seen[1] != NUM_ACTIONS)
    return set_err(MTAZ_E_FAIL, "codec: expected %d codes per side, got %d/%d", NUM_ACTIONS, seen[0], seen[1]);
  h_codec = c;
  h_codec_ok = true;
  return 0;
}

static int ensure_codec_device(int device) {
  if (!h_codec_ok) return set_err(MTAZ_E_FAIL, "codec not loaded (mtaz_load_codec)");
  HIPCHK(hipSetDevice(device));
  if (dev_upload_codec(h_codec)) return set_err(MTAZ_E_DEVICE, "codec upload failed");
  return 0;
}

// ---------------------------------------------------------------------------------------
// host rules
static inline Pos pos_in(const uint32_t* p) { Pos x; memcpy(&x, p, sizeof(Pos)); return x; }
static inline void pos_out(const Pos& x, uint32_t* p) { memcpy(p, &x, sizeof(Pos)); }

static int host_legal(const BB& b, uint32_t flags, uint16_t* out, int cap) {
  const uint32_t own = b.white ? b.w : b.b;
  const int side = b.white ? 0 : 1;
  int k = 0;
  uint32_t m = own;
  while (m) {
    const int s = lsb(m);
    m &= m - 1;
    uint32_t tg = legal_targets(b, s, flags);
    while (tg) {
      const int to = lsb(tg);
      tg &= tg - 1;
      const int code = h_codec.enc[side][s * 30 + to];
      const int mult = move_mult(b, s, to, flags);
      for (int r = 0; r < mult; ++r) {
        if (k >= cap) return -1;
        out[k++] = (uint16_t)code;
      }
    }
  }
  std::sort(out, out + k);
  return k;
}

static const char* PIECES = ".pnbrqk";

extern "C" int mtaz_pos_from_fen(const char* fen, uint32_t out[5]) {
  BB b{};
  int r = 5, f = 0;
  const char* p = fen;
  for (; *p && *p != ' '; ++p) {
    const char ch = *p;
    if (ch == '/') {
      if (f != 5) return set_err(MTAZ_E_FAIL, "bad FEN rank in '%s'", fen);
      --r; f = 0;
      if (r < 0) return set_err(MTAZ_E_FAIL, "too many ranks in '%s'", fen);
    } else if (ch >= '1' && ch <= '5') {
      f += ch - '0';
    } else {
      const char lc = (ch >= 'A' && ch <= 'Z') ? ch - 'A' + 'a' : ch;
      const char* q = strchr(PIECES + 1, lc);
      if (!q || f >= 5) return set_err(MTAZ_E_FAIL, "bad FEN piece in '%s'", fen);
      set_piece(b, r * 5 + f, (int)(q - PIECES), ch >= 'A' && ch <= 'Z');
      ++f;
    }
    if (f > 5) return set_err(MTAZ_E_FAIL, "bad FEN rank in '%s'", fen);
  }
  if (r != 0 || f != 5) return set_err(MTAZ_E_FAIL, "FEN must have 6 ranks of 5 files: '%s'", fen);
  char turn = 0;
  int half = -1, full = -1;
  if (sscanf(p, " %c %d %d", &turn, &half, &full) != 3 || (turn != 'w' && turn != 'b') || half < 0 || full < 0 ||
      half > 255 || full > 65535)
    return set_err(MTAZ_E_FAIL, "expected 4-field MinitChess FEN 'board turn half full': '%s'", fen);
  b.white = turn == 'w';
  b.half = half;
  b.full = full;
  pos_out(pack(b), out);
  return 0;
}

extern "C" int mtaz_pos_to_fen(const uint32_t pos[5], char* buf, int cap) {
  const BB b = unpack(pos_in(pos));
  std::string s;
  for (int r = 5; r >= 0; --r) {
    int e = 0;
    for (int f = 0; f < 5; ++f) {
      const int sq = r * 5 + f, t = piece_type_at(b, sq);
      if (!t) { ++e; continue; }
      if (e) { s += (char)('0' + e); e = 0; }
      char ch = PIECES[t];
      if ((b.w >> sq) & 1u) ch = ch - 'a' + 'A';
      s += ch;
    }
    if (e) s += (char)('0' + e);
    if (r) s += '/';
  }
  s += b.white ? " w " : " b ";
  s += std::to_string(b.half) + " " + std::to_string(b.full);
  if ((int)s.size() + 1 > cap) return set_err(MTAZ_E_CAPACITY, "fen buffer too small");
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

extern "C" int mtaz_pos_legal(const uint32_t pos[5], uint32_t flags, uint16_t* codes, int cap) {
  if (!h_codec_ok) return set_err(MTAZ_E_FAIL, "codec not loaded");
  const int k = host_legal(unpack(pos_in(pos)), flags, codes, cap);
  return k < 0 ? set_err(MTAZ_E_CAPACITY, "legal list longer than %d", cap) : k;
}

extern "C" int mtaz_pos_outcome(const uint32_t pos[5], uint32_t flags, int move_cap, int reps) {
  if (!h_codec_ok) return set_err(MTAZ_E_FAIL, "codec not loaded");
  const BB b = unpack(pos_in(pos));
  uint16_t tmp[KMAX];
  const int k = host_legal(b, flags, tmp, KMAX);
  if (k < 0) return set_err(MTAZ_E_CAPACITY, "legal list too long");
  return outcome(b, k, in_check(b), flags, move_cap, reps);
}

static int host_decode(const BB& b, int code, int* from, int* to) {
  if (code < 0 || code >= NUM_ACTIONS) return -1;
  const uint16_t ft = h_codec.dec[b.white ? 0 : 1][code];
  *from = ft & 0xff;
  *to = ft >> 8;
  return 0;
}

extern "C" int mtaz_pos_step(const uint32_t pos[5], int code, uint32_t flags, uint32_t out[5]) {
  if (!h_codec_ok) return set_err(MTAZ_E_FAIL, "codec not loaded");
  const BB b = unpack(pos_in(pos));
  int from, to;
  if (host_decode(b, code, &from, &to)) return set_err(MTAZ_E_ILLEGAL, "action %d out of range", code);
  const uint32_t own = b.white ? b.w : b.b;
  if (!((own >> from) & 1u) || !((legal_targets(b, from, flags) >> to) & 1u))
    return set_err(MTAZ_E_ILLEGAL, "action %d is not legal", code);
  const int promo = (((b.pawn >> from) & 1u) && (to / 5 == (b.white ? 5 : 0))) ? QUEEN : 0;
  pos_out(pack(make_move(b, from, to, promo)), out);
  return 0;
}

extern "C" int mtaz_pos_zeroing(const uint32_t pos[5], int code) {
  const BB b = unpack(pos_in(pos));
  int from, to;
  if (host_decode(b, code, &from, &to)) return set_err(MTAZ_E_ILLEGAL, "action out of range");
  return is_zeroing(b, from, to) ? 1 : 0;
}

extern "C" int mtaz_pos_encode(const uint32_t pos[5], uint8_t tokens[60], float* clock) {
  const BB b = unpack(pos_in(pos));
  encode_tokens(b, tokens);
  *clock = encode_clock(b);
  return 0;
}

// ---------------------------------------------------------------------------------------
// numpy legacy RandomState (numpy/random/src/mt19937, src/legacy/legacy-distributions.c,
// mtrand.pyx dirichlet / choice / randint).  One state per game.
namespace {
struct MTState {
  uint32_t key[624];
  int pos;
  int has_gauss;
  double gauss;
};

void mt_seed(MTState& s, uint32_t seed) {
  for (int i = 0; i < 624; ++i) {
    s.key[i] = seed;
    seed = 1812433253u * (seed ^ (seed >> 30)) + (uint32_t)(i + 1);
  }
  s.pos = 624;
  s.has_gauss = 0;
  s.gauss = 0.0;
}

void mt_gen(MTState& s) {
  const uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATRIX_A = 0x9908b0dfu;
  int i;
  uint32_t y;
  for (i = 0; i < 624 - 397; ++i) {
    y = (s.key[i] & UPPER) | (s.key[i + 1] & LOWER);
    s.key[i] = s.key[i + 397] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
  }
  for (; i < 623; ++i) {
    y = (s.key[i] & UPPER) | (s.key[i + 1] & LOWER);
    s.key[i] = s.key[i + (397 - 624)] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
  }
  y = (s.key[623] & UPPER) | (s.key[0] & LOWER);
  s.key[623] = s.key[396] ^ (y >> 1) ^ (-(y & 1u) & MATRIX_A);
  s.pos = 0;
}

inline uint32_t mt_next(MTState& s) {
  if (s.pos == 624) mt_gen(s);
  uint32_t y = s.key[s.pos++];
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

inline double legacy_double(MTState& s) {
  const int32_t a = mt_next(s) >> 5;
  const int32_t b = mt_next(s) >> 6;
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

double legacy_gauss(MTState& s) {
  if (s.has_gauss) {
    const double t = s.gauss;
    s.has_gauss = 0;
    s.gauss = 0.0;
    return t;
  }
  double f, x1, x2, r2;
  do {
    x1 = 2.0 * legacy_double(s) - 1.0;
    x2 = 2.0 * legacy_double(s) - 1.0;
    r2 = x1 * x1 + x2 * x2;
  } while (r2 >= 1.0 || r2 == 0.0);
  f = sqrt(-2.0 * log(r2) / r2);
  s.gauss = f * x1;
  s.has_gauss = 1;
  return f * x2;
}

inline double legacy_exponential(MTState& s) { return -log(1.0 - legacy_double(s)); }

double legacy_gamma(MTState& s, double shape) {
  if (shape == 1.0) return legacy_exponential(s);
  if (shape == 0.0) return 0.0;
  if (shape < 1.0) {
    for (;;) {
      const double U = legacy_double(s);
      const double V = legacy_exponential(s);
      if (U <= 1.0 - shape) {
        const double X = pow(U, 1. / shape);
        if (X <= V) return X;
      } else {
        const double Y = -log((1 - U) / shape);
        const double X = pow(1.0 - shape + shape * Y, 1. / shape);
        if (X <= (V + Y)) return X;
      }
    }
  }
  const double b = shape - 1. / 3.;
  const double c = 1. / sqrt(9 * b);
  for (;;) {
    double X, V;
    do {
      X = legacy_gauss(s);
      V = 1.0 + c * X;
    } while (V <= 0.0);
    V = V * V * V;
    const double U = legacy_double(s);
    if (U < 1.0 - 0.0331 * (X * X) * (X * X)) return b * V;
    if (log(U) < 0.5 * X * X + b * (1. - V + log(V))) return b * V;
  }
}

void legacy_dirichlet(MTState& s, double alpha, int k, double* out) {
  double acc = 0.0;
  for (int j = 0; j < k; ++j) {
    out[j] = legacy_gamma(s, alpha);
    acc = acc + out[j];
  }
  const double invacc = 1 / acc;
  for (int j = 0; j < k; ++j) out[j] = out[j] * invacc;
}

int64_t legacy_choice_p(MTState& s, const double* p, int k) {
  // cdf = p.cumsum(); cdf /= cdf[-1]; searchsorted(random_sample(), side='right')
  double cdf[KMAX];
  double acc = 0.0;
  for (int i = 0; i < k; ++i) { acc = acc + p[i]; cdf[i] = acc; }
  const double last = cdf[k - 1];
  for (int i = 0; i < k; ++i) cdf[i] = cdf[i] / last;
  const double u = legacy_double(s);
  int64_t idx = 0;
  while (idx < k && cdf[idx] <= u) ++idx;
  return idx;
}

int64_t legacy_randint(MTState& s, int64_t m) {
  // randint(0, m): rng = m - 1, masked rejection on 32-bit draws; rng == 0 draws nothing
  const uint64_t rng = (uint64_t)(m - 1);
  if (rng == 0) return 0;
  uint64_t mask = rng;
  mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
  if (rng == 0xffffffffull) return mt_next(s);
  uint32_t v;
  while ((v = (mt_next(s) & (uint32_t)mask)) > rng) {
  }
  return v;
}
}  // namespace

extern "C" size_t mtaz_rng_state_size(void) { return sizeof(MTState); }
extern "C" void mtaz_rng_seed(void* st, uint32_t seed) { mt_seed(*(MTState*)st, seed); }
extern "C" double mtaz_rng_double(void* st) { return legacy_double(*(MTState*)st); }
extern "C" void mtaz_rng_dirichlet(void* st, double alpha, int k, double* out) { legacy_dirichlet(*(MTState*)st, alpha, k, out); }
extern "C" int64_t mtaz_rng_choice_p(void* st, const double* p, int k) {
  if (k <= 0 || k > KMAX) return set_err(MTAZ_E_CAPACITY, "choice size %d", k);
  return legacy_choice_p(*(MTState*)st, p, k);
}
extern "C" int64_t mtaz_rng_randint(void* st, int64_t m) { return legacy_randint(*(MTState*)st, m); }

// ---------------------------------------------------------------------------------------
// batched rules kernels
extern "C" int mtaz_legal_batch(int device, const uint32_t* d_pos, int n, uint32_t flags, int move_cap, uint16_t* d_codes,
                                int32_t* d_counts, uint32_t* d_masks, int32_t* d_outcomes, void* stream) {
  if (int e = ensure_codec_device(device)) return e;
  launch_legal_batch(reinterpret_cast<const Pos*>(d_pos), n, flags, move_cap, d_codes, d_counts, d_masks, d_outcomes,
                     (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

extern "C" int mtaz_replay_put(int device, int n, const uint32_t* d_pos, const int32_t* d_k, const int64_t* d_e0,
                               const uint16_t* d_codes, const uint32_t* d_visits, const float* d_reward, int64_t cap,
                               int64_t head, uint8_t* d_tokens, float* d_clocks, float* d_pi, float* d_reward_out,
                               void* stream) {
  if (n < 0 || cap <= 0 || head < 0 || n > cap) return set_err(MTAZ_E_FAIL, "replay_put: bad n/cap/head");
  HIPCHK(hipSetDevice(device));
  launch_replay_put(reinterpret_cast<const Pos*>(d_pos), d_k, d_e0, d_codes, d_visits, d_reward, n, cap, head, d_tokens,
                    d_clocks, d_pi, d_reward_out, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int mtaz_encode_batch(int device, const uint32_t* d_pos, int n, uint8_t* d_tokens, float* d_clocks, void* stream) {
  HIPCHK(hipSetDevice(device));
  launch_encode_batch(reinterpret_cast<const Pos*>(d_pos), n, d_tokens, d_clocks, (hipStream_t)stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize((hipStream_t)stream));
  return 0;
}

// ---------------------------------------------------------------------------------------
// engine
namespace {
// One game's InfoRecorder records (exp/callbacks.py:40-47): per ply the observation, the action
// and its legal list length; the legal codes and root visit counts of all plies concatenated
// (no allocation per ply: the vectors keep their capacity across plays).
struct GameRec {
  std::vector<Pos> pos;
  std::vector<int32_t> action, k;
  std::vector<uint16_t> codes;
  std::vector<uint32_t> visits;
  size_t plies() const { return pos.size(); }
  void clear() {
    pos.clear();
    action.clear();
    k.clear();
    codes.clear();
    visits.clear();
  }
  void add(const Pos& p, int32_t a, const uint16_t* c, const uint32_t* v, int kk) {
    pos.push_back(p);
    action.push_back(a);
    k.push_back(kk);
    codes.insert(codes.end(), c, c + kk);
    visits.insert(visits.end(), v, v + kk);
  }
};

enum Stat {
  ST_PLIES, ST_SIMS, ST_NN_EVALS, ST_TERMINAL_SIMS, ST_TRUNK_MS, ST_TRUNK_BOARDS, ST_WAVES, ST_HOST_RNG_MS,
  ST_WALL_MS, ST_GAMES, ST_DECISIVE, ST_MOVES, ST_TRUNK_LAUNCHES, ST_MAX_NODES, ST_MAX_EDGES, ST_SYNC_MS, ST_NET_PREC, ST_SELECT_MS,
  ST_NODE_CAP, ST_EDGE_CAP, ST_COMPACT_MS, ST_MEMO_HITS, ST_POOL_EDGES, ST_POOL_CAP, ST_MEMO_BATCH_HITS, ST_CHOICE_MS, ST_GAP_MS, ST_EXTRA_WAVES,
  ST_RNG_DEVICE, ST_RNG_DEV_MS, ST_SCHEDULE, ST_COUNT
};

// Host worker pool for the per-move work (Dirichlet draws, action choice): one pool per calling
// thread (the main thread, or each stream group's thread), created on first use and joined when
// that thread exits, so a move does not pay for starting threads.  Workers 1..nt-1 take equal
// contiguous ranges; the calling thread runs range 0.
class HostPool {
 public:
  explicit HostPool(int nt) : nt_(nt) {
    for (int t = 1; t < nt_; ++t) th_.emplace_back([this, t] { worker(t); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& x : th_) x.join();
  }
  int size() const { return nt_; }
  void run(int n, const std::function<void(int)>& f) {
    const int chunk = (n + nt_ - 1) / nt_;
    {
      std::lock_guard<std::mutex> lk(m_);
      job_ = &f;
      n_ = n;
      chunk_ = chunk;
      pending_ = nt_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    for (int i = 0; i < std::min(n, chunk); ++i) f(i);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void worker(int t) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int)>* f;
      int a, b;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = job_;
        a = t * chunk_;
        b = std::min(n_, a + chunk_);
      }
      for (int i = a; i < b; ++i) (*f)(i);
      {
        std::lock_guard<std::mutex> lk(m_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  int nt_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* job_ = nullptr;
  int n_ = 0, chunk_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// The host threads this process may use: the CPUs of its affinity mask (not the machine's count:
// one rank per GPU runs on its own slice of the host, launch.py / bench.py pin them), at most 16.
int default_host_threads() {
  cpu_set_t cs;
  int n = 0;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
  if (n <= 0) n = (int)std::thread::hardware_concurrency();
  return std::max(1, std::min(n, 16));
}

// One pool per calling thread (the main thread, or each stream group's thread) for every
// parallel_for, rebuilt only when the requested size changes.
HostPool* host_pool(int nt) {
  thread_local std::unique_ptr<HostPool> pool;
  if (!pool || pool->size() != nt) pool.reset(new HostPool(nt));
  return pool.get();
}

template <class F>
void parallel_for(int n, int nt, F f) {
  if (n < 64 || nt <= 1) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  const std::function<void(int)> fn = [&f](int i) { f(i); };
  host_pool(nt)->run(n, fn);
}

double now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}
}  // namespace

// round to the nearest OCP e4m3fn value, ties to even (bias 7, subnormal step 2^-9; the
// callers keep |v| < 448, larger magnitudes saturate to 448)
static uint8_t to_e4m3(double v) {
  const uint8_t sgn = v < 0 ? 0x80 : 0;
  const double a = fabs(v);
  if (a == 0) return sgn;
  int e = ilogb(a);
  if (e < -6) return sgn | (uint8_t)nearbyint(a * 512.0);   // 8 (= 0x08) is the least normal, 2^-6
  double m = nearbyint(ldexp(a, 3 - e));                    // [8, 16]
  if (m == 16) {
    m = 8;
    ++e;
  }
  if (e + 7 > 15 || (e + 7 == 15 && m - 8 >= 7)) return sgn | 0x7e;
  return sgn | (uint8_t)(((e + 7) << 3) | (int)(m - 8));
}

// e2m3 (fp6: 1 sign, 2 exponent bits with bias 1, 3 mantissa bits) code of v, |v| <= 7.5, round
// to nearest even: e4m3's grid below 2^-3 is e2m3's grid scaled by 2^-6, so round there
static uint8_t to_e2m3(double v) {
  const uint8_t b = to_e4m3(ldexp(v, -6));
  return (uint8_t)((b & 0x1f) | ((b & 0x80) >> 2));
}

struct mtaz_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  int G = 0, sims = 0, tau = 6, cast_mode = 2, move_cap = 30;
  double cpuct = 1.0, alpha = 0.6, eps = 0.25;
  uint64_t seed_base = 0;
  uint32_t flags = RF_DEFAULT;
  Dev d{};
  NetWeights w{};
  NetBuffers nb{};
  bool weights_ok = false;
  // k_net_y (fp16x3, fp32-accurate to ~1e-8): within the north_star's 1e-5 on every tested net,
  // the round-3 stress checkpoint included; NET_F16F8 = k_net_z (e4m3 cross terms) is not within
  // 1e-5 there (tests/test_gpu_stress.py), so it is an option, not the default
  int precision = NET_F16X3;
  int variant = 0;   // network kernel variant of the current precision (0 = product; mtaz_set_net_variant)
  uint4* wxbuf = nullptr;
  float* wxinv = nullptr;
  float* wyrange = nullptr;
  std::vector<void*> allocs;
  std::vector<void*> edge_allocs;       // the edge arrays (alloc_edges; mtaz_set_edge_capacity replaces them)
  std::vector<void*> memo_allocs;       // the batch memo (ensure_batch_memo)
  float* wbuf = nullptr;
  // scratch
  int32_t* d_actions = nullptr;
  uint16_t* d_root_codes = nullptr;
  uint32_t* d_root_visits = nullptr;
  uint16_t* d_leaf_codes = nullptr;
  int32_t* d_leaf_k = nullptr;
  int32_t* d_trees = nullptr;
  int32_t* d_count_log = nullptr;
  double* d_sqrt = nullptr;
  int count_log_cap = 0;
  bool last_play_grouped = false;       // the last mtaz_play ran in pipeline groups (mtaz_wave_log)
  size_t noise_cap = 0;
  double* noise_host = nullptr;         // pinned staging of mtaz_play's draw-major noise
  size_t noise_host_cap = 0;
  // pinned staging of mtaz_play's per-move transfers (ensure_play_pinned) and of check_err's flag
  // word: copies to and from pageable memory are staged and synchronous, one round trip each
  // (round 5a: ~13 of them per move, 20-40 us apart in the trace)
  struct PlayPinned {
    uint32_t* roots[2] = {nullptr, nullptr};   // double-buffered: the next move's states arrive
    uint8_t* active[2] = {nullptr, nullptr};   // while the host still reads this move's
    int32_t *agents = nullptr, *outcome = nullptr, *root_k = nullptr, *root_new = nullptr, *actions = nullptr;
    int32_t* js = nullptr;
    int64_t* offs = nullptr;
    uint16_t* codes = nullptr;
    uint32_t* visits = nullptr;
  } pin;
  void* pin_block = nullptr;
  int32_t* err_host = nullptr;
  std::vector<int32_t> last_root_k;     // root legal counts of the last mtaz_move_begin
  std::vector<MTState> rng;
  std::vector<GameRec> rec;
  std::vector<int32_t> final_outcome;
  int n_played = 0;
  double stats[ST_COUNT] = {0};
  bool timing = false;
  std::vector<hipEvent_t> ev;
  int wave = 0;
  int groups = 1;                       // mtaz_set_pipeline
  std::vector<mtaz_engine*> parts;      // per-group engines (borrow this engine's weights)
  std::unique_ptr<HostPool> group_pool; // one persistent host thread per group (play_groups)
  // two-network play (arena, exp/learner.py:97-145): weight slot 0 / 1; the active slot's
  // buffers are the fields above (w, wbuf, wxbuf, wxinv, wyrange, weights_ok), the other
  // slot's are parked here; agent_slot maps agent 0 (first mover) / agent 1 to a slot
  struct Parked {
    NetWeights w{};
    float* wbuf = nullptr;
    uint4* wxbuf = nullptr;
    float* wxinv = nullptr;
    float* wyrange = nullptr;
    bool ok = false;
  } parked;
  int cur_slot = 0;
  int agent_slot[2] = {0, 0};
  int memo = 1;                         // leaf memo mode (mtaz_set_memo; Params::memo)
  int host_threads = default_host_threads();   // per-move host work (mtaz_set_host_threads)
  // how the host thread waits for its stream (mtaz_set_sync_mode): 0 = hipStreamSynchronize (HIP's
  // default wait), 1 = an event created with hipEventBlockingSync (the thread sleeps until the GPU
  // signals, leaving its CPU to the other ranks' host work)
  int sync_mode = 0;
  hipEvent_t sync_ev = nullptr;
  // deferred tails (mtaz_set_defer): in mtaz_play each wave evaluates only the whole rounds of
  // 4 boards x ncu leaves; the rest wait for the next wave (Games::simc, k_leaf_compact).  2 (the
  // default since round 6's leaf order): every remainder waits; 1: the remainders a tail launch would
  // take wait, a larger one runs as a partial round
  int defer = 2;
  int ncu = 0;
  int32_t* d_remaining = nullptr;
  // mtaz_play's numpy-legacy RNG (mtaz_set_rng_device): 1 (the default) = per-game MT19937 state in
  // HBM, Dirichlet draws (k_noise) and action choice (k_choose) on the device; 0 = the host C++ RNG
  // (h->rng), drawn in chunks that overlap the simulations.  The device path needs dir_alpha < 1
  // (the reference's 0.6: every gamma attempt then takes 4 words); other alphas use the host
  int rng_device = 1;
  hipEvent_t rng_ev[4] = {nullptr, nullptr, nullptr, nullptr};   // [noise begin, end, choose begin, end]
  // mtaz_play's schedule (mtaz_set_schedule): 0 (default) = moves in lockstep (every game's move ends
  // with the same wave, host hand-offs per move); 1 = free-running moves: a game that completes a move
  // finishes it and starts the next on the device (k_turn) within the wave loop, so no game waits for
  // the others' moves and the host syncs only every few waves.  Identical games; measured 1.5% slower
  // on the bench workload, hence not the default.  Free-running needs the
  // device RNG and one network for both agents; otherwise mtaz_play runs lockstep.
  int schedule = 0;
  std::vector<hipEvent_t> ev_turn;      // per free-running wave: [k_turn begin, end]
  int32_t* cnt_host = nullptr;          // pinned: the active-game count of free-running play
  int64_t* d_rec_off = nullptr;
  uint16_t* d_pack_codes = nullptr;     // the packed records of a free-running play (grown)
  uint32_t* d_pack_visits = nullptr;
  size_t pack_cap = 0;

  ~mtaz_engine() {
    group_pool.reset();
    if (sync_ev) (void)hipEventDestroy(sync_ev);
    for (mtaz_engine* p : parts) delete p;
    if (device >= 0) (void)hipSetDevice(device);
    if (noise_host) (void)hipHostFree(noise_host);
    for (auto e : rng_ev)
      if (e) (void)hipEventDestroy(e);
    for (auto e : ev_turn) (void)hipEventDestroy(e);
    if (cnt_host) (void)hipHostFree(cnt_host);
    if (d_pack_codes) (void)hipFree(d_pack_codes);
    if (d_pack_visits) (void)hipFree(d_pack_visits);
    if (pin_block) (void)hipHostFree(pin_block);
    if (err_host) (void)hipHostFree(err_host);
    for (auto e : ev) (void)hipEventDestroy(e);
    for (void* p : allocs) (void)hipFree(p);
    for (void* p : edge_allocs) (void)hipFree(p);
    for (void* p : memo_allocs) (void)hipFree(p);
    if (d.gm.noise) (void)hipFree(d.gm.noise);
    if (stream) (void)hipStreamDestroy(stream);
  }

  template <class T>
  int dalloc(T** p, size_t n) {
    void* q = nullptr;
    const size_t bytes = std::max<size_t>(n * sizeof(T), 16);
    HIPCHK(hipMalloc(&q, bytes));
    allocs.push_back(q);
    *p = (T*)q;
    return 0;
  }
};

#define ECHK(x)            \
  do {                     \
    int e_ = (x);          \
    if (e_ < 0) return e_; \
  } while (0)

// Edge arrays: T regions of `ec` edges (one per tree) followed by a shared pool of `pool` edges
// (Trees).  Edge indices are u32, so T * ec + pool must stay below 2^32.
static int alloc_edges(mtaz_engine* h, int64_t ec, int64_t pool) {
  Trees& tr = h->d.tr;
  const int64_t T = 2 * (int64_t)h->G;
  if (ec < 1 || pool < 0 || T * ec + pool >= (int64_t)NONE)
    return set_err(MTAZ_E_CAPACITY, "edge capacity %lld per tree x %lld trees + pool %lld exceeds 32-bit edge indices",
                   (long long)ec, (long long)T, (long long)pool);
  for (void* p : h->edge_allocs) (void)hipFree(p);
  h->edge_allocs.clear();
  const size_t TE = (size_t)(T * ec + pool);
  auto grab = [&](auto** p, size_t elt) -> int {
    void* q = nullptr;
    HIPCHK(hipMalloc(&q, std::max<size_t>(TE * elt, 16)));
    h->edge_allocs.push_back(q);
    *p = (std::remove_reference_t<decltype(*p)>)q;
    return 0;
  };
  ECHK(grab(&tr.e_code, 2));
  ECHK(grab(&tr.e_P, 4));
  ECHK(grab(&tr.e_Q, 8));
  ECHK(grab(&tr.e_N, 4));
  ECHK(grab(&tr.e_child, 4));
  tr.EC = (int)ec;
  tr.pool_base = (uint32_t)(T * ec);
  tr.pool_cap = (uint32_t)pool;
  HIPCHK(hipMemset(tr.pool_used, 0, 4));
  HIPCHK(hipMemset(tr.n_edges, 0, T * 4));
  return 0;
}

// the device buffer of a move's Dirichlet draws, grown geometrically (the old buffer is freed:
// callers have synchronised the stream, nothing reads it any more)
static int ensure_noise(mtaz_engine* h, size_t n) {
  if (n <= h->noise_cap && h->d.gm.noise) return 0;
  const size_t cap = std::max(n, 2 * h->noise_cap);
  if (h->d.gm.noise) HIPCHK(hipFree(h->d.gm.noise));
  h->d.gm.noise = nullptr;
  h->noise_cap = 0;
  HIPCHK(hipMalloc(&h->d.gm.noise, cap * 8));
  h->noise_cap = cap;
  return 0;
}

static int engine_alloc(mtaz_engine* h) {
  const int G = h->G, T = 2 * G;
  Trees& tr = h->d.tr;
  Games& gm = h->d.gm;
  Leaves& lf = h->d.lf;
  const int max_moves = h->move_cap > 0 ? h->move_cap : 200;     // searches per agent per game
  tr.NC = h->sims * max_moves + 2;
  int hc = 1;
  while (hc < 2 * tr.NC) hc <<= 1;
  tr.HC = hc;
  gm.DMAX = 2 * max_moves + 8;
  gm.HMAX = 2 * max_moves + 8;
  const size_t TN = (size_t)T * tr.NC;
  ECHK(h->dalloc(&tr.node_pos, TN));
  ECHK(h->dalloc(&tr.node_hdr, TN));
  ECHK(h->dalloc(&tr.hash, (size_t)T * tr.HC));
  ECHK(h->dalloc(&tr.n_nodes, T));
  ECHK(h->dalloc(&tr.n_edges, T));
  ECHK(h->dalloc(&tr.pool_used, 1));
  HIPCHK(hipMemset(tr.hash, 0, (size_t)T * tr.HC * 4));
  HIPCHK(hipMemset(tr.n_nodes, 0, T * 4));
  // edges: 16 per node in each tree's region (random-init games average ~7.5 legal moves per
  // node, the C3 net ~11) plus a shared pool of 8 per node per tree for the trees that outgrow
  // theirs (a C3 game at 256 sims reached 16+ per node), capped by the 32-bit edge index
  {
    int64_t ec = 16 * (int64_t)tr.NC, pool = 8 * (int64_t)tr.NC * T;
    const int64_t lim = (int64_t)NONE - 1;
    if ((int64_t)T * ec + pool > lim) pool = std::max<int64_t>(0, lim - (int64_t)T * ec);
    ECHK(alloc_edges(h, ec, pool));
  }
  ECHK(h->dalloc(&gm.root, G));
  ECHK(h->dalloc(&gm.root_node, G));
  HIPCHK(hipMemset(gm.root_node, 0xff, G * 4));
  ECHK(h->dalloc(&gm.agent, G));
  // (k_select reads the active bytes as aligned 32-bit words: the allocation is padded to whole words,
  // the padding zeroed below with the rest)
  ECHK(h->dalloc(&gm.active, (size_t)(G + 3) / 4 * 4));
  ECHK(h->dalloc(&gm.outcome, G));
  ECHK(h->dalloc(&gm.root_new, G));
  ECHK(h->dalloc(&gm.root_k, G));
  ECHK(h->dalloc(&gm.noise_off, G));
  ECHK(h->dalloc(&gm.noise_js, G));
  ECHK(h->dalloc(&gm.path_node, (size_t)G * gm.DMAX));
  ECHK(h->dalloc(&gm.path_edge, (size_t)G * gm.DMAX));
  ECHK(h->dalloc(&gm.path_len, G));
  ECHK(h->dalloc(&gm.simc, G));
  ECHK(h->dalloc(&gm.hist, (size_t)G * gm.HMAX));
  ECHK(h->dalloc(&gm.nhist, G));
  ECHK(h->dalloc(&gm.mt_key, (size_t)G * 624));
  ECHK(h->dalloc(&gm.mt_pos, G));
  ECHK(h->dalloc(&gm.stot, G));
  HIPCHK(hipMemset(gm.stot, 0, (size_t)G * 4));
  gm.PLY = gm.HMAX;   // a game has at most HMAX plies (k_apply's history capacity)
  gm.RC = (int64_t)gm.PLY * KMAX;
  HIPCHK(hipMemset(gm.active, 0, (size_t)(G + 3) / 4 * 4));
  HIPCHK(hipMemset(gm.agent, 0, G * 4));
  HIPCHK(hipMemset(gm.nhist, 0, G * 4));
  HIPCHK(hipMemset(gm.outcome, 0, G * 4));
  ECHK(ensure_noise(h, (size_t)G * h->sims * 16));
  ECHK(h->dalloc(&lf.gnode, G));
  ECHK(h->dalloc(&lf.gpos, G));
  ECHK(h->dalloc(&lf.count, 1));
  ECHK(h->dalloc(&lf.game, G));
  ECHK(h->dalloc(&lf.tree, G));
  ECHK(h->dalloc(&lf.node, G));
  ECHK(h->dalloc(&lf.pos, G));
  ECHK(h->dalloc(&lf.P, (size_t)G * KMAX));
  ECHK(h->dalloc(&lf.v, G));
  ECHK(h->dalloc(&lf.ghit, G));
  HIPCHK(hipMemset(lf.ghit, 0, G));
  ECHK(h->dalloc(&h->d_actions, G));
  ECHK(h->dalloc(&h->d_root_codes, (size_t)G * KMAX));
  ECHK(h->dalloc(&h->d_root_visits, (size_t)G * KMAX));
  ECHK(h->dalloc(&h->d_leaf_codes, (size_t)G * KMAX));
  ECHK(h->dalloc(&h->d_leaf_k, G));
  ECHK(h->dalloc(&h->d_trees, T));
  // waves (two per simulation and move: deferred tails add waves at the end of a move); three ints
  // each (evaluated leaves, game / batch memo hits)
  // the deferred-tail guard of mtaz_play lets a move run sims + 4 sims + 8 waves
  h->count_log_cap = (5 * h->sims + 8) * (2 * max_moves + 8);
  ECHK(h->dalloc(&h->d_count_log, 3 * (size_t)h->count_log_cap));
  ECHK(h->dalloc(&h->d_remaining, 1));
  HIPCHK(hipMemset(lf.gnode, 0xff, (size_t)G * 4));   // no leaf pending
  HIPCHK(hipMemset(gm.simc, 0, (size_t)G * 4));
  if (hipDeviceGetAttribute(&h->ncu, hipDeviceAttributeMultiprocessorCount, h->device) != hipSuccess) h->ncu = 0;
  // exact sqrt(N.sum()) table: N.sum() <= sims * searches per agent
  const int sqn = tr.NC + 2;
  std::vector<double> sq(sqn);
  for (int i = 0; i < sqn; ++i) sq[i] = sqrt((double)i);
  ECHK(h->dalloc(&h->d_sqrt, sqn));
  HIPCHK(hipMemcpy(h->d_sqrt, sq.data(), sqn * 8, hipMemcpyHostToDevice));
  ECHK(h->dalloc(&h->d.pr.err, 1));
  HIPCHK(hipMemset(h->d.pr.err, 0, 4));
  Params& pr = h->d.pr;
  pr.G = G;
  pr.sims = h->sims;
  pr.cpuct = h->cpuct;
  pr.cpuct_f = (float)h->cpuct;
  pr.cast_mode = h->cast_mode;
  pr.flags = h->flags;
  pr.move_cap = h->move_cap;
  pr.sqrt_tab = h->d_sqrt;
  pr.sqrt_n = sqn;
  pr.memo = h->memo;
  pr.lag_order = 0;
  pr.alpha = h->alpha;
  pr.tau = h->tau;
  // network activations: [G][256][32] x 3
  h->nb.B = G;
  ECHK(h->dalloc(&h->nb.x0, (size_t)G * 8192));
  ECHK(h->dalloc(&h->nb.x1, (size_t)G * 8192));
  ECHK(h->dalloc(&h->nb.t, (size_t)G * 8192));
  h->rng.resize(G);
  return 0;
}

extern "C" mtaz_engine* mtaz_create(int device, int n_games, int sims, double cpuct, int tau_change, double dir_alpha,
                                    double dir_eps, uint64_t seed_base, int numpy_cast_mode, uint32_t rules_flags,
                                    int move_cap) {
  if (n_games <= 0 || sims <= 0) { set_err(MTAZ_E_FAIL, "n_games and sims must be positive"); return nullptr; }
  if (numpy_cast_mode != 1 && numpy_cast_mode != 2) { set_err(MTAZ_E_FAIL, "numpy_cast_mode must be 1 or 2"); return nullptr; }
  // the PUCT kernel hard-codes the reference's 0.75 / 0.25 mix (exp/agent.py:82)
  if (dir_eps != 0.25 || !(dir_alpha > 0)) {
    set_err(MTAZ_E_FAIL, "dir_eps must be 0.25 (exp/agent.py:82) and dir_alpha > 0");
    return nullptr;
  }
  if (ensure_codec_device(device)) return nullptr;
  mtaz_engine* h = new mtaz_engine();
  h->device = device;
  h->G = n_games;
  h->sims = sims;
  h->cpuct = cpuct;
  h->tau = tau_change;
  h->alpha = dir_alpha;
  h->eps = dir_eps;
  h->seed_base = seed_base;
  h->cast_mode = numpy_cast_mode;
  h->flags = rules_flags;
  h->move_cap = move_cap;
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess || engine_alloc(h) < 0) {
    const std::string e = g_err.empty() ? "engine allocation failed" : g_err;
    delete h;
    set_err(MTAZ_E_DEVICE, "%s", e.c_str());
    return nullptr;
  }
  return h;
}

extern "C" void mtaz_destroy(mtaz_engine* h) { delete h; }

// Wait for the engine's stream (every host sync point of the engine goes through here).
static hipError_t stream_wait(mtaz_engine* h) {
  if (h->sync_mode == 0) return hipStreamSynchronize(h->stream);
  if (!h->sync_ev) {
    const hipError_t e = hipEventCreateWithFlags(&h->sync_ev, hipEventBlockingSync | hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  const hipError_t e = hipEventRecord(h->sync_ev, h->stream);
  return e != hipSuccess ? e : hipEventSynchronize(h->sync_ev);
}

// memo_path: the call ran simulations whose leaves a memo (mtaz_set_memo >= 1) can hand to another
// batch; there ERR_ZRANGE (k_net_z's per-workgroup exponent left 0) is an error, elsewhere a note.
static int check_err(mtaz_engine* h, bool memo_path = true) {
  int32_t e = 0;
  if (!h->err_host) HIPCHK(hipHostMalloc(&h->err_host, 4, hipHostMallocDefault));
  HIPCHK(hipMemcpyAsync(h->err_host, h->d.pr.err, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(stream_wait(h));
  e = *h->err_host;
  if (e) {
    HIPCHK(hipMemsetAsync(h->d.pr.err, 0, 4, h->stream));
    if ((e & ERR_ZRANGE) && !(memo_path && h->d.pr.memo >= 1)) e &= ~ERR_ZRANGE;
    if (!e) return 0;
    std::string m;
    if (e & ERR_NODES) m += " node-capacity";
    if (e & ERR_EDGES) m += " edge-capacity";
    if (e & ERR_DEPTH) m += " search-depth";
    if (e & ERR_KMAX) m += " legal-list>256";
    if (e & ERR_SQRT) m += " visit-sum";
    if (e & ERR_ROOT) m += " root-state";
    if (e & ERR_ILLEGAL) m += " illegal-action";
    if (e & ERR_HIST) m += " history-capacity";
    if (e & ERR_HASH) m += " hash-full";
    if (e & ERR_F16) m += " activation-exceeds-f16-range";
    if (e & ERR_RNG) m += " rng-words";
    if (e & ERR_PUCT) m += " puct-argmax";
    if (e & ERR_ZRANGE)
      m += " f16f8-range-with-memo (k_net_z keeps one exponent per workgroup: past 2^14 its results depend"
           " on the batch, so memo >= 1 would hand them to other games; use f16x3 or mtaz_set_memo(0))";
    return set_err((e & ERR_ILLEGAL) ? MTAZ_E_ILLEGAL : MTAZ_E_CAPACITY, "device error flags 0x%x:%s", e, m.c_str());
  }
  return 0;
}

// ---- weights --------------------------------------------------------------------------
static int clear_batch_memo(mtaz_engine* h);

extern "C" int mtaz_set_weights(mtaz_engine* h, const float* const* d_tensors, const int64_t* numels, int n) {
  if (n != 133) return set_err(MTAZ_E_FAIL, "expected 133 state_dict tensors (num_batches_tracked skipped), got %d", n);
  HIPCHK(hipSetDevice(h->device));
  std::vector<std::vector<float>> t(n);
  for (int i = 0; i < n; ++i) {
    t[i].resize(numels[i]);
    HIPCHK(hipMemcpy(t[i].data(), d_tensors[i], numels[i] * 4, hipMemcpyDeviceToHost));
  }
  auto expect = [&](int i, int64_t ne) { return numels[i] == ne; };
  // layout checks (exp/policy.py:54-69)
  bool ok = expect(0, 28) && expect(1, 256 * 8 * 9) && expect(121, 554 * 61) && expect(122, 554) && expect(123, 256) &&
            expect(129, 256 * 31) && expect(130, 256) && expect(131, 256) && expect(132, 1) && expect(115, 512);
  for (int j = 0; j < 18 && ok; ++j) ok = expect(7 + j * 6, 256 * 256 * 9) && expect(8 + j * 6, 256);
  if (!ok) return set_err(MTAZ_E_FAIL, "state_dict tensor sizes do not match exp/policy.py Network");
  const double bn_eps = 1e-5;   // torch.nn.BatchNorm2d default (exp/policy.py:32)
  // conv at tensor index base: w, b, gamma, beta, mean, var -> folded scale/shift per out channel
  auto fold = [&](int base, int cout, std::vector<double>& scale, std::vector<double>& shift) {
    scale.resize(cout);
    shift.resize(cout);
    for (int c = 0; c < cout; ++c) {
      const double s = (double)t[base + 2][c] / sqrt((double)t[base + 5][c] + bn_eps);
      scale[c] = s;
      shift[c] = ((double)t[base + 1][c] - (double)t[base + 4][c]) * s + (double)t[base + 3][c];
    }
  };
  const size_t n_emb = 28, n_stem = 256 * 72 + 256, n_conv = (size_t)CONV_LAYERS * (CONV_W_FLOATS + 256);
  const size_t n_heads = 512 + 2 + 554 * 61 + 554 + 256 + 1 + 256 * 31 + 256 + 256 + 1;
  const size_t total = n_emb + n_stem + n_conv + n_heads + 64;
  std::vector<float> buf(total, 0.f);
  size_t off = 0;
  auto take = [&](size_t cnt) { size_t o = off; off += (cnt + 15) & ~(size_t)15; return o; };
  const size_t o_emb = take(28), o_stem_w = take(256 * 72), o_stem_b = take(256);
  const size_t o_conv_w = take((size_t)CONV_LAYERS * CONV_W_FLOATS), o_conv_b = take(CONV_LAYERS * 256);
  const size_t o_pw = take(512), o_pb = take(2), o_plw = take(554 * 61), o_plb = take(554), o_vw = take(256),
               o_vb = take(1), o_v1w = take(256 * 31), o_v1b = take(256), o_v2w = take(256), o_v2b = take(1);
  if (off > buf.size()) buf.resize(off);
  std::copy(t[0].begin(), t[0].end(), buf.begin() + o_emb);
  std::vector<double> sc, sh;
  fold(1, 256, sc, sh);
  for (int co = 0; co < 256; ++co) {
    for (int j = 0; j < 72; ++j) buf[o_stem_w + co * 72 + j] = (float)(t[1][co * 72 + j] * sc[co]);
    buf[o_stem_b + co] = (float)sh[co];
  }
  for (int L = 0; L < CONV_LAYERS; ++L) {
    const int base = 7 + L * 6;
    fold(base, 256, sc, sh);
    const std::vector<float>& W = t[base];   // [co][ci][3][3]
    float* dst = buf.data() + o_conv_w + (size_t)L * CONV_W_FLOATS;
    for (int ct = 0; ct < 8; ++ct)
      for (int q = 0; q < 288; ++q)
        for (int lane = 0; lane < 64; ++lane)
          for (int e = 0; e < 4; ++e) {
            const int s = 4 * q + e, k = 2 * s + (lane >> 5);
            const int tap = k >> 8, ci = k & 255, co = ct * 32 + (lane & 31);
            dst[(((size_t)ct * 288 + q) * 64 + lane) * 4 + e] = (float)(W[((size_t)co * 256 + ci) * 9 + tap] * sc[co]);
          }
    for (int co = 0; co < 256; ++co) buf[o_conv_b + L * 256 + co] = (float)sh[co];
  }
  fold(115, 2, sc, sh);
  for (int o = 0; o < 2; ++o) {
    for (int c = 0; c < 256; ++c) buf[o_pw + o * 256 + c] = (float)(t[115][o * 256 + c] * sc[o]);
    buf[o_pb + o] = (float)sh[o];
  }
  std::copy(t[121].begin(), t[121].end(), buf.begin() + o_plw);
  std::copy(t[122].begin(), t[122].end(), buf.begin() + o_plb);
  fold(123, 1, sc, sh);
  for (int c = 0; c < 256; ++c) buf[o_vw + c] = (float)(t[123][c] * sc[0]);
  buf[o_vb] = (float)sh[0];
  std::copy(t[129].begin(), t[129].end(), buf.begin() + o_v1w);
  std::copy(t[130].begin(), t[130].end(), buf.begin() + o_v1b);
  std::copy(t[131].begin(), t[131].end(), buf.begin() + o_v2w);
  buf[o_v2b] = t[132][0];
  if (!h->wbuf) ECHK(h->dalloc(&h->wbuf, buf.size()));
  HIPCHK(hipMemcpy(h->wbuf, buf.data(), buf.size() * 4, hipMemcpyHostToDevice));
  float* b = h->wbuf;
  h->w.emb = b + o_emb;
  h->w.stem_w = b + o_stem_w;
  h->w.stem_b = b + o_stem_b;
  h->w.conv_w = b + o_conv_w;
  h->w.conv_b = b + o_conv_b;
  h->w.pconv_w = b + o_pw;
  h->w.pconv_b = b + o_pb;
  h->w.plin_w = b + o_plw;
  h->w.plin_b = b + o_plb;
  h->w.vconv_w = b + o_vw;
  h->w.vconv_b = b + o_vb;
  h->w.vl1_w = b + o_v1w;
  h->w.vl1_b = b + o_v1b;
  h->w.vl2_w = b + o_v2w;
  h->w.vl2_b = b + o_v2b;

  // fp16x3 trunk weights: per layer scale 2^e (max |w| * 2^e <= 8192), hi = f16(w),
  // lo = f16(w - hi); host staging in the 32x32x16 A-operand order (round 1's k_net_x), from
  // which the 16x16x32 layouts below are gathered.
  std::vector<_Float16> wx((size_t)CONV_LAYERS * CONVX_U4_PER_LAYER * 8);
  std::vector<float> winv(CONV_LAYERS);
  for (int L = 0; L < CONV_LAYERS; ++L) {
    const int base = 7 + L * 6;
    fold(base, 256, sc, sh);
    const std::vector<float>& W = t[base];
    double mx = 0;
    for (int co = 0; co < 256; ++co)
      for (int j = 0; j < 256 * 9; ++j) mx = std::max(mx, fabs(W[(size_t)co * 2304 + j] * sc[co]));
    const int e = mx > 0 ? (int)floor(log2(8192.0 / mx)) : 0;
    const double s = ldexp(1.0, e);
    winv[L] = (float)ldexp(1.0, -e);
    _Float16* dst = wx.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    for (int ct = 0; ct < 8; ++ct)
      for (int kb = 0; kb < 144; ++kb)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int co = ct * 32 + (lane & 31), k = kb * 16 + 8 * (lane >> 5) + j;
            const int tap = k >> 8, ci = k & 255;
            const double v = (double)W[((size_t)co * 256 + ci) * 9 + tap] * sc[co] * s;
            const _Float16 hi = (_Float16)v;
            const _Float16 lo = (_Float16)(v - (double)hi);
            const size_t u4 = ((size_t)ct * 144 + kb) * 128 + lane;
            dst[u4 * 8 + j] = hi;
            dst[(u4 + 64) * 8 + j] = lo;
          }
  }
  // stem (tensor 1: [256][8][3][3]) in the same split form, 5 k-blocks of 2 taps x 8 channels
  std::vector<_Float16> sx((size_t)8 * 5 * 128 * 8);
  {
    fold(1, 256, sc, sh);
    double mx = 0;
    for (int co = 0; co < 256; ++co)
      for (int j = 0; j < 72; ++j) mx = std::max(mx, fabs(t[1][co * 72 + j] * sc[co]));
    const int e = mx > 0 ? (int)floor(log2(8192.0 / mx)) : 0;
    const double s = ldexp(1.0, e);
    winv.push_back((float)ldexp(1.0, -e));
    for (int ct = 0; ct < 8; ++ct)
      for (int kb = 0; kb < 5; ++kb)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int co = ct * 32 + (lane & 31), tap = 2 * kb + (lane >> 5), c = j;
            const double v = tap < 9 ? (double)t[1][co * 72 + c * 9 + tap] * sc[co] * s : 0.0;
            const _Float16 hi = (_Float16)v;
            const _Float16 lo = (_Float16)(v - (double)hi);
            const size_t u4 = ((size_t)ct * 5 + kb) * 128 + lane;
            sx[u4 * 8 + j] = hi;
            sx[(u4 + 64) * 8 + j] = lo;
          }
  }
  // the same split values re-laid out as the A operand of v_mfma_f32_16x16x32_f16 (k_net_y)
  std::vector<_Float16> wy(wx.size());
  for (int L = 0; L < CONV_LAYERS; ++L) {
    const _Float16* src = wx.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    _Float16* dst = wy.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    for (int ct = 0; ct < 16; ++ct)
      for (int kb = 0; kb < 72; ++kb)
        for (int part = 0; part < 2; ++part)
          for (int lane = 0; lane < 64; ++lane)
            for (int j = 0; j < 8; ++j) {
              const int co = 16 * ct + (lane & 15), k = 32 * kb + 8 * (lane >> 4) + j;
              // position of (co, k) in the 32x32x16 layout: cotile co/32, kblock k/16, lane (co%32) + 32*((k%16)/8)
              const size_t xu4 = ((size_t)(co >> 5) * 144 + (k >> 4)) * 128 + part * 64 + (co & 31) + 32 * ((k & 15) >> 3);
              dst[((((size_t)ct * 72 + kb) * 2 + part) * 64 + lane) * 8 + j] = src[xu4 * 8 + (k & 7)];
            }
  }
  std::vector<_Float16> sy((size_t)16 * 3 * 128 * 8);
  for (int ct = 0; ct < 16; ++ct)
    for (int kb = 0; kb < 3; ++kb)
      for (int part = 0; part < 2; ++part)
        for (int lane = 0; lane < 64; ++lane)
          for (int j = 0; j < 8; ++j) {
            const int co = 16 * ct + (lane & 15), tap = 4 * kb + (lane >> 4);
            _Float16 v = (_Float16)0.f;
            if (tap < 9) {   // stemx: cotile co/32, kblock tap/2, lane (co%32) + 32*(tap%2)
              const size_t xu4 = ((size_t)(co >> 5) * 5 + (tap >> 1)) * 128 + part * 64 + (co & 31) + 32 * (tap & 1);
              v = sx[xu4 * 8 + j];
            }
            sy[((((size_t)ct * 3 + kb) * 2 + part) * 64 + lane) * 8 + j] = v;
          }
  // k_net_z: the split parts of wy (f16 hi / lo of W * 2^e) once more, each scaled by a per-layer
  // power of two 2^a (largest |part| -> [128, 256)) and rounded to OCP e4m3, in the A-operand
  // order of v_mfma_scale_f32_16x16x128_f8f6f4 (engine.h NetWeights::conv8); scale 127 - a.
  std::vector<uint8_t> w8((size_t)CONV_LAYERS * CONV8_U4_PER_LAYER * 16);
  std::vector<int32_t> sc8(2 * CONV_LAYERS + 4, 127);
  for (int L = 0; L < CONV_LAYERS; ++L) {
    const _Float16* src = wy.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    // wy: [ct 16][kb 72][part 2][lane 64][8]; element (co, k) of part at lane (co&15) + 16*((k&31)>>3)
    auto at = [&](int part, int co, int k) {
      const int ct = co >> 4, kb = k >> 5, ln = (co & 15) + 16 * ((k & 31) >> 3);
      return (double)src[((((size_t)ct * 72 + kb) * 2 + part) * 64 + ln) * 8 + (k & 7)];
    };
    int a[2];
    for (int part = 0; part < 2; ++part) {
      double mx = 0;
      for (size_t i = 0; i < CONVX_U4_PER_LAYER * 8; ++i)
        if (((i / 512) & 1) == (size_t)part) mx = std::max(mx, fabs((double)src[i]));
      a[part] = mx > 0 ? 7 - ilogb(mx) : 0;
      sc8[2 * L + part] = 127 - a[part];
    }
    uint8_t* dst = w8.data() + (size_t)L * CONV8_U4_PER_LAYER * 16;
    for (int ct = 0; ct < 16; ++ct)
      for (int t = 0; t < 9; ++t)
        for (int c = 0; c < 2; ++c)
          for (int part = 0; part < 2; ++part)
            for (int half = 0; half < 2; ++half)
              for (int lane = 0; lane < 64; ++lane)
                for (int byte = 0; byte < 16; ++byte) {
                  const int co = zrow_co(ct, lane & 15), ci = 128 * c + 32 * (lane >> 4) + 16 * half + byte;
                  const size_t u4 = (((((size_t)ct * 9 + t) * 2 + c) * 2 + part) * 2 + half) * 64 + lane;
                  dst[u4 * 16 + byte] = to_e4m3(ldexp(at(part, co, t * 256 + ci), a[part]));
                }
  }
  // k_net_z VAR 8192: the same parts in e2m3 blocks of 32 K with one e8m0 scale each
  // (NetWeights::conv6)
  std::vector<uint8_t> w6((size_t)CONV_LAYERS * CONV6_U4_PER_LAYER * 16, 0);
  for (int L = 0; L < CONV_LAYERS; ++L) {
    const _Float16* src = wy.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    auto at = [&](int part, int co, int k) {
      const int ct = co >> 4, kb = k >> 5, ln = (co & 15) + 16 * ((k & 31) >> 3);
      return (double)src[((((size_t)ct * 72 + kb) * 2 + part) * 64 + ln) * 8 + (k & 7)];
    };
    uint8_t* dst = w6.data() + (size_t)L * CONV6_U4_PER_LAYER * 16;
    for (int ct = 0; ct < 16; ++ct)
      for (int t = 0; t < 9; ++t)
        for (int c = 0; c < 2; ++c)
          for (int part = 0; part < 2; ++part) {
            uint8_t* gb = dst + ((((size_t)ct * 9 + t) * 2 + c) * 2 + part) * 112 * 16;
            for (int lane = 0; lane < 64; ++lane) {
              const int co = zrow_co(ct, lane & 15);
              double v[32], mx = 0;
              for (int q = 0; q < 32; ++q) {
                const int ci = 128 * c + 32 * (lane >> 4) + q;
                v[q] = at(part, co, t * 256 + ci);
                mx = std::max(mx, fabs(v[q]));
              }
              int sc = -126;   // smallest s with mx * 2^-s <= 7.5
              if (mx > 0) {
                sc = ilogb(mx) - 2;
                if (ldexp(mx, -sc) > 7.5) ++sc;
                sc = std::max(-126, std::min(126, sc));
              }
              uint8_t bytes[24] = {0};
              for (int q = 0; q < 32; ++q) {
                const uint32_t code = to_e2m3(ldexp(v[q], -sc));
                for (int b = 0; b < 6; ++b)
                  if (code >> b & 1) bytes[(6 * q + b) >> 3] |= (uint8_t)(1u << ((6 * q + b) & 7));
              }
              memcpy(gb + 16 * lane, bytes, 16);
              memcpy(gb + 1024 + 8 * lane, bytes + 16, 8);
              gb[1536 + 4 * lane] = (uint8_t)(127 + sc);
            }
          }
  }
  // round 4's k_net_y: wy k-block-major (NetWeights::convyk)
  std::vector<_Float16> wk(wy.size());
  for (int L = 0; L < CONV_LAYERS; ++L) {
    const _Float16* src = wy.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    _Float16* dst = wk.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    for (int ct = 0; ct < 16; ++ct)
      for (int kb = 0; kb < 72; ++kb)
        memcpy(dst + ((size_t)kb * 16 + ct) * 2 * 64 * 8, src + ((size_t)ct * 72 + kb) * 2 * 64 * 8, 2 * 64 * 8 * 2);
  }
  // k_net_z's row-interleaved copies of wy and sy (NetWeights::convz, stemz)
  std::vector<_Float16> wz(wy.size()), sz(sy.size());
  for (int L = 0; L < CONV_LAYERS; ++L) {
    const _Float16* src = wy.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    _Float16* dst = wz.data() + (size_t)L * CONVX_U4_PER_LAYER * 8;
    for (int T = 0; T < 16; ++T)
      for (int kb = 0; kb < 72; ++kb)
        for (int part = 0; part < 2; ++part)
          for (int lane = 0; lane < 64; ++lane) {
            const int c = zrow_co(T, lane & 15);
            const size_t si = ((((size_t)(c >> 4) * 72 + kb) * 2 + part) * 64 + (c & 15) + 16 * (lane >> 4)) * 8;
            const size_t di = ((((size_t)T * 72 + kb) * 2 + part) * 64 + lane) * 8;
            for (int j = 0; j < 8; ++j) dst[di + j] = src[si + j];
          }
  }
  for (int T = 0; T < 16; ++T)
    for (int kb = 0; kb < 3; ++kb)
      for (int part = 0; part < 2; ++part)
        for (int lane = 0; lane < 64; ++lane) {
          const int c = zrow_co(T, lane & 15);
          const size_t si = ((((size_t)(c >> 4) * 3 + kb) * 2 + part) * 64 + (c & 15) + 16 * (lane >> 4)) * 8;
          const size_t di = ((((size_t)T * 3 + kb) * 2 + part) * 64 + lane) * 8;
          for (int j = 0; j < 8; ++j) sz[di + j] = sy[si + j];
        }
  // k_net_y output bounds (NetWeights::yrange): per conv the max over output channels of the
  // L1 norm of the folded weights and the max |folded bias|; the stem's; max |embedding|.
  std::vector<float> yr(2 * CONV_LAYERS + 3);
  auto up = [](double d) {   // float >= d
    float f = (float)d;
    if ((double)f < d) f = std::nextafter(f, INFINITY);
    return f;
  };
  for (int L = 0; L <= CONV_LAYERS; ++L) {
    const bool stem = L == CONV_LAYERS;
    const int base = stem ? 1 : 7 + L * 6, kk = stem ? 72 : 2304;
    fold(base, 256, sc, sh);
    double g = 0, b = 0;
    for (int co = 0; co < 256; ++co) {
      double r = 0;
      for (int j = 0; j < kk; ++j) r += fabs((double)t[base][(size_t)co * kk + j]);
      g = std::max(g, r * fabs(sc[co]));
      b = std::max(b, fabs(sh[co]));
    }
    yr[2 * L] = up(g);
    yr[2 * L + 1] = up(b);
  }
  {
    double e = 0;
    for (float v : t[0]) e = std::max(e, fabs((double)v));
    yr[2 * CONV_LAYERS + 2] = up(e);
  }
  if (!h->wyrange) ECHK(h->dalloc(&h->wyrange, yr.size()));
  HIPCHK(hipMemcpy(h->wyrange, yr.data(), yr.size() * 4, hipMemcpyHostToDevice));
  h->w.yrange = h->wyrange;
  const size_t nx = wy.size() / 8, nsy = sy.size() / 8, n8 = w8.size() / 16;
  const size_t nsc = (sc8.size() + 3) / 4, n6 = w6.size() / 16;
  // device layout (16-B units): convy | stemy | conv8 | conv8_sc | conv6 | convz | stemz | convyk
  const size_t o_sy = nx, o_w8 = o_sy + nsy, o_sc = o_w8 + n8, o_w6 = o_sc + nsc, o_wz = o_w6 + n6;
  const size_t o_sz = o_wz + nx, o_wk = o_sz + nsy, o_end = o_wk + nx;
  if (!h->wxbuf) ECHK(h->dalloc(&h->wxbuf, o_end));
  if (!h->wxinv) ECHK(h->dalloc(&h->wxinv, CONV_LAYERS + 1));
  HIPCHK(hipMemcpy(h->wxbuf, wy.data(), nx * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxbuf + o_sy, sy.data(), nsy * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxbuf + o_w8, w8.data(), n8 * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxbuf + o_sc, sc8.data(), sc8.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxbuf + o_w6, w6.data(), n6 * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxbuf + o_wz, wz.data(), nx * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxbuf + o_sz, sz.data(), nsy * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxbuf + o_wk, wk.data(), nx * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(h->wxinv, winv.data(), (CONV_LAYERS + 1) * 4, hipMemcpyHostToDevice));
  h->w.convx_inv = h->wxinv;
  h->w.stemx_inv = h->wxinv + CONV_LAYERS;
  h->w.convy = h->wxbuf;
  h->w.stemy = h->wxbuf + o_sy;
  h->w.conv8 = h->wxbuf + o_w8;
  h->w.conv8_sc = reinterpret_cast<const int32_t*>(h->wxbuf + o_sc);
  h->w.conv6 = h->wxbuf + o_w6;
  h->w.convz = h->wxbuf + o_wz;
  h->w.stemz = h->wxbuf + o_sz;
  h->w.convyk = h->wxbuf + o_wk;
  h->weights_ok = true;
  ECHK(clear_batch_memo(h));   // results of the previous network
  return 0;
}

static void launch_network(mtaz_engine* h, const Pos* pos, const int32_t* count, int max_b, int mode, float* logits,
                           float* values, hipEvent_t eb, hipEvent_t ee) {
  // f16x3 variant 268435456 (diagnostic library): k_net_y's arithmetic in k_net_z's structure
  // (mtaz_net8.hip, W3; without k_net_y's chunked accumulation)
  if (h->precision == NET_F16F8 || (h->precision == NET_F16X3 && h->variant == 268435456)) {
    launch_net_z(h->d, h->w, pos, count, max_b, mode, logits, values, h->stream, eb, ee, h->variant);
  } else if (h->precision == NET_F16X3) {
    launch_net_f16x3(h->d, h->w, pos, count, max_b, mode, logits, values, h->stream, eb, ee, h->variant);
  } else {
    NetBuffers nb = h->nb;
    nb.logits = logits;
    launch_net(h->d, h->w, nb, pos, count, max_b, mode, values, h->stream, eb, ee);
  }
}

// Kernel timing harness for the network alone (tools/bench_net.py): `iters` back-to-back
// full-logit launches on n device positions timed with HIP events; optionally one more
// launch of the stamp-instrumented diagnostic build (phase cycle shares per workgroup).
extern "C" int mtaz_net_time(mtaz_engine* h, const uint32_t* d_pos, int n, int iters, int stamped, float* ms_out,
                             uint64_t* stamps_out) {
  if (!h->weights_ok) return set_err(MTAZ_E_FAIL, "weights not set (mtaz_set_weights)");
  if (n <= 0 || iters <= 0) return set_err(MTAZ_E_FAIL, "n and iters must be positive");
  HIPCHK(hipSetDevice(h->device));
  float *logits = nullptr, *values = nullptr;
  unsigned long long* st = nullptr;
  const int nwg = (n + 3) / 4;
  const int NST = 10;   // per workgroup: 6 phase stamps, then (in a second region) 4 exponent records
  HIPCHK(hipMalloc(&logits, (size_t)n * NUM_ACTIONS * 4));
  HIPCHK(hipMalloc(&values, (size_t)n * 4));
  HIPCHK(hipMalloc(&st, (size_t)nwg * NST * 8));
  HIPCHK(hipMemset(st, 0, (size_t)nwg * NST * 8));
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  const Pos* pos = reinterpret_cast<const Pos*>(d_pos);
  if (h->precision == NET_FP32 && n > h->G) return set_err(MTAZ_E_CAPACITY, "fp32 path: n must be <= engine games");
  launch_network(h, pos, nullptr, n, NET_FULL_LOGITS, logits, values, nullptr, nullptr);   // warm-up
  HIPCHK(hipEventRecord(e0, h->stream));
  for (int i = 0; i < iters; ++i) launch_network(h, pos, nullptr, n, NET_FULL_LOGITS, logits, values, nullptr, nullptr);
  HIPCHK(hipEventRecord(e1, h->stream));
  HIPCHK(hipEventSynchronize(e1));
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, e0, e1));
  *ms_out = ms / iters;
  if (stamped && stamps_out) {
    if (h->precision == NET_F16F8)
      launch_net_z_stamped(h->d, h->w, pos, n, logits, values, st, h->stream, h->variant);
    else
      launch_net_f16x3_stamped(h->d, h->w, pos, n, logits, values, st, h->stream, h->variant);
    HIPCHK(hipMemcpyAsync(stamps_out, st, (size_t)nwg * NST * 8, hipMemcpyDeviceToHost, h->stream));
  }
  HIPCHK(stream_wait(h));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(logits);
  (void)hipFree(values);
  (void)hipFree(st);
  return check_err(h, false);
}

// Variants a product library accepts: each parity-green against the reference fixtures
// (tests/test_gpu_net.py).  k_net_y: 1 = 4 boards per workgroup in every round (no tail launch),
// 2 = the class tiles without the tap skip (bit-identity reference of the skip), 5 = the first
// round-4 tail instances.  (3 = round 3's kernel, k_net_y3 in mtaz_net16_r3.hip, batch-dependent
// past 2^14: in the diagnostic library only, VERDICT r4 #7.)  k_net_z:
// 1 = the product kernel with 4 boards per workgroup in every round (no tail launches; bit-identity
// reference and A/B for the tail-balanced assignment), 2097152 = unfused epilogue (bit-identity reference), 8192 = e2m3 (fp6) cross terms,
// 25165824 = the round-2 K loop (per-step fragment addresses, global-address weights; bit-identity
// reference for the product's tap-major loop), 33554432 = the round-2 epilogue (unscaled
// conversions), 58720256 = both (the round-2 product).  The
// timing-only diagnostic builds (wrong results by construction) exist only in a library built
// with MTAZ_NET_DIAG (tools/bench_net.py --diag).
#ifdef MTAZ_NET_DIAG
// diagnostic library only (tools/select_stamps.py): k_select phase cycle sums since the last reset
extern "C" int mtaz_diag_select_stamps(unsigned long long* out8, int reset) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  return diag_select_stamps(out8, reset);
}
#endif

extern "C" int mtaz_set_net_variant(mtaz_engine* h, int variant) {
  bool ok = variant == 0;
  if (h->precision == NET_F16X3) ok = ok || variant == 1 || variant == 2 || variant == 5;
  if (h->precision == NET_F16F8)
    ok = ok || variant == 1 || variant == 2097152 || variant == 8192 || variant == 8388608 + 16777216 ||
         variant == 33554432 || variant == 8388608 + 16777216 + 33554432;
#ifdef MTAZ_NET_DIAG
  ok = true;
#endif
  if (!ok) return set_err(MTAZ_E_FAIL, "network variant %d is not a parity-tested build of precision %d", variant,
                          h->precision);
  h->variant = variant;
  return 0;
}

static void swap_slot(mtaz_engine* h) {
  std::swap(h->w, h->parked.w);
  std::swap(h->wbuf, h->parked.wbuf);
  std::swap(h->wxbuf, h->parked.wxbuf);
  std::swap(h->wxinv, h->parked.wxinv);
  std::swap(h->wyrange, h->parked.wyrange);
  std::swap(h->weights_ok, h->parked.ok);
  h->cur_slot ^= 1;
}

static void activate_slot(mtaz_engine* h, int slot) {
  if (slot != h->cur_slot) swap_slot(h);
}

extern "C" int mtaz_set_weights_slot(mtaz_engine* h, int slot, const float* const* d_tensors, const int64_t* numels,
                                     int n) {
  if (slot != 0 && slot != 1) return set_err(MTAZ_E_FAIL, "weight slot must be 0 or 1");
  const int cur = h->cur_slot;
  activate_slot(h, slot);
  const int rc = mtaz_set_weights(h, d_tensors, numels, n);
  activate_slot(h, cur);
  return rc;
}

// the memo shares leaf results between a game's two tables (and the batch's games): only when both
// agents search with the same network
static void sync_memo(mtaz_engine* h) { h->d.pr.memo = h->agent_slot[0] == h->agent_slot[1] ? h->memo : 0; }

// The batch memo's table.  A play evaluates at most one leaf per game and simulation; the table
// holds 2 slots per leaf of a 64-ply game (move_cap searches per agent, at most 32 each), a power
// of two, at most 2^26 slots (222 B each): 2^25 = 7.4 GB for 4096 games x 64 sims.  A full table,
// or a probe run past MEMO_PROBES, only skips inserts (memo misses, never a wrong entry).
static int ensure_batch_memo(mtaz_engine* h) {
  if (h->memo < 2 || h->d.bm.cap) return 0;
  const int plies = 2 * (h->move_cap > 0 && h->move_cap < 32 ? h->move_cap : 32);
  const uint64_t want = 2ull * (uint64_t)h->G * (uint64_t)plies * (uint64_t)h->sims;
  uint64_t cap = 1024;
  while (cap < want && cap < (1ull << 26)) cap <<= 1;
  BatchMemo& B = h->d.bm;
  auto grab = [&](auto** p, size_t elt) -> int {
    void* q = nullptr;
    HIPCHK(hipMalloc(&q, cap * elt));
    h->memo_allocs.push_back(q);
    *p = (std::remove_reference_t<decltype(*p)>)q;
    return 0;
  };
  ECHK(grab(&B.state, 4));
  ECHK(grab(&B.key, sizeof(Pos)));
  ECHK(grab(&B.v, 4));
  ECHK(grab(&B.k, 2));
  ECHK(grab(&B.codes, 2 * MEMO_K));
  ECHK(grab(&B.P, 4 * MEMO_K));
  B.cap = (uint32_t)cap;
  HIPCHK(hipMemset(B.state, 0, cap * 4));
  return 0;
}

// frees the batch memo (play_groups: the groups' engines keep their own, sized for their games)
static void release_batch_memo(mtaz_engine* h) {
  for (void* p : h->memo_allocs) (void)hipFree(p);
  h->memo_allocs.clear();
  h->d.bm = BatchMemo{};
}

// empties the batch memo (new weights, new play)
static int clear_batch_memo(mtaz_engine* h) {
  if (!h->d.bm.cap) return 0;
  launch_memo_clear(h->d, h->stream);
  HIPCHK(hipGetLastError());
  return 0;
}

extern "C" int mtaz_set_agent_slots(mtaz_engine* h, int slot_agent0, int slot_agent1) {
  if ((slot_agent0 | slot_agent1) & ~1) return set_err(MTAZ_E_FAIL, "weight slots must be 0 or 1");
  h->agent_slot[0] = slot_agent0;
  h->agent_slot[1] = slot_agent1;
  sync_memo(h);
  return 0;
}

extern "C" int mtaz_set_memo(mtaz_engine* h, int mode) {
  if (mode < 0 || mode > 2) return set_err(MTAZ_E_FAIL, "memo mode must be 0 (off), 1 (per game) or 2 (per game + batch)");
  HIPCHK(hipSetDevice(h->device));
  h->memo = mode;
  ECHK(ensure_batch_memo(h));
  ECHK(clear_batch_memo(h));
  sync_memo(h);
  return 0;
}

extern "C" int mtaz_set_pipeline(mtaz_engine* h, int groups) {
  if (groups < 1 || h->G % groups != 0) return set_err(MTAZ_E_FAIL, "groups=%d must divide n_games=%d", groups, h->G);
  if (groups != h->groups) {
    for (mtaz_engine* p : h->parts) delete p;
    h->parts.clear();
  }
  h->groups = groups;
  return 0;
}

// per-wave log of the last mtaz_play: [waves][evaluated leaves, game-memo hits, batch-memo hits]
extern "C" int mtaz_wave_log(mtaz_engine* h, int32_t* out, int max_waves) {
  if (h->last_play_grouped) {   // the groups' logs, group after group
    int n = 0;
    for (mtaz_engine* p : h->parts) {
      const int r = mtaz_wave_log(p, out + 3 * (size_t)n, max_waves - n);
      if (r < 0) return r;
      n += r;
    }
    return n;
  }
  const int n = std::min(std::min(h->wave, h->count_log_cap), max_waves);
  if (n > 0) HIPCHK(hipMemcpy(out, h->d_count_log, (size_t)n * 3 * 4, hipMemcpyDeviceToHost));
  return n;
}

extern "C" int mtaz_set_defer(mtaz_engine* h, int mode) {
  if (mode < 0 || mode > 2)
    return set_err(MTAZ_E_FAIL, "defer must be 0 (every leaf each wave), 1 (deferred tails) or 2 (every remainder)");
  h->defer = mode;
  for (mtaz_engine* p : h->parts) p->defer = mode;
  return 0;
}

extern "C" int mtaz_set_lag_order(mtaz_engine* h, int order) {
  if (order != 0 && order != 1) return set_err(MTAZ_E_FAIL, "lag order must be 0 (round 6) or 1 (round 5)");
  h->d.pr.lag_order = order;
  for (mtaz_engine* p : h->parts) p->d.pr.lag_order = order;
  return 0;
}

extern "C" int mtaz_set_schedule(mtaz_engine* h, int mode) {
  if (mode != 0 && mode != 1) return set_err(MTAZ_E_FAIL, "schedule must be 0 (moves in lockstep) or 1 (free-running moves)");
  h->schedule = mode;
  for (mtaz_engine* p : h->parts) p->schedule = mode;
  return 0;
}

extern "C" int mtaz_set_rng_device(mtaz_engine* h, int on) {
  if (on != 0 && on != 1) return set_err(MTAZ_E_FAIL, "rng_device must be 0 (host) or 1 (device)");
  h->rng_device = on;
  for (mtaz_engine* p : h->parts) p->rng_device = on;
  return 0;
}

// the device RNG's test entry (tests/test_gpu_rng.py): stream s = RandomState(seeds[s]) draws n_vec
// Dirichlet(alpha x ks[s]) vectors (rows of ks[s] doubles, streams one after another in out) with the
// kernels' own code (wave_dirichlet), then one random_sample() into tail[s].  Host buffers.
extern "C" int mtaz_rng_dirichlet_device(int device, const uint32_t* seeds, const int32_t* ks, int n_streams, int n_vec,
                                         double alpha, double* out, double* tail) {
  if (n_streams <= 0 || n_vec < 0) return set_err(MTAZ_E_FAIL, "n_streams must be positive, n_vec >= 0");
  if (!(alpha > 0 && alpha < 1)) return set_err(MTAZ_E_FAIL, "the device gamma sampler needs 0 < alpha < 1");
  std::vector<int64_t> offs(n_streams);
  int64_t tot = 0;
  for (int s = 0; s < n_streams; ++s) {
    if (ks[s] <= 0 || ks[s] > KMAX) return set_err(MTAZ_E_CAPACITY, "k = %d out of [1, %d]", ks[s], KMAX);
    offs[s] = tot;
    tot += (int64_t)ks[s] * n_vec;
  }
  HIPCHK(hipSetDevice(device));
  uint32_t *d_seeds = nullptr, *d_scr = nullptr;
  int32_t* d_ks = nullptr;
  int64_t* d_offs = nullptr;
  double *d_out = nullptr, *d_tail = nullptr;
  int rc = 0;
  auto fin = [&](int r) {
    (void)hipFree(d_seeds); (void)hipFree(d_scr); (void)hipFree(d_ks);
    (void)hipFree(d_offs); (void)hipFree(d_out); (void)hipFree(d_tail);
    return r;
  };
#define RNGCHK(x)                                                                       \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) return fin(set_err(MTAZ_E_DEVICE, "%s", hipGetErrorString(e_))); \
  } while (0)
  RNGCHK(hipMalloc(&d_seeds, n_streams * 4));
  RNGCHK(hipMalloc(&d_scr, (size_t)n_streams * 624 * 4));
  RNGCHK(hipMalloc(&d_ks, n_streams * 4));
  RNGCHK(hipMalloc(&d_offs, n_streams * 8));
  RNGCHK(hipMalloc(&d_out, std::max<int64_t>(tot, 1) * 8));
  RNGCHK(hipMalloc(&d_tail, n_streams * 8));
  RNGCHK(hipMemcpy(d_seeds, seeds, n_streams * 4, hipMemcpyHostToDevice));
  RNGCHK(hipMemcpy(d_ks, ks, n_streams * 4, hipMemcpyHostToDevice));
  RNGCHK(hipMemcpy(d_offs, offs.data(), n_streams * 8, hipMemcpyHostToDevice));
  launch_rng_dirichlet_test(d_seeds, d_ks, d_offs, n_streams, n_vec, alpha, d_out, d_tail, d_scr, nullptr);
  RNGCHK(hipGetLastError());
  RNGCHK(hipDeviceSynchronize());
  if (tot) RNGCHK(hipMemcpy(out, d_out, tot * 8, hipMemcpyDeviceToHost));
  RNGCHK(hipMemcpy(tail, d_tail, n_streams * 8, hipMemcpyDeviceToHost));
#undef RNGCHK
  return fin(rc);
}

extern "C" int mtaz_set_sync_mode(mtaz_engine* h, int mode) {
  if (mode != 0 && mode != 1) return set_err(MTAZ_E_FAIL, "sync mode must be 0 (stream sync) or 1 (blocking event)");
  h->sync_mode = mode;
  for (mtaz_engine* p : h->parts) p->sync_mode = mode;
  return 0;
}

extern "C" int mtaz_set_host_threads(mtaz_engine* h, int n) {
  if (n < 0) return set_err(MTAZ_E_FAIL, "host thread count must be >= 0");
  h->host_threads = n ? n : default_host_threads();
  return 0;
}

extern "C" int mtaz_set_seed_base(mtaz_engine* h, uint64_t seed_base) {
  h->seed_base = seed_base;
  return 0;
}

extern "C" int mtaz_set_precision(mtaz_engine* h, int precision) {
  if (precision != NET_FP32 && precision != NET_F16X3 && precision != NET_F16F8)
    return set_err(MTAZ_E_FAIL, "precision must be 0 (fp32), 1 (fp16x3) or 2 (f16 + e4m3 cross terms)");
  h->precision = precision;
  h->variant = 0;   // variants are per precision
  return 0;
}

extern "C" int mtaz_evaluate(mtaz_engine* h, const uint32_t* d_pos, int n, float* d_logits, float* d_values) {
  if (!h->weights_ok) return set_err(MTAZ_E_FAIL, "weights not set (mtaz_set_weights)");
  HIPCHK(hipSetDevice(h->device));
  for (int s = 0; s < n; s += h->G) {
    const int m = std::min(h->G, n - s);
    launch_network(h, reinterpret_cast<const Pos*>(d_pos) + s, nullptr, m, NET_FULL_LOGITS,
                   d_logits + (size_t)s * NUM_ACTIONS, d_values + s, nullptr, nullptr);
    HIPCHK(hipGetLastError());
  }
  HIPCHK(stream_wait(h));
  return check_err(h, false);   // batch evaluation: no memo hands these results on
}

// ---- fine-grained search API ----------------------------------------------------------------
extern "C" int mtaz_set_games(mtaz_engine* h, const uint32_t* roots, const int32_t* agents, const uint8_t* active, int n) {
  if (n > h->G) return set_err(MTAZ_E_CAPACITY, "n=%d > engine games %d", n, h->G);
  HIPCHK(hipSetDevice(h->device));
  std::vector<uint8_t> act(h->G, 0);
  std::vector<int32_t> ag(h->G, 0), zero(h->G, 0);
  std::vector<Pos> rt(h->G);
  for (int g = 0; g < n; ++g) {
    act[g] = active ? active[g] : 1;
    ag[g] = agents ? agents[g] : 0;
    rt[g] = pos_in(roots + 5 * g);
  }
  HIPCHK(hipMemcpyAsync(h->d.gm.root, rt.data(), h->G * sizeof(Pos), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d.gm.agent, ag.data(), h->G * 4, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d.gm.active, act.data(), h->G, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d.gm.nhist, zero.data(), h->G * 4, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d.gm.outcome, zero.data(), h->G * 4, hipMemcpyHostToDevice, h->stream));
  HIPCHK(stream_wait(h));
  h->last_root_k.clear();   // new roots: the next mtaz_set_noise needs a fresh mtaz_move_begin or strides
  return 0;
}

extern "C" int mtaz_get_games(mtaz_engine* h, uint32_t* roots, int32_t* agents, uint8_t* active, int32_t* outcome) {
  HIPCHK(hipSetDevice(h->device));
  if (roots) HIPCHK(hipMemcpyAsync(roots, h->d.gm.root, h->G * sizeof(Pos), hipMemcpyDeviceToHost, h->stream));
  if (agents) HIPCHK(hipMemcpyAsync(agents, h->d.gm.agent, h->G * 4, hipMemcpyDeviceToHost, h->stream));
  if (active) HIPCHK(hipMemcpyAsync(active, h->d.gm.active, h->G, hipMemcpyDeviceToHost, h->stream));
  if (outcome) HIPCHK(hipMemcpyAsync(outcome, h->d.gm.outcome, h->G * 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(stream_wait(h));
  return 0;
}

extern "C" int mtaz_clear_trees(mtaz_engine* h, const int32_t* trees, int n) {
  HIPCHK(hipSetDevice(h->device));
  std::vector<int32_t> all;
  if (!trees) {
    all.resize(2 * h->G);
    for (int i = 0; i < 2 * h->G; ++i) all[i] = i;
    trees = all.data();
    n = 2 * h->G;
  }
  if (n > 2 * h->G) return set_err(MTAZ_E_CAPACITY, "too many trees");
  for (int i = 0; i < n; ++i)
    if (trees[i] < 0 || trees[i] >= 2 * h->G) return set_err(MTAZ_E_FAIL, "tree index %d out of range", trees[i]);
  HIPCHK(hipMemcpyAsync(h->d_trees, trees, n * 4, hipMemcpyHostToDevice, h->stream));
  launch_reset_trees(h->d, h->d_trees, n, !all.empty(), h->stream);
  if (!all.empty()) ECHK(clear_batch_memo(h));   // all tables cleared (a new play): a new batch
  HIPCHK(hipGetLastError());
  HIPCHK(stream_wait(h));
  return 0;
}

extern "C" int mtaz_move_begin(mtaz_engine* h, int32_t* root_k, int32_t* root_new) {
  HIPCHK(hipSetDevice(h->device));
  launch_move_begin(h->d, h->stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(root_k, h->d.gm.root_k, h->G * 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(root_new, h->d.gm.root_new, h->G * 4, hipMemcpyDeviceToHost, h->stream));
  const int rc = check_err(h);   // (synchronises the stream)
  h->last_root_k.assign(root_k, root_k + h->G);
  return rc;
}

extern "C" int mtaz_set_noise(mtaz_engine* h, const double* noise, const int64_t* offsets, const int32_t* strides,
                              int64_t total) {
  HIPCHK(hipSetDevice(h->device));
  // per-game contiguous draws: the draw stride of game g is its vector length, the root's legal
  // count: strides[g], or (strides NULL) the counts of this move's mtaz_move_begin
  std::vector<int32_t> js(h->G, 0);
  if (strides) {
    for (int g = 0; g < h->G; ++g) js[g] = strides[g];
  } else {
    if ((int)h->last_root_k.size() != h->G)
      return set_err(MTAZ_E_FAIL, "mtaz_set_noise without strides needs mtaz_move_begin first");
    js = h->last_root_k;
  }
  HIPCHK(stream_wait(h));
  ECHK(ensure_noise(h, (size_t)std::max<int64_t>(total, 1)));
  if (total > 0) HIPCHK(hipMemcpyAsync(h->d.gm.noise, noise, total * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d.gm.noise_off, offsets, h->G * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d.gm.noise_js, js.data(), h->G * 4, hipMemcpyHostToDevice, h->stream));
  HIPCHK(stream_wait(h));
  return 0;
}

static int sim_gpu(mtaz_engine* h, int sim, int defer = 0, int cut = 0) {
  // timing: per wave four events on the engine stream: [select begin, leaf compaction begin,
  // network begin, network end]
  hipEvent_t em = nullptr, eb = nullptr, ee = nullptr;
  if (h->timing) {
    const size_t need = 4 * (size_t)(h->wave + 1);
    while (h->ev.size() < need) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      h->ev.push_back(e);
    }
    HIPCHK(hipEventRecord(h->ev[4 * h->wave], h->stream));
    em = h->ev[4 * h->wave + 1];
    eb = h->ev[4 * h->wave + 2];
    ee = h->ev[4 * h->wave + 3];
  }
  launch_select(h->d, sim, h->stream, h->wave < h->count_log_cap ? h->d_count_log + 3 * (size_t)h->wave : nullptr, em,
                defer, cut, 4 * h->ncu);
  launch_network(h, h->d.lf.pos, h->d.lf.count, h->G, NET_LEAVES, nullptr, nullptr, eb, ee);
  launch_backup(h->d, h->stream);
  HIPCHK(hipGetLastError());
  ++h->wave;
  return 0;
}

extern "C" int mtaz_simulate(mtaz_engine* h, int first_sim, int n_sims) {
  if (!h->weights_ok) return set_err(MTAZ_E_FAIL, "weights not set (mtaz_set_weights)");
  HIPCHK(hipSetDevice(h->device));
  for (int s = first_sim; s < first_sim + n_sims; ++s) ECHK(sim_gpu(h, s));
  return check_err(h);
}

extern "C" int mtaz_sim_select(mtaz_engine* h, int sim) {
  HIPCHK(hipSetDevice(h->device));
  launch_select(h->d, sim, h->stream);
  HIPCHK(hipGetLastError());
  return check_err(h);
}

extern "C" int mtaz_leaves_get(mtaz_engine* h, int32_t* count, uint32_t* pos, int32_t* game, int32_t* k, uint16_t* codes) {
  HIPCHK(hipSetDevice(h->device));
  int32_t c = 0;
  HIPCHK(hipMemcpyAsync(&c, h->d.lf.count, 4, hipMemcpyDeviceToHost, h->stream));
  launch_gather_leaf_codes(h->d, h->d_leaf_codes, h->d_leaf_k, h->stream);
  HIPCHK(stream_wait(h));
  *count = c;
  if (c > 0) {
    HIPCHK(hipMemcpyAsync(pos, h->d.lf.pos, c * sizeof(Pos), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(game, h->d.lf.game, c * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(k, h->d_leaf_k, c * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(codes, h->d_leaf_codes, (size_t)c * KMAX * 2, hipMemcpyDeviceToHost, h->stream));
  }
  HIPCHK(stream_wait(h));
  return 0;
}

extern "C" int mtaz_leaves_set(mtaz_engine* h, const float* P, const float* v, int count) {
  HIPCHK(hipSetDevice(h->device));
  if (count > 0) {
    HIPCHK(hipMemcpyAsync(h->d.lf.P, P, (size_t)count * KMAX * 4, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d.lf.v, v, count * 4, hipMemcpyHostToDevice, h->stream));
  }
  HIPCHK(stream_wait(h));
  return 0;
}

extern "C" int mtaz_sim_evaluate(mtaz_engine* h) {
  if (!h->weights_ok) return set_err(MTAZ_E_FAIL, "weights not set (mtaz_set_weights)");
  HIPCHK(hipSetDevice(h->device));
  launch_network(h, h->d.lf.pos, h->d.lf.count, h->G, NET_LEAVES, nullptr, nullptr, nullptr, nullptr);
  HIPCHK(hipGetLastError());
  return check_err(h);
}

extern "C" int mtaz_leaves_result(mtaz_engine* h, float* P, float* v, int count) {
  HIPCHK(hipSetDevice(h->device));
  int32_t c = 0;
  HIPCHK(hipMemcpyAsync(&c, h->d.lf.count, 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(stream_wait(h));
  if (count < c) return set_err(MTAZ_E_CAPACITY, "leaf batch holds %d leaves, buffer %d", c, count);
  if (c > 0) {
    HIPCHK(hipMemcpyAsync(P, h->d.lf.P, (size_t)c * KMAX * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(v, h->d.lf.v, c * 4, hipMemcpyDeviceToHost, h->stream));
  }
  HIPCHK(stream_wait(h));
  return c;
}

extern "C" int mtaz_sim_backup(mtaz_engine* h) {
  HIPCHK(hipSetDevice(h->device));
  launch_backup(h->d, h->stream);
  HIPCHK(hipGetLastError());
  return check_err(h);
}

extern "C" int mtaz_move_end(mtaz_engine* h, uint16_t* codes, uint32_t* visits, int32_t* k, int kout) {
  HIPCHK(hipSetDevice(h->device));
  if (kout > KMAX) kout = KMAX;
  launch_move_end(h->d, h->d_root_codes, h->d_root_visits, kout, h->stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(codes, h->d_root_codes, (size_t)h->G * kout * 2, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(visits, h->d_root_visits, (size_t)h->G * kout * 4, hipMemcpyDeviceToHost, h->stream));
  if (k) HIPCHK(hipMemcpyAsync(k, h->d.gm.root_k, h->G * 4, hipMemcpyDeviceToHost, h->stream));
  return check_err(h);
}

extern "C" int mtaz_apply(mtaz_engine* h, const int32_t* actions) {
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipMemcpyAsync(h->d_actions, actions, h->G * 4, hipMemcpyHostToDevice, h->stream));
  launch_apply(h->d, h->d_actions, h->stream);
  HIPCHK(hipGetLastError());
  return check_err(h);
}

static int read_tree_headers(mtaz_engine* h, int tree, std::vector<NodeHdr>& hd) {
  if (tree < 0 || tree >= 2 * h->G) return set_err(MTAZ_E_FAIL, "tree out of range");
  HIPCHK(hipSetDevice(h->device));
  int32_t nn = 0;
  HIPCHK(hipMemcpy(&nn, h->d.tr.n_nodes + tree, 4, hipMemcpyDeviceToHost));
  hd.resize(nn);
  if (nn) HIPCHK(hipMemcpy(hd.data(), h->d.tr.node_hdr + (size_t)tree * h->d.tr.NC, nn * sizeof(NodeHdr), hipMemcpyDeviceToHost));
  return 0;
}

// edges = the summed legal-list length of the tree's expanded (non-terminal) nodes
extern "C" int mtaz_tree_size(mtaz_engine* h, int tree, int32_t* nodes, int32_t* edges) {
  std::vector<NodeHdr> hd;
  ECHK(read_tree_headers(h, tree, hd));
  int64_t ne = 0;
  for (const NodeHdr& x : hd)
    if (!hdr_term(x)) ne += hdr_k(x);
  *nodes = (int32_t)hd.size();
  *edges = (int32_t)ne;
  return 0;
}

// Node i's children are written at [e0[i], e0[i] + k[i]) of the output arrays, node after node
// (the device places them in the tree's region or the shared pool; this view is compact).
extern "C" int mtaz_tree_get(mtaz_engine* h, int tree, uint32_t* pos, uint32_t* e0, uint16_t* k, uint8_t* term,
                             double* tval, uint16_t* codes, float* P, double* Q, uint32_t* N) {
  std::vector<NodeHdr> hd;
  ECHK(read_tree_headers(h, tree, hd));
  const int nn = (int)hd.size();
  const Trees& T = h->d.tr;
  if (nn) HIPCHK(hipMemcpy(pos, T.node_pos + (size_t)tree * T.NC, nn * sizeof(Pos), hipMemcpyDeviceToHost));
  uint32_t o = 0;
  for (int i = 0; i < nn; ++i) {
    const int kk = hdr_term(hd[i]) ? 0 : hdr_k(hd[i]);
    e0[i] = o;
    k[i] = (uint16_t)hdr_k(hd[i]);
    term[i] = hdr_term(hd[i]) ? 1 : 0;
    tval[i] = (double)hd[i].tval;
    if (kk) {
      const size_t s = hd[i].e0;
      HIPCHK(hipMemcpy(codes + o, T.e_code + s, kk * 2, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(P + o, T.e_P + s, kk * 4, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(Q + o, T.e_Q + s, kk * 8, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(N + o, T.e_N + s, kk * 4, hipMemcpyDeviceToHost));
    }
    o += kk;
  }
  return nn;
}

// Load table `tree` from the mtaz_tree_get layout (nodes in order; node i's children at
// [e0[i], e0[i] + k[i]) of codes / P / Q / N for non-terminal nodes).  The hash index, the visit
// sums and the node headers are rebuilt; child links start unset (k_select relinks them by lookup).
extern "C" int mtaz_tree_set(mtaz_engine* h, int tree, int n, const uint32_t* pos, const uint32_t* e0,
                             const uint16_t* k, const uint8_t* term, const double* tval, const uint16_t* codes,
                             const float* P, const double* Q, const uint32_t* N) {
  if (tree < 0 || tree >= 2 * h->G) return set_err(MTAZ_E_FAIL, "tree out of range");
  Trees& T = h->d.tr;
  if (n < 0 || n > T.NC) return set_err(MTAZ_E_CAPACITY, "%d nodes do not fit a table of %d", n, T.NC);
  HIPCHK(hipSetDevice(h->device));
  std::vector<Pos> np(n);
  std::vector<NodeHdr> hd(n);
  std::vector<uint32_t> hash(T.HC, 0u);
  const uint32_t ebase = (uint32_t)tree * (uint32_t)T.EC;
  // edges go to the table's own region while whole nodes fit there, the rest (from the first node
  // that does not fit on) to one block of the shared pool, as k_select spills
  int64_t ne = 0, nreg = 0;
  bool spill = false;
  std::vector<int64_t> off(n, 0);
  for (int i = 0; i < n; ++i) {
    np[i] = pos_in(pos + 5 * i);
    uint32_t s = pos_hash(np[i]) & (uint32_t)(T.HC - 1);
    while (hash[s]) s = (s + 1) & (uint32_t)(T.HC - 1);
    hash[s] = (uint32_t)i + 1;
    if (term[i]) {
      hd[i] = NodeHdr{0u, 0u, HDR_TERM, (float)tval[i]};
      continue;
    }
    uint64_t sum = 0;
    for (int c = 0; c < k[i]; ++c) sum += N[e0[i] + c];
    if (!spill && nreg + k[i] > T.EC) spill = true;
    off[i] = ne;
    if (!spill) nreg += k[i];
    hd[i] = NodeHdr{0u, (uint32_t)sum, (uint32_t)k[i], (float)tval[i]};
    ne += k[i];
  }
  const int64_t npool = ne - nreg;
  uint32_t q = 0;
  if (npool > 0) {   // one block of the pool (the stream is idle between moves: plain copies suffice)
    HIPCHK(stream_wait(h));
    HIPCHK(hipMemcpy(&q, T.pool_used, 4, hipMemcpyDeviceToHost));
    if ((uint64_t)q + (uint64_t)npool > (uint64_t)T.pool_cap)
      return set_err(MTAZ_E_CAPACITY, "%lld edges beyond the table region do not fit the edge pool (%u of %u used)",
                     (long long)npool, q, T.pool_cap);
    const uint32_t q2 = q + (uint32_t)npool;
    HIPCHK(hipMemcpy(T.pool_used, &q2, 4, hipMemcpyHostToDevice));
  }
  for (int i = 0; i < n; ++i)
    if (!term[i])
      hd[i].e0 = off[i] < nreg ? ebase + (uint32_t)off[i] : T.pool_base + q + (uint32_t)(off[i] - nreg);
  std::vector<uint16_t> ec(ne);
  std::vector<float> ep(ne);
  std::vector<double> eq(ne);
  std::vector<uint32_t> en(ne), ech(ne, NONE);
  for (int i = 0, o = 0; i < n; ++i) {
    if (term[i]) continue;
    for (int c = 0; c < k[i]; ++c, ++o) {
      ec[o] = codes[e0[i] + c];
      ep[o] = P[e0[i] + c];
      eq[o] = Q[e0[i] + c];
      en[o] = N[e0[i] + c];
    }
  }
  const uint32_t nn32 = (uint32_t)n, ne32 = (uint32_t)nreg;
  HIPCHK(hipMemcpy(T.node_pos + (size_t)tree * T.NC, np.data(), n * sizeof(Pos), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(T.node_hdr + (size_t)tree * T.NC, hd.data(), n * sizeof(NodeHdr), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(T.hash + (size_t)tree * T.HC, hash.data(), (size_t)T.HC * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(T.n_nodes + tree, &nn32, 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(T.n_edges + tree, &ne32, 4, hipMemcpyHostToDevice));
  // the region part at ebase, the pool part at pool_base + q
  for (int part = 0; part < 2; ++part) {
    const int64_t o = part ? nreg : 0, cnt = part ? npool : nreg;
    if (cnt <= 0) continue;
    const size_t d = part ? (size_t)T.pool_base + q : ebase;
    HIPCHK(hipMemcpy(T.e_code + d, ec.data() + o, cnt * 2, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(T.e_P + d, ep.data() + o, cnt * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(T.e_Q + d, eq.data() + o, cnt * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(T.e_N + d, en.data() + o, cnt * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(T.e_child + d, ech.data() + o, cnt * 4, hipMemcpyHostToDevice));
  }
  return 0;
}

extern "C" int mtaz_set_edge_capacity(mtaz_engine* h, int64_t per_tree, int64_t pool) {
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(stream_wait(h));
  for (mtaz_engine* p : h->parts) delete p;   // groups re-create their engines with the default
  h->parts.clear();
  ECHK(alloc_edges(h, per_tree, pool));
  return mtaz_clear_trees(h, nullptr, 0);
}

extern "C" int mtaz_set_timing(mtaz_engine* h, int on) {
  h->timing = on != 0;
  return 0;
}

// ---- batched self-play ------------------------------------------------------------------------
// Per move: move_begin -> host draws each game's Dirichlet vectors (numpy legacy, exact)
// -> `sims` GPU waves of select / network / backup with no host sync -> root visit
// counts -> host action choice (choice with p while fullmove < tau, else argmax with a
// random tie-break, exp/agent.py:110-119) -> apply on device.
// Full-batch self-play over h->groups game groups, one sub-engine (own stream, trees, leaf
// batch) and one host thread per group.  Sub-engine i plays global games
// [i*G/groups, (i+1)*G/groups) with seed_base + i*G/groups; records and counters are merged
// back in game order, so the result equals the single-group run.
static int play_groups(mtaz_engine* h) {
  const int ng = h->groups, Gp = h->G / ng;
  release_batch_memo(h);   // idle while the groups play (up to 2^26 slots of 222 B); mtaz_play re-creates it
  if (h->parts.empty()) {
    for (int i = 0; i < ng; ++i) {
      mtaz_engine* p = mtaz_create(h->device, Gp, h->sims, h->cpuct, h->tau, h->alpha, h->eps, 0, h->cast_mode,
                                   h->flags, h->move_cap);
      if (!p) return MTAZ_E_DEVICE;
      h->parts.push_back(p);
    }
  }
  for (int i = 0; i < ng; ++i) {
    mtaz_engine* p = h->parts[i];
    p->w = h->w;                 // borrowed device weights (owned by h)
    p->weights_ok = true;
    p->precision = h->precision;
    p->variant = h->variant;
    p->timing = h->timing;
    p->host_threads = std::max(1, h->host_threads / ng);   // the groups share this engine's threads
    p->sync_mode = h->sync_mode;
    p->defer = h->defer;
    p->rng_device = h->rng_device;
    p->schedule = h->schedule;
    p->memo = h->memo;
    p->d.pr.lag_order = h->d.pr.lag_order;
    ECHK(ensure_batch_memo(p));
    sync_memo(p);
    p->seed_base = h->seed_base + (uint64_t)i * Gp;
  }
  std::vector<int> rc(ng, 0);
  std::vector<std::string> err(ng);
  const double t0 = now_ms();
  // the group threads (and the host pools they own) persist across plays
  if (!h->group_pool || h->group_pool->size() != ng) h->group_pool.reset(new HostPool(ng));
  const std::function<void(int)> body = [&](int i) {
    rc[i] = mtaz_play(h->parts[i], Gp, 0);
    if (rc[i] < 0) err[i] = mtaz_last_error();
  };
  h->group_pool->run(ng, body);
  for (int i = 0; i < ng; ++i)
    if (rc[i] < 0) return set_err(rc[i], "group %d: %s", i, err[i].c_str());
  h->rec.resize(h->G);
  h->final_outcome.clear();
  for (int i = 0; i < ST_COUNT; ++i) h->stats[i] = 0;
  h->wave = 0;
  for (int pi = 0; pi < ng; ++pi) {
    mtaz_engine* p = h->parts[pi];
    for (int gi = 0; gi < Gp; ++gi) std::swap(h->rec[(size_t)pi * Gp + gi], p->rec[gi]);
    h->final_outcome.insert(h->final_outcome.end(), p->final_outcome.begin(), p->final_outcome.end());
    for (int i = 0; i < ST_COUNT; ++i) {
      if (i == ST_MAX_NODES || i == ST_MAX_EDGES || i == ST_NET_PREC || i == ST_MOVES || i == ST_RNG_DEVICE ||
          i == ST_SCHEDULE)
        h->stats[i] = std::max(h->stats[i], p->stats[i]);
      else if (i != ST_WALL_MS) h->stats[i] += p->stats[i];
    }
    h->wave += p->wave;
  }
  h->stats[ST_WALL_MS] = now_ms() - t0;
  h->n_played = h->G;
  return 0;
}

// the pinned per-move buffers of mtaz_play, one block for the engine's games
static int ensure_play_pinned(mtaz_engine* h) {
  if (h->pin_block) return 0;
  const size_t G = (size_t)h->G;
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
  const size_t o_r0 = take(G * 20), o_r1 = take(G * 20), o_a0 = take(G), o_a1 = take(G), o_ag = take(G * 4),
               o_oc = take(G * 4), o_rk = take(G * 4), o_rn = take(G * 4), o_ac = take(G * 4), o_js = take(G * 4),
               o_of = take(G * 8), o_co = take(G * KMAX * 2), o_vi = take(G * KMAX * 4);
  void* q = nullptr;
  HIPCHK(hipHostMalloc(&q, off, hipHostMallocDefault));
  h->pin_block = q;
  char* b = (char*)q;
  auto& P = h->pin;
  P.roots[0] = (uint32_t*)(b + o_r0);
  P.roots[1] = (uint32_t*)(b + o_r1);
  P.active[0] = (uint8_t*)(b + o_a0);
  P.active[1] = (uint8_t*)(b + o_a1);
  P.agents = (int32_t*)(b + o_ag);
  P.outcome = (int32_t*)(b + o_oc);
  P.root_k = (int32_t*)(b + o_rk);
  P.root_new = (int32_t*)(b + o_rn);
  P.actions = (int32_t*)(b + o_ac);
  P.js = (int32_t*)(b + o_js);
  P.offs = (int64_t*)(b + o_of);
  P.codes = (uint16_t*)(b + o_co);
  P.visits = (uint32_t*)(b + o_vi);
  return 0;
}

// ---- free-running moves (mtaz_set_schedule 1) ------------------------------
static int ensure_free_run(mtaz_engine* h) {
  Games& gm = h->d.gm;
  if (gm.rec_pos) return 0;
  const size_t G = (size_t)h->G;
  ECHK(h->dalloc(&gm.nply, G));
  ECHK(h->dalloc(&gm.ndraw, G));
  ECHK(h->dalloc(&gm.rec_cur, G));
  ECHK(h->dalloc(&gm.rec_pos, G * gm.PLY));
  ECHK(h->dalloc(&gm.rec_action, G * gm.PLY));
  ECHK(h->dalloc(&gm.rec_k, G * gm.PLY));
  ECHK(h->dalloc(&gm.rec_codes, G * (size_t)gm.RC));
  ECHK(h->dalloc(&gm.rec_visits, G * (size_t)gm.RC));
  ECHK(h->dalloc(&h->d_rec_off, G));
  HIPCHK(hipHostMalloc(&h->cnt_host, 4, hipHostMallocDefault));
  return 0;
}

// The play's waves with no per-move host step: each wave is k_turn (games whose move is complete
// record it, choose, step and start the next move, noise included) + select / leaf list / network /
// backup; the host reads the active-game count every W waves.  Every game runs the simulations of
// each move in order on the same tables, draws and network results as in lockstep, so the records
// are identical; only the wave each simulation runs in differs.  The records come from the device at
// the end.  -> moves = the longest game's plies.
static int play_free(mtaz_engine* h, int* moves, double* sync_ms, double* turn_ms) {
  const int G = h->G;
  Games& gm = h->d.gm;
  ECHK(ensure_free_run(h));
  ECHK(ensure_noise(h, (size_t)G * h->sims * KMAX));   // each game's region: sims draws x KMAX
  HIPCHK(hipMemsetAsync(gm.nply, 0, (size_t)G * 4, h->stream));
  HIPCHK(hipMemsetAsync(gm.rec_cur, 0, (size_t)G * 4, h->stream));
  HIPCHK(hipMemsetAsync(gm.simc, 0, (size_t)G * 4, h->stream));
  HIPCHK(hipMemsetAsync(h->d.lf.gnode, 0xff, (size_t)G * 4, h->stream));
  launch_turn(h->d, 1, h->stream);
  HIPCHK(hipGetLastError());
  constexpr int W = 16;   // waves between the host's reads of the active count
  for (;;) {
    for (int i = 0; i < W; ++i) {
      if (h->timing) {
        const size_t need = 2 * (size_t)(h->wave + 1);
        while (h->ev_turn.size() < need) {
          hipEvent_t e;
          HIPCHK(hipEventCreate(&e));
          h->ev_turn.push_back(e);
        }
        HIPCHK(hipEventRecord(h->ev_turn[2 * h->wave], h->stream));
      }
      launch_turn(h->d, 0, h->stream);
      if (h->timing) HIPCHK(hipEventRecord(h->ev_turn[2 * h->wave + 1], h->stream));
      ECHK(sim_gpu(h, 0, 1, h->defer));
    }
    launch_count_active(h->d, h->d_remaining, h->stream);
    HIPCHK(hipMemcpyAsync(h->cnt_host, h->d_remaining, 4, hipMemcpyDeviceToHost, h->stream));
    const double ts = now_ms();
    ECHK(check_err(h));   // (synchronises the stream)
    *sync_ms += now_ms() - ts;
    if (*h->cnt_host == 0) break;
    if (h->wave >= h->count_log_cap)
      return set_err(MTAZ_E_FAIL, "free-running moves: %d games still active after %d waves", *h->cnt_host, h->wave);
  }
  // the records: per game its plies, appended legal lists and visit counts packed game after game
  std::vector<int32_t> nply(G), cur(G), outc(G);
  HIPCHK(hipMemcpy(nply.data(), gm.nply, (size_t)G * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(cur.data(), gm.rec_cur, (size_t)G * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(outc.data(), gm.outcome, (size_t)G * 4, hipMemcpyDeviceToHost));
  std::vector<int64_t> off(G + 1, 0);
  for (int g = 0; g < G; ++g) off[g + 1] = off[g] + cur[g];
  const size_t tot = (size_t)std::max<int64_t>(off[G], 1);
  if (tot > h->pack_cap) {
    if (h->d_pack_codes) HIPCHK(hipFree(h->d_pack_codes));
    if (h->d_pack_visits) HIPCHK(hipFree(h->d_pack_visits));
    const size_t cap = std::max(tot, 2 * h->pack_cap);
    h->d_pack_codes = nullptr;
    h->d_pack_visits = nullptr;
    h->pack_cap = 0;
    HIPCHK(hipMalloc(&h->d_pack_codes, cap * 2));
    HIPCHK(hipMalloc(&h->d_pack_visits, cap * 4));
    h->pack_cap = cap;
  }
  HIPCHK(hipMemcpy(h->d_rec_off, off.data(), (size_t)G * 8, hipMemcpyHostToDevice));
  launch_rec_pack(h->d, h->d_rec_off, h->d_pack_codes, h->d_pack_visits, h->stream);
  HIPCHK(hipGetLastError());
  const size_t PLY = (size_t)gm.PLY;
  std::vector<Pos> rpos((size_t)G * PLY);
  std::vector<int32_t> ract((size_t)G * PLY), rk((size_t)G * PLY);
  std::vector<uint16_t> codes(tot);
  std::vector<uint32_t> visits(tot);
  HIPCHK(hipMemcpyAsync(rpos.data(), gm.rec_pos, rpos.size() * sizeof(Pos), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(ract.data(), gm.rec_action, ract.size() * 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(rk.data(), gm.rec_k, rk.size() * 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(codes.data(), h->d_pack_codes, tot * 2, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(visits.data(), h->d_pack_visits, tot * 4, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(stream_wait(h));
  parallel_for(G, h->host_threads, [&](int g) {
    int64_t e = off[g];
    for (int p = 0; p < nply[g]; ++p) {
      const size_t r = (size_t)g * PLY + p;
      h->rec[g].add(rpos[r], ract[r], codes.data() + e, visits.data() + e, rk[r]);
      e += rk[r];
    }
  });
  int mx = 0;
  double sims = 0;
  for (int g = 0; g < G; ++g) {
    h->final_outcome[g] = outc[g];
    mx = std::max(mx, nply[g]);
    sims += (double)nply[g] * h->sims;
  }
  *moves = mx;
  h->stats[ST_SIMS] = sims;
  h->stats[ST_EXTRA_WAVES] = std::max(0.0, (double)h->wave - (double)mx * h->sims);
  if (h->timing)
    for (int w = 0; w < h->wave; ++w) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, h->ev_turn[2 * w], h->ev_turn[2 * w + 1]));
      *turn_ms += ms;
    }
  return 0;
}

extern "C" int mtaz_play(mtaz_engine* h, int n_games, int from_current) {
  if (!h->weights_ok) return set_err(MTAZ_E_FAIL, "weights not set (mtaz_set_weights)");
  if (n_games > h->G || n_games <= 0) return set_err(MTAZ_E_CAPACITY, "n_games=%d (engine has %d)", n_games, h->G);
  const bool two_nets = h->agent_slot[0] != h->agent_slot[1];
  if (two_nets) {
    for (int a = 0; a < 2; ++a) {
      activate_slot(h, h->agent_slot[a]);
      if (!h->weights_ok) {
        activate_slot(h, 0);
        return set_err(MTAZ_E_FAIL, "two-network play: weight slot %d is empty", h->agent_slot[a]);
      }
    }
  }
  h->last_play_grouped = h->groups > 1 && !two_nets && !from_current && n_games == h->G;
  if (h->last_play_grouped) return play_groups(h);
  HIPCHK(hipSetDevice(h->device));
  ECHK(ensure_batch_memo(h));   // (released while pipeline groups played)
  const double t0 = now_ms();
  const int G = h->G;
  for (int i = 0; i < ST_COUNT; ++i) h->stats[i] = 0;
  if (!from_current) {
    uint32_t start[5];
    ECHK(mtaz_pos_from_fen("2nbk/2ppp/5/5/PPP2/KBN2 w 0 1", start));   // exp/environment.py:6
    std::vector<uint32_t> roots((size_t)G * 5);
    std::vector<uint8_t> act(G, 0);
    for (int g = 0; g < G; ++g) {
      memcpy(&roots[5 * g], start, 20);
      act[g] = g < n_games;
    }
    ECHK(mtaz_set_games(h, roots.data(), nullptr, act.data(), G));
  }
  ECHK(mtaz_clear_trees(h, nullptr, 0));
  const bool dev_rng = h->rng_device && h->alpha < 1.0;
  if (dev_rng) {
    launch_rng_seed(h->d, h->seed_base, h->stream);
    HIPCHK(hipGetLastError());
    if (h->timing)
      for (auto& e : h->rng_ev)
        if (!e) HIPCHK(hipEventCreate(&e));
  } else {
    for (int g = 0; g < G; ++g) mt_seed(h->rng[g], (uint32_t)(h->seed_base + (uint64_t)g));
  }
  h->rec.resize(G);
  for (auto& r : h->rec) r.clear();
  h->final_outcome.assign(G, 0);
  h->wave = 0;
  h->n_played = n_games;
  HIPCHK(hipMemsetAsync(h->d.gm.stot, 0, (size_t)G * 4, h->stream));
  const bool free_run = dev_rng && h->schedule == 1 && !two_nets;
  double rng_ms = 0, sync_ms = 0, choice_ms = 0, gap_ms = 0, rng_dev_ms = 0;
  int moves = 0;
  if (free_run) {
    ECHK(play_free(h, &moves, &sync_ms, &rng_dev_ms));
  } else {
  ECHK(ensure_play_pinned(h));
  auto& PP = h->pin;
  int cur = 0;   // PP.roots[cur] / PP.active[cur]: this move's game states
  uint32_t* roots = PP.roots[0];
  uint8_t* active = PP.active[0];
  int32_t *agents = PP.agents, *outcome_v = PP.outcome, *root_k = PP.root_k, *root_new = PP.root_new;
  int32_t *actions = PP.actions, *js = PP.js;
  int64_t* offs = PP.offs;
  uint16_t* codes = PP.codes;
  uint32_t* visits = PP.visits;
  for (int g = 0; g < G; ++g) actions[g] = 0;
  ECHK(mtaz_get_games(h, roots, agents, active, outcome_v));
  double t_gap = -1;   // when the last move's root visit counts reached the host
  for (;;) {
    int n_active = 0;
    for (int g = 0; g < G; ++g) n_active += active[g];
    if (!n_active) break;
    if (two_nets) {   // lockstep games: every active game has the same agent to move
      int a = -1;
      for (int g = 0; g < G; ++g)
        if (active[g]) {
          if (a >= 0 && agents[g] != a) return set_err(MTAZ_E_FAIL, "two-network play needs games in lockstep");
          a = agents[g];
        }
      activate_slot(h, h->agent_slot[a]);
    }
    double ts = now_ms();
    ECHK(mtaz_move_begin(h, root_k, root_new));
    sync_ms += now_ms() - ts;
    // Dirichlet draws: sims - root_new vectors of size k per active game, draw-major (draw j of
    // every game in one block of K = sum k), generated and uploaded in chunks of NCH draws so
    // that the host draws chunk c + 1 while the GPU runs the simulations of chunk c.  Each
    // game's generator still runs its draws in order (exp/agent.py:82), so the streams are
    // unchanged.
    double tr = now_ms();
    int64_t K = 0;
    for (int g = 0; g < G; ++g) {
      offs[g] = K;
      if (active[g]) K += root_k[g];
    }
    const size_t need = (size_t)std::max<int64_t>(K, 1) * h->sims;
    ECHK(ensure_noise(h, need));   // (mtaz_move_begin synchronised the stream)
    if (!dev_rng && need > h->noise_host_cap) {
      // grown geometrically, as the device buffer: pinning a fresh buffer costs ~4 ms, and the
      // legal counts grow over a game's first moves (round 5a regrew it on about twenty of them)
      const size_t cap = std::max(need, 2 * h->noise_host_cap);
      if (h->noise_host) HIPCHK(hipHostFree(h->noise_host));
      h->noise_host = nullptr;
      h->noise_host_cap = 0;
      HIPCHK(hipHostMalloc(&h->noise_host, cap * 8, hipHostMallocDefault));
      h->noise_host_cap = cap;
    }
    for (int g = 0; g < G; ++g) js[g] = (int32_t)K;
    HIPCHK(hipMemcpyAsync(h->d.gm.noise_off, offs, G * 8, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->d.gm.noise_js, js, G * 4, hipMemcpyHostToDevice, h->stream));
    if (dev_rng) {
      // every game's draws of the move in one launch, in stream order, ahead of its simulations
      if (h->timing) HIPCHK(hipEventRecord(h->rng_ev[0], h->stream));
      launch_noise(h->d, h->stream);
      HIPCHK(hipGetLastError());
      if (h->timing) HIPCHK(hipEventRecord(h->rng_ev[1], h->stream));
    }
    // chunks [0, 1), [1, 3), [3, 7), [7, 15), [15, 23), ...: the GPU starts after one draw per game,
    // and each later chunk is drawn while the previous chunk's simulations run.  The chunks double
    // up to 8 draws so that a chunk's draws never take longer than the simulations they overlap:
    // a draw of every game costs about a fifth of a wave on 2 host threads (the 8-rank share), and
    // round 4's [1, 9) after a single wave left the GPU idle for ~2 ms per move there
    constexpr int NCH = 8;
    auto chunk_end = [&](int j0) { return std::min(j0 + std::min(NCH, j0 + 1), h->sims); };
    auto draw_chunk = [&](int j0) {   // draws [j0, chunk_end(j0)) of every active game
      const int je = chunk_end(j0);
      if (dev_rng) return 0;
      parallel_for(G, h->host_threads, [&](int g) {
        if (!active[g]) return;
        const int k = root_k[g], jn = std::min(je, h->sims - root_new[g]);
        for (int j = j0; j < jn; ++j) legacy_dirichlet(h->rng[g], h->alpha, k, h->noise_host + (size_t)j * K + offs[g]);
      });
      if (je > j0 && K > 0)
        HIPCHK(hipMemcpyAsync(h->d.gm.noise + (size_t)j0 * K, h->noise_host + (size_t)j0 * K, (size_t)(je - j0) * K * 8,
                              hipMemcpyHostToDevice, h->stream));
      return 0;
    };
    ECHK(draw_chunk(0));
    rng_ms += now_ms() - tr;
    // host time between two moves' simulations: action choice, apply, game states, move start,
    // the first chunk of Dirichlet draws (the GPU idles meanwhile)
    if (t_gap >= 0) gap_ms += now_ms() - t_gap;
    for (int s0 = 0; s0 < h->sims; s0 = chunk_end(s0)) {
      // simulation s uses draw s - root_new <= s: the chunk holding draw s is on the stream first
      // (with deferred tails a game runs simulation s in wave s or later)
      for (int s = s0; s < chunk_end(s0); ++s) ECHK(sim_gpu(h, s, h->defer ? 1 : 0, h->defer));
      if (chunk_end(s0) < h->sims) {
        tr = now_ms();
        ECHK(draw_chunk(chunk_end(s0)));
        rng_ms += now_ms() - tr;
      }
    }
    if (h->defer) {
      // deferred tails: the waves the games still need (simulations not yet started, a leaf still
      // pending), each evaluating every leaf, so that every game ends the move with `sims` simulations
      // (deferring too, so that they also run whole rounds; a game with a leaf pending or a
      // simulation left needs at least one more wave, so every round of this loop makes progress)
      for (int extra = 0;;) {
        ts = now_ms();
        launch_remaining(h->d, h->d_remaining, h->stream);
        int32_t rem = 0;
        HIPCHK(hipMemcpyAsync(&rem, h->d_remaining, 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(stream_wait(h));
        sync_ms += now_ms() - ts;
        if (rem == 0) break;
        if (extra + rem > 4 * h->sims + 8) return set_err(MTAZ_E_FAIL, "deferred tails: %d waves pending after %d", rem, extra);
        for (int i = 0; i < rem; ++i, ++extra) ECHK(sim_gpu(h, h->sims + extra, 1, h->defer));
        h->stats[ST_EXTRA_WAVES] += rem;
      }
    }
    // root visit counts, rows of the longest active legal list (not KMAX: 8x fewer bytes to the host)
    int kmx = 1;
    for (int g = 0; g < G; ++g)
      if (active[g]) kmx = std::max(kmx, root_k[g]);
    ts = now_ms();
    if (dev_rng) {
      // action choice on the device from the root rows k_move_end leaves in HBM; the rows and the
      // actions then come to the host (records) with the move's one sync
      launch_move_end(h->d, h->d_root_codes, h->d_root_visits, kmx, h->stream);
      if (h->timing) HIPCHK(hipEventRecord(h->rng_ev[2], h->stream));
      launch_choose(h->d, h->d_root_codes, h->d_root_visits, kmx, h->d_actions, h->stream);
      if (h->timing) HIPCHK(hipEventRecord(h->rng_ev[3], h->stream));
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(codes, h->d_root_codes, (size_t)G * kmx * 2, hipMemcpyDeviceToHost, h->stream));
      HIPCHK(hipMemcpyAsync(visits, h->d_root_visits, (size_t)G * kmx * 4, hipMemcpyDeviceToHost, h->stream));
      HIPCHK(hipMemcpyAsync(actions, h->d_actions, G * 4, hipMemcpyDeviceToHost, h->stream));
      ECHK(check_err(h));
      if (h->timing) {
        float a = 0, b = 0;
        HIPCHK(hipEventElapsedTime(&a, h->rng_ev[0], h->rng_ev[1]));
        HIPCHK(hipEventElapsedTime(&b, h->rng_ev[2], h->rng_ev[3]));
        rng_dev_ms += a + b;
      }
    } else {
      ECHK(mtaz_move_end(h, codes, visits, nullptr, kmx));
    }
    sync_ms += now_ms() - ts;
    t_gap = now_ms();
    // action selection (exp/agent.py:110-119)
    tr = now_ms();
    if (!dev_rng) parallel_for(G, h->host_threads, [&](int g) {
      if (!active[g]) return;
      const int k = root_k[g];
      const uint16_t* c = codes + (size_t)g * kmx;
      const uint32_t* v = visits + (size_t)g * kmx;
      double pi[KMAX];
      double sum = 0;
      for (int i = 0; i < k; ++i) sum += (double)v[i];
      for (int i = 0; i < k; ++i) pi[i] = (double)v[i] / sum;
      const int fullmove = (int)(roots[5 * g + 4] >> 16);
      int idx;
      if (fullmove < h->tau) {
        idx = (int)legacy_choice_p(h->rng[g], pi, k);
      } else {
        double mx = pi[0];
        for (int i = 1; i < k; ++i) mx = std::max(mx, pi[i]);
        int maxima[KMAX], m = 0;
        for (int i = 0; i < k; ++i)
          if (pi[i] == mx) maxima[m++] = i;
        idx = maxima[legacy_randint(h->rng[g], m)];
      }
      actions[g] = c[idx];
    });
    rng_ms += now_ms() - tr;
    choice_ms += now_ms() - tr;
    // the actions applied on the GPU and the next states on their way back while the host appends
    // this move's records (exp/callbacks.py:40-47) from this move's buffers
    ts = now_ms();
    const int nxt = cur ^ 1;
    if (!dev_rng) HIPCHK(hipMemcpyAsync(h->d_actions, actions, G * 4, hipMemcpyHostToDevice, h->stream));
    launch_apply(h->d, h->d_actions, h->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(PP.roots[nxt], h->d.gm.root, (size_t)G * sizeof(Pos), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(agents, h->d.gm.agent, G * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(PP.active[nxt], h->d.gm.active, G, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipMemcpyAsync(outcome_v, h->d.gm.outcome, G * 4, hipMemcpyDeviceToHost, h->stream));
    parallel_for(G, h->host_threads, [&](int g) {
      if (!active[g]) return;
      h->rec[g].add(pos_in(&roots[5 * g]), actions[g], codes + (size_t)g * kmx, visits + (size_t)g * kmx, root_k[g]);
    });
    ECHK(check_err(h));   // (synchronises the stream: the apply's flags and the states are in)
    cur = nxt;
    roots = PP.roots[cur];
    active = PP.active[cur];
    sync_ms += now_ms() - ts;
    h->stats[ST_SIMS] += (double)n_active * h->sims;
    ++moves;
  }
  if (two_nets) activate_slot(h, 0);
  for (int g = 0; g < G; ++g) h->final_outcome[g] = outcome_v[g];
  }   // lockstep
  // stats
  const int nlog = std::min(h->wave, h->count_log_cap);
  std::vector<int32_t> clog(3 * (size_t)nlog), counts(nlog);
  if (nlog) HIPCHK(hipMemcpy(clog.data(), h->d_count_log, clog.size() * 4, hipMemcpyDeviceToHost));
  double evals = 0, hits = 0, bhits = 0;
  for (int wv = 0; wv < nlog; ++wv) {
    counts[wv] = clog[3 * wv];
    evals += clog[3 * wv];
    hits += clog[3 * wv + 1];
    bhits += clog[3 * wv + 2];
  }
  double trunk_ms = 0, trunk_boards = 0, select_ms = 0, compact_ms = 0;
  if (h->timing) {
    for (int wv = 0; wv < h->wave && wv < (int)counts.size(); ++wv) {
      float ms = 0, sms = 0, cms = 0;
      HIPCHK(hipEventElapsedTime(&ms, h->ev[4 * wv + 2], h->ev[4 * wv + 3]));
      HIPCHK(hipEventElapsedTime(&sms, h->ev[4 * wv], h->ev[4 * wv + 1]));
      HIPCHK(hipEventElapsedTime(&cms, h->ev[4 * wv + 1], h->ev[4 * wv + 2]));
      trunk_ms += ms;
      select_ms += sms;
      compact_ms += cms;
      trunk_boards += counts[wv];
    }
  }
  int64_t plies = 0, decisive = 0;
  for (int g = 0; g < n_games; ++g) {
    plies += (int64_t)h->rec[g].plies();
    decisive += h->final_outcome[g] == DECISIVE;
  }
  // largest table of the batch (device error flags already guard the capacities)
  int32_t mxn = 0, mxe = 0;
  {
    std::vector<int32_t> nn(2 * n_games), ne(2 * n_games);
    HIPCHK(hipMemcpy(nn.data(), h->d.tr.n_nodes, nn.size() * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(ne.data(), h->d.tr.n_edges, ne.size() * 4, hipMemcpyDeviceToHost));
    for (size_t t = 0; t < nn.size(); ++t) mxn = std::max(mxn, nn[t]), mxe = std::max(mxe, ne[t]);
  }
  h->stats[ST_PLIES] = (double)plies;
  h->stats[ST_NN_EVALS] = evals;                              // network evaluations computed
  h->stats[ST_MEMO_HITS] = hits + bhits;                      // leaves the memo supplied
  h->stats[ST_MEMO_BATCH_HITS] = bhits;                       //   of which from the batch memo
  h->stats[ST_TERMINAL_SIMS] = h->stats[ST_SIMS] - evals - hits - bhits;
  h->stats[ST_TRUNK_MS] = trunk_ms;
  h->stats[ST_TRUNK_BOARDS] = trunk_boards;
  h->stats[ST_WAVES] = h->wave;
  h->stats[ST_HOST_RNG_MS] = rng_ms;
  h->stats[ST_WALL_MS] = now_ms() - t0;
  h->stats[ST_GAMES] = n_games;
  h->stats[ST_DECISIVE] = (double)decisive;
  h->stats[ST_MOVES] = moves;
  h->stats[ST_TRUNK_LAUNCHES] = h->timing ? 18.0 * h->wave : 0;
  h->stats[ST_MAX_NODES] = mxn;
  h->stats[ST_MAX_EDGES] = mxe;
  {
    uint32_t pu = 0;
    HIPCHK(hipMemcpy(&pu, h->d.tr.pool_used, 4, hipMemcpyDeviceToHost));
    h->stats[ST_POOL_EDGES] = pu;
  }
  h->stats[ST_SYNC_MS] = sync_ms;
  h->stats[ST_NET_PREC] = h->precision;
  h->stats[ST_SELECT_MS] = select_ms;
  h->stats[ST_CHOICE_MS] = choice_ms;
  h->stats[ST_GAP_MS] = gap_ms;
  h->stats[ST_COMPACT_MS] = compact_ms;
  h->stats[ST_RNG_DEVICE] = dev_rng ? 1 : 0;
  h->stats[ST_RNG_DEV_MS] = rng_dev_ms;
  h->stats[ST_SCHEDULE] = free_run ? 1 : 0;
  return 0;
}

extern "C" int mtaz_stats(mtaz_engine* h, double* out, int n) {
  h->stats[ST_NODE_CAP] = h->d.tr.NC;   // per-table capacities (engine_alloc)
  h->stats[ST_EDGE_CAP] = h->d.tr.EC;
  h->stats[ST_POOL_CAP] = h->d.tr.pool_cap;
  for (int i = 0; i < n && i < ST_COUNT; ++i) out[i] = h->stats[i];
  return ST_COUNT;
}

extern "C" int mtaz_records_counts(mtaz_engine* h, int32_t* plies_per_game, int64_t* total_plies, int64_t* total_entries) {
  int64_t tp = 0, te = 0;
  for (int g = 0; g < h->n_played; ++g) {
    plies_per_game[g] = (int32_t)h->rec[g].plies();
    tp += (int64_t)h->rec[g].plies();
    te += (int64_t)h->rec[g].codes.size();
  }
  *total_plies = tp;
  *total_entries = te;
  return 0;
}

// reward back-fill as exp/callbacks.py:49-54: last step's reward (1.0 decisive, 0.0 draw),
// alternating sign towards the first step.
extern "C" int mtaz_records_get(mtaz_engine* h, uint32_t* pos, int32_t* action, int32_t* k, uint16_t* codes,
                                uint32_t* visits, float* reward, int32_t* outcome_out) {
  int64_t p = 0, e = 0;
  for (int g = 0; g < h->n_played; ++g) {
    const auto& R = h->rec[g];
    const int oc = h->final_outcome[g];
    if (outcome_out) outcome_out[g] = oc;
    const int np = (int)R.plies();
    // the last ply's reward is the game's (1 decisive, 0 draw), alternating in sign towards ply 0
    float rw = ((np - 1) & 1) ? -(oc == DECISIVE ? 1.0f : 0.0f) : (oc == DECISIVE ? 1.0f : 0.0f);
    for (int i = 0; i < np; ++i, ++p) {
      pos_out(R.pos[i], pos + 5 * p);
      action[p] = R.action[i];
      k[p] = R.k[i];
      reward[p] = rw;
      rw = -rw;
    }
    memcpy(codes + e, R.codes.data(), R.codes.size() * 2);
    memcpy(visits + e, R.visits.data(), R.visits.size() * 4);
    e += (int64_t)R.codes.size();
  }
  return 0;
}
