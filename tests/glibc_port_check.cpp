// CPU pin of csrc/glibc_math.h (TEST INFRASTRUCTURE; built and run by tests/test_glibc_port_cpu.py):
// the host build of the port must equal this machine's glibc `log` and `pow` bit for bit.
//
//   glibc_port_check N SEED   ->  one JSON line {"case": mismatches, ...}; exit 1 on any mismatch
//
// Cases (N arguments each, a splitmix64 stream seeded with SEED):
//   log_sampler   log(1 - U), U = numpy's legacy double (a*2^26 + b) / 2^53 from two 32-bit words:
//                 legacy_standard_exponential's argument (legacy-distributions.c)
//   log_ratio     log((1 - U) / 0.6) for U > 0.4: the gamma sampler's second branch (shape 0.6)
//   log_general   random positive doubles (bit patterns over the normal and subnormal range)
//   pow_low       pow(U, 1 / 0.6) for U <= 0.4 (the first branch)
//   pow_high      pow(1 - 0.6 + 0.6 * Y, 1 / 0.6), Y = -log((1 - U) / 0.6), U > 0.4 (the second branch)
//   pow_general   x random positive in [2^-200, 2^200], y random in [-40, 40] (results from subnormal
//                 to large, the exp specialcase included)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define MTAZ_GLIBC_FN static inline
#define MTAZ_GLIBC_CONST static const
#include "../minitchess_alphazero_amd/csrc/glibc_math.h"

static uint64_t sm_state;
static uint64_t splitmix() {
  uint64_t z = (sm_state += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static double legacy_double_bits() {
  const uint32_t w0 = (uint32_t)splitmix(), w1 = (uint32_t)splitmix();
  const int32_t a = (int32_t)(w0 >> 5), b = (int32_t)(w1 >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}
static int same(double a, double b) { return glibc_asu64(a) == glibc_asu64(b); }

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  sm_state = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
  const double shape = 0.6, inv = 1. / shape;
  long bad[6] = {0, 0, 0, 0, 0, 0}, cnt[6] = {0, 0, 0, 0, 0, 0};
  int shown = 0;
#define CHECK(ci, fn, ref, got)                                                                    \
  do {                                                                                             \
    ++cnt[ci];                                                                                     \
    if (!same(ref, got)) {                                                                         \
      ++bad[ci];                                                                                   \
      if (shown++ < 8) fprintf(stderr, "%s: ref %a got %a\n", fn, ref, got);                       \
    }                                                                                              \
  } while (0)
  for (long i = 0; i < n; ++i) {
    const double U = legacy_double_bits();
    const double x0 = 1.0 - U;
    CHECK(0, "log_sampler", log(x0), glibc_log(x0));
    double U2 = legacy_double_bits();
    if (U2 <= 1.0 - shape) U2 = 1.0 - U2 * (1.0 - shape) / (1.0 - shape) * 0.999999;   // into (0.4, 1)
    if (U2 > 1.0 - shape) {
      const double x1 = (1 - U2) / shape;
      CHECK(1, "log_ratio", log(x1), glibc_log(x1));
      const double Y = -log(x1);
      const double b = 1.0 - shape + shape * Y;
      CHECK(4, "pow_high", pow(b, inv), glibc_pow(b, inv));
    }
    uint64_t r = splitmix() & 0x7fffffffffffffffull;
    if ((r >> 52) == 0x7ff) r &= 0x7fefffffffffffffull;
    const double xg = glibc_asdbl(r);
    if (xg > 0) CHECK(2, "log_general", log(xg), glibc_log(xg));
    const double U3 = legacy_double_bits() * (1.0 - shape);
    CHECK(3, "pow_low", pow(U3, inv), glibc_pow(U3, inv));
    const double xp = ldexp(1.0 + (double)(splitmix() >> 12) * 0x1p-52, (int)(splitmix() % 401) - 200);
    const double yp = ((double)(splitmix() >> 11) * 0x1p-53 - 0.5) * 80.0;
    if (fabs(yp) >= 0x1p-65) CHECK(5, "pow_general", pow(xp, yp), glibc_pow(xp, yp));
  }
  const char* names[6] = {"log_sampler", "log_ratio", "log_general", "pow_low", "pow_high", "pow_general"};
  long tot = 0;
  printf("{");
  for (int c = 0; c < 6; ++c) {
    printf("%s\"%s\": [%ld, %ld]", c ? ", " : "", names[c], bad[c], cnt[c]);
    tot += bad[c];
  }
  printf("}\n");
  return tot ? 1 : 0;
}
