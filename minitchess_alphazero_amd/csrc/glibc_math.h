// Bit-exact port of glibc 2.35's `log` and `pow` as numpy's legacy gamma sampler calls them on this
// image (the Dirichlet noise of exp/agent.py:82 on the device).
//
// numpy's legacy_standard_gamma (numpy/random/src/legacy/legacy-distributions.c) calls the C
// library's log and pow.  glibc's x86_64 ifunc picks the FMA builds of sysdeps/ieee754/dbl-64/e_log.c
// and e_pow.c (ARM optimized-routines, table-driven, ~0.52 ULP: not correctly rounded, so only the same
// algorithm with the same tables and the same rounding steps reproduces them).  gcc contracted some of
// their a*b+c expressions into FMAs in those builds; the sequences below follow the instruction
// sequences of libm.so.6's __log_fma / __pow_fma (disassembled with llvm-objdump): every fma() here is
// one vfmadd/vfmsub/vfnmadd there, every other operation one IEEE double add/sub/mul, nothing contracted
// beyond that (MTAZ_GLIBC_NOCONTRACT).  The tables come from the same libm (tools/glibc_tables.py ->
// glibc_math_tables.h).  tests/test_glibc_port_cpu.py checks a host build of this file against the
// machine's glibc log and pow bitwise on 10^8 arguments each (the gamma loop's ranges and general ones);
// tests/test_gpu_rng.py checks the device build's Dirichlet draws against numpy.random.RandomState.
//
// Include with MTAZ_GLIBC_FN (function qualifiers) and MTAZ_GLIBC_CONST (table qualifiers) defined:
// host: `static inline` / `static const`; device: `static __device__ __forceinline__` /
// `static __device__ const`.
#pragma once
#include <stdint.h>

#include "glibc_math_tables.h"

#if defined(__clang__)
#define MTAZ_GLIBC_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define MTAZ_GLIBC_NOCONTRACT   // gcc: build with -ffp-contract=off
#endif

MTAZ_GLIBC_FN uint64_t glibc_asu64(double x) { return __builtin_bit_cast(uint64_t, x); }
MTAZ_GLIBC_FN double glibc_asdbl(uint64_t u) { return __builtin_bit_cast(double, u); }
MTAZ_GLIBC_FN double glibc_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }

// log (e_log.c, __log_fma).  Returns NaN for x < 0 and -inf for 0 without raising (errno and flags are
// not modelled: the sampler's arguments are in (0, 1]).
MTAZ_GLIBC_FN double glibc_log(double x) {
  MTAZ_GLIBC_NOCONTRACT
  const double* A = g_log_poly;
  const double* B = g_log_poly1;
  const double ln2hi = 0x1.62e42fefa3800p-1, ln2lo = 0x1.ef35793c76730p-45;
  uint64_t ix = glibc_asu64(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  if (ix - 0x3fee000000000000ull < 0x3090000000000ull) {   // 1 - 2^-4 <= x < 1 + 0x1.09p-4
    if (ix == 0x3ff0000000000000ull) return 0;
    const double r = x - 1.0;
    const double r2 = r * r;
    const double r3 = r * r2;
    double q1 = glibc_fma(r, B[2], B[1]);
    double q2 = glibc_fma(r, B[5], B[4]);
    double q3 = glibc_fma(r, B[8], B[7]);
    q1 = glibc_fma(r2, B[3], q1);
    q2 = glibc_fma(r2, B[6], q2);
    q3 = glibc_fma(r2, B[9], q3);
    q3 = glibc_fma(r3, B[10], q3);
    double y = glibc_fma(q3, r3, q2);
    y = glibc_fma(y, r3, q1);
    // rhi = r + w - w with w = r * 2^27, contracted as fma(r, 2^27, r) - r * 2^27
    const double t = glibc_fma(r, 0x1p27, r);
    const double rhi = glibc_fma(-0x1p27, r, t);
    const double rhi2 = rhi * rhi;
    const double rlo = r - rhi;
    const double hi = glibc_fma(rhi2, B[0], r);
    double lo = glibc_fma(rhi2, B[0], r - hi);
    lo = glibc_fma(B[0] * rlo, r + rhi, lo);
    y = glibc_fma(y, r3, lo);
    return hi + y;
  }
  if (top - 0x0010u >= 0x7ff0u - 0x0010u) {
    if (ix * 2 == 0) return -__builtin_inf();
    if (ix == 0x7ff0000000000000ull) return x;
    if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return __builtin_nan("");
    ix = glibc_asu64(x * 0x1p52);   // subnormal: normalise
    ix -= 52ull << 52;
  }
  const uint64_t tmp = ix - 0x3fe6000000000000ull;
  const int i = (int)((tmp >> 45) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = glibc_asdbl(iz);
  const double kd = (double)k;
  const double r = glibc_fma(z, g_log_invc[i], -1.0);
  const double w = glibc_fma(kd, ln2hi, g_log_logc[i]);
  const double q1 = glibc_fma(r, A[2], A[1]);
  const double hi = r + w;
  const double r2 = r * r;
  double lo = (w - hi) + r;
  lo = glibc_fma(kd, ln2lo, lo);
  const double r3 = r * r2;
  const double q2 = glibc_fma(r, A[4], A[3]);
  const double lo2 = glibc_fma(r2, A[0], lo);
  const double q = glibc_fma(q2, r2, q1);
  const double y = glibc_fma(r3, q, lo2);
  return y + hi;
}

// pow's log_inline: log(x) = hi + *tail with ~15 extra bits (e_pow.c, FMA build).
MTAZ_GLIBC_FN double glibc_pow_log(uint64_t ix, double* tail) {
  MTAZ_GLIBC_NOCONTRACT
  const double* A = g_pow_poly;
  const double ln2hi = 0x1.62e42fefa3800p-1, ln2lo = 0x1.ef35793c76730p-45;
  const uint64_t tmp = ix - 0x3fe6955500000000ull;
  const int i = (int)((tmp >> 45) & 127);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double z = glibc_asdbl(iz);
  const double kd = (double)k;
  const double t1 = glibc_fma(kd, ln2hi, g_pow_logc[i]);
  const double r = glibc_fma(z, g_pow_invc[i], -1.0);
  const double ar = r * A[0];
  const double lo1 = glibc_fma(kd, ln2lo, g_pow_logctail[i]);
  const double p1 = glibc_fma(r, A[2], A[1]);
  const double p2 = glibc_fma(r, A[4], A[3]);
  const double t2 = r + t1;
  const double ar2 = r * ar;
  const double d = t1 - t2;
  const double ar3 = r * ar2;
  const double lo3 = glibc_fma(ar, r, -ar2);
  const double lo2 = d + r;
  double p3 = glibc_fma(r, A[6], A[5]);
  const double hi = t2 + ar2;
  const double e = t2 - hi;
  p3 = glibc_fma(p3, ar2, p2);
  const double lo4 = e + ar2;
  const double p = glibc_fma(ar2, p3, p1);
  double s = lo1 + lo2;
  s = s + lo3;
  s = s + lo4;
  const double lo = glibc_fma(ar3, p, s);
  const double y = hi + lo;
  *tail = (hi - y) + lo;
  return y;
}

// exp_inline(x, xtail) with sign_bias 0 (e_pow.c; EXP_TABLE_BITS 7, EXP_POLY_ORDER 5).
MTAZ_GLIBC_FN double glibc_pow_exp(double x, double xtail) {
  MTAZ_GLIBC_NOCONTRACT
  const double* C = g_exp_poly;   // C2..C5
  uint32_t abstop = (uint32_t)(glibc_asu64(x) >> 52) & 0x7ffu;
  if (abstop - 0x3c9u >= 0x408u - 0x3c9u) {
    if ((int32_t)(abstop - 0x3c9u) < 0) return 1.0 + x;   // |x| < 2^-54
    if (abstop >= 0x409u) return (glibc_asu64(x) >> 63) ? 0.0 : __builtin_inf();   // under/overflow
    abstop = 0;   // large |x|: specialcase below
  }
  const double kds = glibc_fma(x, g_exp_invln2N, g_exp_shift);
  const uint64_t ki = glibc_asu64(kds);
  const double kd = kds - g_exp_shift;
  double r = glibc_fma(kd, g_exp_negln2hiN, x);
  r = glibc_fma(kd, g_exp_negln2loN, r);
  const int idx = 2 * (int)(ki & 127);
  const uint64_t top = ki << 45;
  uint64_t sbits = g_exp_tab[idx + 1] + top;
  r = xtail + r;
  double c = glibc_fma(r, C[1], C[0]);
  const double tr = r + glibc_asdbl(g_exp_tab[idx]);
  const double r2 = r * r;
  const double c45 = glibc_fma(r, C[3], C[2]);
  c = glibc_fma(c, r2, tr);
  const double r4 = r2 * r2;
  const double tmp = glibc_fma(c45, r4, c);
  if (abstop == 0) {   // specialcase(tmp, sbits, ki)
    if ((ki & 0x80000000ull) == 0) {
      sbits -= 1009ull << 52;
      const double scale = glibc_asdbl(sbits);
      return 0x1p1009 * glibc_fma(scale, tmp, scale);
    }
    sbits += 1022ull << 52;
    const double scale = glibc_asdbl(sbits);
    const double st = scale * tmp;
    double y = scale + st;
    if (__builtin_fabs(y) < 1.0) {
      const double one = y < 0.0 ? -1.0 : 1.0;
      const double lo = (scale - y) + st;
      const double hi = y + one;
      double l2 = (one - hi) + y;
      l2 = l2 + lo;
      y = (l2 + hi) - one;
      if (y == 0) y = glibc_asdbl(sbits & 0x8000000000000000ull);
    }
    return 0x1p-1022 * y;
  }
  const double scale = glibc_asdbl(sbits);
  return glibc_fma(tmp, scale, scale);
}

// pow (e_pow.c, __pow_fma) for x >= 0 (x = +0 gives +0 for y > 0) and |y| in [2^-65, 2^63): the
// sampler's pow(U, 1/shape) and pow(1 - shape + shape*Y, 1/shape).  Other arguments return NaN.
MTAZ_GLIBC_FN double glibc_pow(double x, double y) {
  MTAZ_GLIBC_NOCONTRACT
  uint64_t ix = glibc_asu64(x);
  const uint64_t iy = glibc_asu64(y);
  const uint32_t topx = (uint32_t)(ix >> 52), topy = (uint32_t)(iy >> 52) & 0x7ffu;
  if (topy - 0x3beu >= 0x43eu - 0x3beu) return __builtin_nan("");
  if (topx - 0x001u >= 0x7ffu - 0x001u) {
    if (ix == 0) return (iy >> 63) ? __builtin_inf() : 0.0;
    if (topx != 0) return __builtin_nan("");   // negative, inf or nan x
    ix = glibc_asu64(x * 0x1p52);               // subnormal: normalise
    ix &= 0x7fffffffffffffffull;
    ix -= 52ull << 52;
  }
  double lo;
  const double hi = glibc_pow_log(ix, &lo);
  const double ehi = y * hi;
  const double t = glibc_fma(hi, y, -ehi);
  const double elo = glibc_fma(y, lo, t);
  return glibc_pow_exp(ehi, elo);
}
