// Probe for the e2m3 cross-term path of k_net_z (VAR 8192):
// (1) per-lane E8M0 scales of v_mfma_scale_f32_16x16x128_f8f6f4 with e2m3 x e2m3: lane l's
//     scale_a byte applies to A row (l & 15), K block (l >> 4); scale_b byte to B column (l & 15),
//     K block (l >> 4);
// (2) the e2m3 encoder used by the epilogue: e4m3 RNE (v_cvt_pk_fp8_f32) of v * 2^-6 lands on
//     e4m3's exponent fields 0..3, whose grid is e2m3's grid scaled by 2^-6, so
//     code6 = (b & 0x1f) | ((b & 0x80) >> 2), checked against a CPU round-to-nearest-even e2m3
//     on every step of [-7.5, 7.5] at 2^-12 resolution and on random values.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_scaled(const i32x8* a, const i32x8* b, const int* sa, const int* sb, f32x4* d) {
  const int l = threadIdx.x;
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 2, 2, 0, sa[l], 0, sb[l]);
  d[l] = c;
}

__global__ void k_enc(const float* v, int* code, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int b = __builtin_amdgcn_cvt_pk_fp8_f32(v[i] * 0.015625f, 0.f, 0, false) & 0xff;
  code[i] = (b & 0x1f) | ((b & 0x80) >> 2);
}

static float e2m3_to_f(int v) {   // 1 sign, 2 exponent (bias 1), 3 mantissa
  int s = (v >> 5) & 1, e = (v >> 3) & 3, m = v & 7;
  float r = e == 0 ? m / 8.f : ldexpf(1.f + m / 8.f, e - 1);
  return s ? -r : r;
}
static int f_to_e2m3(float x) {   // RNE to the e2m3 grid (|x| <= 7.5)
  int best = 0;
  float bd = 1e30f;
  for (int c = 0; c < 64; ++c) {
    const float d = fabsf(e2m3_to_f(c) - x);
    if (d < bd || (d == bd && (c & 1) == 0)) bd = d, best = c;
  }
  return best;
}

int main() {
  srand(5);
  std::vector<int> av(64 * 32), bv(64 * 32), sa(64), sb(64);
  for (auto& x : av) x = rand() & 63;
  for (auto& x : bv) x = rand() & 63;
  for (auto& x : sa) x = 120 + rand() % 14;
  for (auto& x : sb) x = 120 + rand() % 14;
  auto pack6 = [](const std::vector<int>& v, std::vector<uint32_t>& w) {
    w.assign(64 * 8, 0);
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int bit = 6 * j;
        w[l * 8 + bit / 32] |= (uint32_t)v[l * 32 + j] << (bit % 32);
        if (bit % 32 > 26) w[l * 8 + bit / 32 + 1] |= (uint32_t)v[l * 32 + j] >> (32 - bit % 32);
      }
  };
  std::vector<uint32_t> aw, bw;
  pack6(av, aw);
  pack6(bv, bw);
  i32x8 *da, *db;
  int *dsa, *dsb;
  f32x4* dd;
  (void)hipMalloc(&da, 2048); (void)hipMalloc(&db, 2048); (void)hipMalloc(&dd, 1024);
  (void)hipMalloc(&dsa, 256); (void)hipMalloc(&dsb, 256);
  (void)hipMemcpy(da, aw.data(), 2048, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, bw.data(), 2048, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice);
  (void)hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_scaled, dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
  std::vector<float> d(256);
  (void)hipMemcpy(d.data(), dd, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  double maxrel = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int col = l & 15, row = 4 * (l >> 4) + i;
      double s = 0;
      for (int g = 0; g < 4; ++g) {
        double t = 0;
        for (int j = 0; j < 32; ++j) t += (double)e2m3_to_f(av[(16 * g + row) * 32 + j]) * e2m3_to_f(bv[(16 * g + col) * 32 + j]);
        s += t * ldexp(1.0, sa[16 * g + row] - 127) * ldexp(1.0, sb[16 * g + col] - 127);
      }
      const double rel = fabs(s - d[l * 4 + i]) / (fabs(s) + 1e-30);
      if (rel > maxrel) maxrel = rel;
      if (rel > 1e-6) ++bad;
    }
  printf("per-lane scales e2m3 x e2m3: %d / 256 mismatches, max rel %.3g\n", bad, maxrel);

  // encoder
  std::vector<float> v;
  for (int k = -30720; k <= 30720; ++k) v.push_back(k / 4096.f);   // [-7.5, 7.5]
  for (int k = 0; k < 100000; ++k) v.push_back(((float)rand() / RAND_MAX * 2.f - 1.f) * 7.5f);
  for (int k = 0; k < 1000; ++k) v.push_back(ldexpf((float)rand() / RAND_MAX, -(rand() % 20)));
  const int n = (int)v.size();
  float* dv;
  int* dc;
  (void)hipMalloc(&dv, n * 4); (void)hipMalloc(&dc, n * 4);
  (void)hipMemcpy(dv, v.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_enc, dim3((n + 255) / 256), dim3(256), 0, 0, dv, dc, n);
  std::vector<int> c(n);
  (void)hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
  int ebad = 0, shown = 0;
  for (int i = 0; i < n; ++i) {
    const float want = e2m3_to_f(f_to_e2m3(v[i])), got = e2m3_to_f(c[i]);
    if (want != got) {
      ++ebad;
      if (shown++ < 8) printf("  enc mismatch v=%.8g got %g want %g\n", v[i], got, want);
    }
  }
  printf("e2m3 encoder via e4m3 of v*2^-6: %d / %d mismatches\n", ebad, n);
  return (bad || ebad) ? 1 : 0;
}
