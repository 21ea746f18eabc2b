// Probe: block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 with e2m3 (fp6) operands on gfx950.
// (1) packing: 32 e2m3 values per lane, value j at bits [6j, 6j+6) of the first 6 dwords,
//     checked on small integers against CPU products (same k map for A and B as the e4m3 probe);
// (2) throughput and held clock of (A,B) format pairs e4m3/e4m3, e2m3/e4m3, e4m3/e2m3, e2m3/e2m3.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int FA, int FB>
__global__ void k_layout(const i32x8* a, const i32x8* b, f32x4* d) {
  const int l = threadIdx.x;
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, FA, FB, 0, 127, 0, 127);
  d[l] = c;
}

template <int FA, int FB>
__global__ __launch_bounds__(256, 1) void k_rate(const uint4* src, float* out, int iters, unsigned long long* clk) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  f32x4 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = (f32x4){0, 0, 0, 0};
  i32x8 A[2], B[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    uint4 x = src[(t * 8 + 2 * i) & 65535], y = src[(t * 8 + 2 * i + 1) & 65535];
    uint4 z = src[(t * 8 + 4 + 2 * i) & 65535], w = src[(t * 8 + 5 + 2 * i) & 65535];
    A[i] = (i32x8){(int)x.x, (int)x.y, (int)x.z, (int)x.w, (int)y.x, (int)y.y, (int)y.z, (int)y.w};
    B[i] = (i32x8){(int)z.x, (int)z.y, (int)z.z, (int)z.w, (int)w.x, (int)w.y, (int)w.z, (int)w.w};
  }
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; it += 2) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      acc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(A[i & 1], B[(i >> 1) & 1], acc[i], FA, FB, 0, 127, 0, 127);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[t] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

static float e2m3_to_f(int v) {   // 1 sign, 2 exponent (bias 1), 3 mantissa
  int s = (v >> 5) & 1, e = (v >> 3) & 3, m = v & 7;
  float r = e == 0 ? m / 8.f : ldexpf(1.f + m / 8.f, e - 1);
  return s ? -r : r;
}
static float e4m3_to_f(int v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float r = e == 0 ? ldexpf((float)m, -9) : ldexpf(1.f + m / 8.f, e - 7);
  return s ? -r : r;
}

int main() {
  srand(11);
  // ---- fp6 packing, A and B both e2m3 ----
  std::vector<int> av(64 * 32), bv(64 * 32);
  const int v6[7] = {0x00, 0x08, 0x0c, 0x10, 0x14, 0x28, 0x30};   // 0, 1, 1.5, 2, 3, -1, -2
  for (auto& x : av) x = v6[rand() % 7];
  for (auto& x : bv) x = v6[rand() % 7];
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
  f32x4* dd;
  (void)hipMalloc(&da, 2048); (void)hipMalloc(&db, 2048); (void)hipMalloc(&dd, 1024);
  (void)hipMemcpy(da, aw.data(), 2048, hipMemcpyHostToDevice);
  (void)hipMemcpy(db, bw.data(), 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL((k_layout<2, 2>), dim3(1), dim3(64), 0, 0, da, db, dd);
  std::vector<float> d(256);
  (void)hipMemcpy(d.data(), dd, 1024, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int col = l & 15, row = 4 * (l >> 4) + i;
      float s = 0;
      for (int g = 0; g < 4; ++g)
        for (int j = 0; j < 32; ++j) s += e2m3_to_f(av[(16 * g + row) * 32 + j]) * e2m3_to_f(bv[(16 * g + col) * 32 + j]);
      if (s != d[l * 4 + i]) ++bad;
    }
  printf("fp6 packing (value j at bits 6j): %d / 256 mismatches (d[0]=%g)\n", bad, d[0]);
  // ---- mixed: A e2m3 packed, B e4m3 bytes ----
  std::vector<int> b8(64 * 32);
  const int v8[5] = {0x00, 0x38, 0x40, 0xb8, 0x44};   // 0, 1, 2, -1, 3
  for (auto& x : b8) x = v8[rand() % 5];
  std::vector<uint8_t> b8bytes(2048);
  for (int i = 0; i < 2048; ++i) b8bytes[i] = (uint8_t)b8[i];
  (void)hipMemcpy(db, b8bytes.data(), 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL((k_layout<2, 0>), dim3(1), dim3(64), 0, 0, da, db, dd);
  (void)hipMemcpy(d.data(), dd, 1024, hipMemcpyDeviceToHost);
  bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      const int col = l & 15, row = 4 * (l >> 4) + i;
      float s = 0;
      for (int g = 0; g < 4; ++g)
        for (int j = 0; j < 32; ++j) s += e2m3_to_f(av[(16 * g + row) * 32 + j]) * e4m3_to_f(b8[(16 * g + col) * 32 + j]);
      if (s != d[l * 4 + i]) ++bad;
    }
  printf("mixed A e2m3 / B e4m3: %d / 256 mismatches\n", bad);
  // ---- rates ----
  const int NWG = 1024, ITERS = 65536;
  std::vector<uint32_t> r(65536 * 4);
  for (auto& x : r) x = ((uint32_t)rand() * 2654435761u) ^ (uint32_t)rand();
  for (auto& x : r) x &= 0xbfbfbfbfu;   // e4m3 bytes without NaN; any bits are valid e2m3
  uint4* src;
  float* out;
  unsigned long long* clk;
  (void)hipMalloc(&src, r.size() * 4); (void)hipMalloc(&out, NWG * 256 * 4); (void)hipMalloc(&clk, NWG * 16);
  (void)hipMemcpy(src, r.data(), r.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  const char* names[4] = {"e4m3xe4m3", "e2m3xe4m3", "e4m3xe2m3", "e2m3xe2m3"};
  for (int round = 0; round < 2; ++round)
    for (int mode = 0; mode < 4; ++mode) {
      for (int w = 0; w < 3; ++w) {
        (void)hipEventRecord(e0);
        if (mode == 0) hipLaunchKernelGGL((k_rate<0, 0>), dim3(NWG), dim3(256), 0, 0, src, out, ITERS, clk);
        if (mode == 1) hipLaunchKernelGGL((k_rate<2, 0>), dim3(NWG), dim3(256), 0, 0, src, out, ITERS, clk);
        if (mode == 2) hipLaunchKernelGGL((k_rate<0, 2>), dim3(NWG), dim3(256), 0, 0, src, out, ITERS, clk);
        if (mode == 3) hipLaunchKernelGGL((k_rate<2, 2>), dim3(NWG), dim3(256), 0, 0, src, out, ITERS, clk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
      }
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      std::vector<unsigned long long> c(NWG * 2);
      (void)hipMemcpy(c.data(), clk, NWG * 16, hipMemcpyDeviceToHost);
      double cyc = 0, tk = 0;
      for (int i = 0; i < NWG; ++i) { cyc += c[2 * i]; tk += c[2 * i + 1]; }
      const double flop = 2.0 * 8.0 * 16 * 16 * 128 * ITERS * NWG * 4;
      printf("{\"round\": %d, \"formats\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f, \"wave_cycles\": %.0f, \"clock_ghz\": %.3f}\n",
             round, names[mode], ms, flop / (ms * 1e-3) / 1e12, cyc / NWG, cyc / (tk * 10.0));
    }
  return 0;
}
