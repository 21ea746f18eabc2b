// Probe for the gfx950 scaled conversions the k_net_z epilogue could use:
//   v_cvt_scalef32_pk_fp8_f32 (2 f32 -> 2 e4m3), v_cvt_scalef32_pk_fp8_f16 (2 f16 -> 2 e4m3),
//   v_cvt_scalef32_pk_f32_fp8 (2 e4m3 -> 2 f32),
// each against the unscaled conversions of the product (v_cvt_pk_fp8_f32, v_cvt_f32_fp8) with the
// power-of-two scale applied as a separate f32 multiply, x * s or x / s.  Reports, per form and
// per scale exponent, how many of the inputs agree bit for bit.
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/cvt_scale_probe tools/probes/cvt_scale_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef _Float16 v2f16 __attribute__((ext_vector_type(2)));
typedef float v2f32 __attribute__((ext_vector_type(2)));

// out[8 i + ...]: 0 scaled f32->fp8, 1 ref (x*s), 2 ref (x/s), 3 scaled f16->fp8, 4 ref f16 (h*s),
// 5 ref f16 (h/s); fo[4 i + ...]: 0,1 scaled fp8->f32 of byte pair, 2,3 ref (cvt * s)
__global__ void k_probe(const float* x, const unsigned* h2, const unsigned* q, float s, int n, unsigned* out,
                        float* fo) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = x[2 * i], b = x[2 * i + 1];
  out[8 * i + 0] = (unsigned short)__builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_fp8_f32((v2i16){0, 0}, a, b, s, false));
  out[8 * i + 1] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(a * s, b * s, 0, false) & 0xffffu;
  out[8 * i + 2] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(a / s, b / s, 0, false) & 0xffffu;
  const v2f16 hh = __builtin_bit_cast(v2f16, h2[i]);
  out[8 * i + 3] = (unsigned short)__builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_scalef32_pk_fp8_f16((v2i16){0, 0}, hh, s, false));
  out[8 * i + 4] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32((float)hh[0] * s, (float)hh[1] * s, 0, false) & 0xffffu;
  out[8 * i + 5] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32((float)hh[0] / s, (float)hh[1] / s, 0, false) & 0xffffu;
  const v2f32 d = __builtin_amdgcn_cvt_scalef32_pk_f32_fp8(q[i], s, false);
  fo[4 * i + 0] = d[0];
  fo[4 * i + 1] = d[1];
  fo[4 * i + 2] = __builtin_amdgcn_cvt_f32_fp8((int)q[i], 0) * s;
  fo[4 * i + 3] = __builtin_amdgcn_cvt_f32_fp8((int)q[i], 1) * s;
}

int main() {
  const int n = 1 << 16;
  std::vector<float> x(2 * n);
  std::vector<unsigned> h2(n), q(n);
  srand(7);
  for (int i = 0; i < 2 * n; ++i) {
    // magnitudes 2^-30 .. 2^20, both signs, random mantissas
    const float m = 1.f + (float)rand() / RAND_MAX;
    const int e = rand() % 50 - 30;
    x[i] = ldexpf(m, e) * ((rand() & 1) ? -1.f : 1.f);
  }
  for (int i = 0; i < n; ++i) {
    unsigned short a = (unsigned short)(rand() & 0x7bff), b = (unsigned short)(rand() & 0x7bff);   // finite halves
    h2[i] = a | ((unsigned)b << 16);
    q[i] = (unsigned)(rand() & 0xffff);
    if ((q[i] & 0x7f) == 0x7f) q[i] &= ~0x7fu;        // no e4m3 NaN codes
    if (((q[i] >> 8) & 0x7f) == 0x7f) q[i] &= ~0x7f00u;
  }
  float *dx, *dfo;
  unsigned *dh, *dq, *dout;
  hipMalloc(&dx, 8 * n);
  hipMalloc(&dh, 4 * n);
  hipMalloc(&dq, 4 * n);
  hipMalloc(&dout, 32 * n);
  hipMalloc(&dfo, 16 * n);
  hipMemcpy(dx, x.data(), 8 * n, hipMemcpyHostToDevice);
  hipMemcpy(dh, h2.data(), 4 * n, hipMemcpyHostToDevice);
  hipMemcpy(dq, q.data(), 4 * n, hipMemcpyHostToDevice);
  std::vector<unsigned> out(8 * n);
  std::vector<float> fo(4 * n);
  printf("{\"n\": %d, \"rows\": [\n", n);
  for (int k = -24; k <= 24; k += 4) {
    const float s = ldexpf(1.f, k);
    k_probe<<<n / 256, 256>>>(dx, dh, dq, s, n, dout, dfo);
    hipMemcpy(out.data(), dout, 32 * n, hipMemcpyDeviceToHost);
    hipMemcpy(fo.data(), dfo, 16 * n, hipMemcpyDeviceToHost);
    long f32_mul = 0, f32_div = 0, f16_mul = 0, f16_div = 0, dec_mul = 0;
    for (int i = 0; i < n; ++i) {
      f32_mul += out[8 * i] == out[8 * i + 1];
      f32_div += out[8 * i] == out[8 * i + 2];
      f16_mul += out[8 * i + 3] == out[8 * i + 4];
      f16_div += out[8 * i + 3] == out[8 * i + 5];
      dec_mul += memcmp(&fo[4 * i], &fo[4 * i + 2], 8) == 0;
    }
    printf("  {\"scale_exp\": %d, \"enc_f32_eq_mul\": %ld, \"enc_f32_eq_div\": %ld, \"enc_f16_eq_mul\": %ld, "
           "\"enc_f16_eq_div\": %ld, \"dec_eq_mul\": %ld}%s\n",
           k, f32_mul, f32_div, f16_mul, f16_div, dec_mul, k < 24 ? "," : "");
  }
  printf("]}\n");
  return 0;
}
