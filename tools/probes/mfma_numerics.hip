// Numerics of v_mfma_f32_16x16x32_f16 accumulation (diagnostic, not part of the product).
//
// 1. One MFMA: D = C + sum_k A[m][k] B[k][n] over 32 products, compared on the host with the exact
//    sum rounded to nearest-even, rounded toward zero, and a k-ordered fmaf chain.
// 2. A k_net_y-shaped accumulation: 72 k-blocks x (Wh Xh, Wh Xl, Wl Xh) into one accumulator seeded
//    with a residual, against fp64 (error relative to sum |a b|: mean signed and max), next to the same
//    passes with the two cross terms in a second accumulator and next to an fmaf chain over the fp32
//    values.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/mfma_numerics tools/probes/mfma_numerics.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                            \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

// A: [nblk][16 rows][32 k] f16, B: [nblk][32 k][16 cols] f16 (row-major per block).  Lane l holds
// A[row l&15][k 8(l>>4) .. +7] and B[k 8(l>>4) .. +7][col l&15]; D lane l: rows 4(l>>4)+i, col l&15.
__device__ inline f16x8 lda(const _Float16* A, int lane) {
  f16x8 r;
  for (int j = 0; j < 8; ++j) r[j] = A[(lane & 15) * 32 + 8 * (lane >> 4) + j];
  return r;
}
__device__ inline f16x8 ldb(const _Float16* B, int lane) {
  f16x8 r;
  for (int j = 0; j < 8; ++j) r[j] = B[(8 * (lane >> 4) + j) * 16 + (lane & 15)];
  return r;
}

// mode 0: all passes into one accumulator (k_net_y); mode 1: cross terms in a second accumulator;
// mode 2: one MFMA per block (Ah Bh only; the single-instruction test uses nblk 1)
__global__ void k_acc(const _Float16* Ah, const _Float16* Al, const _Float16* Bh, const _Float16* Bl,
                      const float* C, int nblk, int mode, float* D) {
  const int lane = threadIdx.x;
  f32x4 acc, acc2 = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < 4; ++i) acc[i] = C[(4 * (lane >> 4) + i) * 16 + (lane & 15)];
  for (int b = 0; b < nblk; ++b) {
    const f16x8 ah = lda(Ah + b * 512, lane), bh = ldb(Bh + b * 512, lane);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
    if (mode == 2) continue;
    const f16x8 al = lda(Al + b * 512, lane), bl = ldb(Bl + b * 512, lane);
    if (mode == 0) {
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
    } else {
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc2, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc2, 0, 0, 0);
    }
  }
  for (int i = 0; i < 4; ++i) D[(4 * (lane >> 4) + i) * 16 + (lane & 15)] = acc[i] + acc2[i];
}

static float rz(double x) {   // toward zero
  float f = (float)x;
  if (std::fabs((double)f) > std::fabs(x)) f = std::nextafter(f, 0.f);
  return f;
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 200;
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  _Float16 *dAh, *dAl, *dBh, *dBl;
  float *dC, *dD;
  const int NB = 72;
  CHECK(hipMalloc(&dAh, NB * 512 * 2)); CHECK(hipMalloc(&dAl, NB * 512 * 2));
  CHECK(hipMalloc(&dBh, NB * 512 * 2)); CHECK(hipMalloc(&dBl, NB * 512 * 2));
  CHECK(hipMalloc(&dC, 256 * 4)); CHECK(hipMalloc(&dD, 256 * 4));
  std::vector<_Float16> Ah(NB * 512), Al(NB * 512), Bh(NB * 512), Bl(NB * 512);
  std::vector<float> Af(NB * 512), Bf(NB * 512), C(256), D(256);
  auto upload = [&]() {
    CHECK(hipMemcpy(dAh, Ah.data(), NB * 1024, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dAl, Al.data(), NB * 1024, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dBh, Bh.data(), NB * 1024, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dBl, Bl.data(), NB * 1024, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dC, C.data(), 1024, hipMemcpyHostToDevice));
  };
  auto fill = [&](float wscale, float xscale, float cscale, bool relu) {
    for (int i = 0; i < NB * 512; ++i) {
      float w = nd(rng) * wscale, x = nd(rng) * xscale;
      if (relu) x = std::fabs(x);
      Af[i] = w; Bf[i] = x;
      Ah[i] = (_Float16)w; Al[i] = (_Float16)(w - (float)Ah[i]);
      Bh[i] = (_Float16)x; Bl[i] = (_Float16)(x - (float)Bh[i]);
    }
    for (int i = 0; i < 256; ++i) C[i] = nd(rng) * cscale;
  };
  auto run = [&](int nblk, int mode) {
    hipLaunchKernelGGL(k_acc, dim3(1), dim3(64), 0, 0, dAh, dAl, dBh, dBl, dC, nblk, mode, dD);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost));
  };

  // 1. one MFMA, f16 inputs exactly representable, C random: which rounding?
  long rne = 0, rtz = 0, chain = 0, n = 0;
  for (int t = 0; t < trials; ++t) {
    fill(1.f, 1.f, t % 2 ? 1.f : 64.f, false);
    upload();
    run(1, 2);
    for (int m = 0; m < 16; ++m)
      for (int c = 0; c < 16; ++c) {
        double ex = C[m * 16 + c];
        float ch = C[m * 16 + c];
        for (int k = 0; k < 32; ++k) {
          const double p = (double)(float)Ah[m * 32 + k] * (double)(float)Bh[k * 16 + c];
          ex += p;
          ch = std::fmaf((float)Ah[m * 32 + k], (float)Bh[k * 16 + c], ch);
        }
        const float d = D[m * 16 + c];
        rne += d == (float)ex;
        rtz += d == rz(ex);
        chain += d == ch;
        ++n;
      }
  }
  printf("single MFMA (%ld outputs): equal to RNE(exact) %.4f, RTZ(exact) %.4f, fmaf chain %.4f\n", n,
         (double)rne / n, (double)rtz / n, (double)chain / n);

  // 2. k_net_y-shaped accumulation
  for (int relu = 0; relu < 2; ++relu)
    for (int cs = 0; cs < 2; ++cs) {
      double sm[3] = {0, 0, 0}, mx[3] = {0, 0, 0}, sfma = 0, mfma_ = 0;
      long cnt = 0;
      for (int t = 0; t < trials / 4 + 1; ++t) {
        fill(0.02f, 100.f, cs ? 3000.f : 0.f, relu);
        upload();
        std::vector<float> Dm[2];
        for (int mode = 0; mode < 2; ++mode) {
          run(NB, mode);
          Dm[mode] = D;
        }
        for (int m = 0; m < 16; ++m)
          for (int c = 0; c < 16; ++c) {
            double ex = C[m * 16 + c], mag = std::fabs(ex);
            float ch = C[m * 16 + c];
            for (int b = 0; b < NB; ++b)
              for (int k = 0; k < 32; ++k) {
                const double p = (double)Af[b * 512 + m * 32 + k] * (double)Bf[b * 512 + k * 16 + c];
                ex += p;
                mag += std::fabs(p);
                ch = std::fmaf(Af[b * 512 + m * 32 + k], Bf[b * 512 + k * 16 + c], ch);
              }
            for (int mode = 0; mode < 2; ++mode) {
              const double e = (Dm[mode][m * 16 + c] - ex) / mag;
              sm[mode] += e;
              mx[mode] = std::max(mx[mode], std::fabs(e));
            }
            const double e = (ch - ex) / mag;
            sfma += e;
            mfma_ = std::max(mfma_, std::fabs(e));
            ++cnt;
          }
      }
      printf("K=2304 x3 relu=%d residual=%s: one acc mean %+.2e max %.2e | cross acc mean %+.2e max %.2e | "
             "fp32 fmaf chain mean %+.2e max %.2e (relative to sum|ab|)\n",
             relu, cs ? "3000" : "0", sm[0] / cnt, mx[0], sm[1] / cnt, mx[1], sfma / cnt, mfma_);
    }
  return 0;
}
