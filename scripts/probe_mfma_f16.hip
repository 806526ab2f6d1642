// Probe: numerics of v_mfma_f32_32x32x16_f16 on gfx950 (experiment, not product).
//
// The split-f16 score kernel needs a proven error bound for the matrix core's
// f32 accumulation of f16 products.  For each test case this compares the
// MFMA result D = A*B + C element by element with three models:
//   seq   : k-ordered fmaf chain from C (k = 0..15), one rounding per product
//   once  : the exact sum (long double / double-double) rounded once to f32
//   bound : |D - exact| <= 16 * 2^-24 * (|C| + sum |a_k b_k|)   (gamma_16 model)
// Prints mismatch counts and the worst error in units of 2^-24 * (|C| + sum|ab|).
//
// build: hipcc --offload-arch=gfx950 -O2 -o scripts/probe_mfma_f16 scripts/probe_mfma_f16.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// A [32][16], B [16][32], C/D [32][32] row-major; one wave per case
__global__ void k_mfma(const _Float16* A, const _Float16* B, const float* C, float* D, int cases) {
  const int cs = blockIdx.x;
  if (cs >= cases) return;
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  const _Float16* a = A + (size_t)cs * 32 * 16;
  const _Float16* b = B + (size_t)cs * 16 * 32;
  half8 av, bv;
  for (int j = 0; j < 8; ++j) {
    av[j] = a[r * 16 + 8 * h + j];
    bv[j] = b[(8 * h + j) * 32 + r];
  }
  floatx16 acc;
  for (int g = 0; g < 16; ++g) {
    const int row = (g & 3) + 8 * (g >> 2) + 4 * h;
    acc[g] = C[(size_t)cs * 1024 + row * 32 + r];
  }
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(av, bv, acc, 0, 0, 0);
  for (int g = 0; g < 16; ++g) {
    const int row = (g & 3) + 8 * (g >> 2) + 4 * h;
    D[(size_t)cs * 1024 + row * 32 + r] = acc[g];
  }
}

static float h2f(_Float16 v) { return (float)v; }

int main(int argc, char** argv) {
  const int cases = argc > 1 ? atoi(argv[1]) : 2000;
  std::mt19937_64 rng(12345);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::uniform_int_distribution<int> kind_d(0, 5);
  std::vector<_Float16> A((size_t)cases * 512), B((size_t)cases * 512);
  std::vector<float> C((size_t)cases * 1024), D((size_t)cases * 1024);
  std::vector<int> kind(cases);
  for (int cs = 0; cs < cases; ++cs) {
    const int kd = cs < 6 ? cs : kind_d(rng);
    kind[cs] = kd;
    for (int i = 0; i < 512; ++i) {
      float va = nd(rng), vb = nd(rng);
      if (kd == 1) { va = ldexpf(1.0f + 0.001f * i, -13); vb = ldexpf(1.0f, -12); }   // tiny products on C = 1
      if (kd == 2) { va *= (i % 3 == 0) ? 1000.f : 0.01f; }                            // mixed magnitudes
      if (kd == 3) { va = (i & 1) ? 1.0f : -1.0f; vb = 1.0f + ldexpf((float)(i % 7), -10); }  // cancellation
      if (kd == 4) { va = ldexpf(nd(rng), -20); }                                      // subnormal f16 inputs
      A[(size_t)cs * 512 + i] = (_Float16)va;
      B[(size_t)cs * 512 + i] = (_Float16)vb;
    }
    for (int i = 0; i < 1024; ++i) {
      float vc = nd(rng);
      if (kd == 1) vc = 1.0f;
      if (kd == 3) vc = ldexpf(1.0f, -30);
      if (kd == 5) vc = 0.0f;
      C[(size_t)cs * 1024 + i] = vc;
    }
  }
  _Float16 *dA, *dB; float *dC, *dD;
  hipMalloc(&dA, A.size() * 2); hipMalloc(&dB, B.size() * 2);
  hipMalloc(&dC, C.size() * 4); hipMalloc(&dD, D.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_mfma, dim3(cases), dim3(64), 0, 0, dA, dB, dC, dD, cases);
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  long long n = 0, mis_seq[6] = {0}, mis_once[6] = {0}, tot[6] = {0}, over16 = 0;
  double worst = 0.0, worst_kind[6] = {0};
  for (int cs = 0; cs < cases; ++cs) {
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        const float c = C[(size_t)cs * 1024 + i * 32 + j];
        float seq = c;
        long double ex = c, mag = fabsl((long double)c);
        for (int k = 0; k < 16; ++k) {
          const float a = h2f(A[(size_t)cs * 512 + i * 16 + k]), b = h2f(B[(size_t)cs * 512 + k * 32 + j]);
          seq = fmaf(a, b, seq);
          ex += (long double)a * (long double)b;   // exact: f16 x f16 fits; 64-bit mantissa sum
          mag += fabsl((long double)a * (long double)b);
        }
        const float once = (float)ex;
        const float d = D[(size_t)cs * 1024 + i * 32 + j];
        const int kd = kind[cs];
        ++n; ++tot[kd];
        if (d != seq) ++mis_seq[kd];
        if (d != once) ++mis_once[kd];
        const double e = mag > 0 ? (double)(fabsl((long double)d - ex) / (mag * 0x1p-24L)) : 0.0;
        if (e > worst) worst = e;
        if (e > worst_kind[kd]) worst_kind[kd] = e;
        if (e > 16.0) ++over16;
      }
  }
  printf("elements %lld\n", n);
  const char* names[6] = {"normal", "tiny-on-1", "mixed-mag", "cancel", "subnormal", "C=0"};
  for (int k = 0; k < 6; ++k)
    printf("%-10s n=%lld  !=seq %lld  !=once %lld  worst %.3f x 2^-24 x (|C|+sum|ab|)\n", names[k], tot[k],
           mis_seq[k], mis_once[k], worst_kind[k]);
  printf("worst overall %.3f, elements over the gamma_16 model: %lld\n", worst, over16);
  return 0;
}
