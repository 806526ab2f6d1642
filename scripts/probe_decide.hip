// Probe: issue cost of k_score_mf's tile loop on gfx950 (scripts/probe_decide.hip).
// One tile = 4 v_mfma_f32_32x32x16_f16 (a from two chained MFMAs, the band
// sides from one each) + the decisions on the 16 outputs per lane:
//   z1 = fma(a, a, -Ylo), z2 = fma(-a, a, Yhi), s1 = alignbit(s1, z1, 31), s2 = ...
// Variants (cycles per tile per wave from s_memtime, 3 waves per SIMD as in the kernel):
//   0 MFMA only   1 decisions only   2 both (the kernel's loop)
//   3 both, FMAs as packed v_pk_fma_f32 pairs
//   4 decisions only, FMAs packed
//   5 decisions only, sign bits via shift + or (the compiler emits alignbit anyway)
//   6 both, split order: inlier tests (a, Ylo), next tile's Ylo MFMA, outlier
//     tests (a, Yhi), next tile's a and Yhi MFMAs; sched_barrier between phases
//   7 both, two accumulator sets (next tile's MFMAs beside this tile's decisions)
//   8 64 v_fma_f32 only   9 64 v_alignbit_b32 only   10 64 v_lshl_add_u32 only
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -o probe_decide probe_decide.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kWaves = 12;   // per block = 3 per SIMD

template <int MODE>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(3, 3)))
void k_tile(const _Float16* __restrict__ in, unsigned* __restrict__ out, unsigned long long* __restrict__ cyc,
            int iters) {
  const int lane = threadIdx.x & 63;
  h8 A1, A2, AL, AH, B;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    A1[i] = in[lane * 8 + i];
    A2[i] = in[512 + lane * 8 + i];
    AL[i] = in[1024 + lane * 8 + i];
    AH[i] = in[1536 + lane * 8 + i];
    B[i] = in[2048 + lane * 8 + i];
  }
  f16v a, l, h;
#pragma unroll
  for (int g = 0; g < 16; ++g) { a[g] = in[g] ; l[g] = in[16 + g]; h[g] = in[32 + g]; }
  unsigned s1[16], s2[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) { s1[g] = 0; s2[g] = 0; }
  const f16v zero = {};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (MODE == 6 || MODE == 7) {
    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B, zero, 0, 0, 0);
    a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, B, a, 0, 0, 0);
    l = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL, B, zero, 0, 0, 0);
    h = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH, B, zero, 0, 0, 0);
  }
  f16v a2 = a, l2 = l, h2 = h;
  for (int it = 0; it < iters; ++it) {
    if (MODE == 6) {
#pragma unroll
      for (int g = 0; g < 16; ++g)
        s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(__builtin_fmaf(a[g], a[g], -l[g])), 31);
      __builtin_amdgcn_sched_barrier(0);
      B[it & 7] = (_Float16)(float)it;
      l = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL, B, zero, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 16; ++g)
        s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(__builtin_fmaf(-a[g], a[g], h[g])), 31);
      __builtin_amdgcn_sched_barrier(0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B, zero, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, B, a, 0, 0, 0);
      h = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH, B, zero, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
    if (MODE == 7) {
      B[it & 7] = (_Float16)(float)it;
      a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B, zero, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, B, a2, 0, 0, 0);
      l2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL, B, zero, 0, 0, 0);
      h2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH, B, zero, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(__builtin_fmaf(a[g], a[g], -l[g])), 31);
        s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(__builtin_fmaf(-a[g], a[g], h[g])), 31);
      }
      a = a2; l = l2; h = h2;
      continue;
    }
    if (MODE >= 8) {
      a[it & 15] += 1.0f;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        if (MODE == 8) {
          l[g] = __builtin_fmaf(a[g], a[g], -l[g]);
          h[g] = __builtin_fmaf(-a[g], a[g], h[g]);
          l[g] = __builtin_fmaf(a[g], l[g], -h[g]);
          h[g] = __builtin_fmaf(-a[g], h[g], l[g]);
        } else if (MODE == 9) {
          s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(a[g]), 31);
          s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(a[g]), 30);
          s1[g] = __builtin_amdgcn_alignbit(s1[g], s2[g], 29);
          s2[g] = __builtin_amdgcn_alignbit(s2[g], s1[g], 28);
        } else {
          s1[g] = (s1[g] << 1) + __float_as_uint(a[g]);
          s2[g] = (s2[g] << 2) + s1[g];
          s1[g] = (s1[g] << 3) + s2[g];
          s2[g] = (s2[g] << 1) + s1[g];
        }
      }
      continue;
    }
    if (MODE == 0 || MODE == 2 || MODE == 3) {
      a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B, zero, 0, 0, 0);
      a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, B, a, 0, 0, 0);
      l = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL, B, zero, 0, 0, 0);
      h = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH, B, zero, 0, 0, 0);
      B[it & 7] = (_Float16)(float)it;   // keeps every iteration's products live
    } else {
      // decisions only: perturb the inputs with one op so nothing is hoisted
      a[it & 15] += 1.0f;
    }
    if (MODE == 0) {
#pragma unroll
      for (int g = 0; g < 16; g += 4) s1[g] ^= __float_as_uint(a[g] + l[g] + h[g]);
    } else if (MODE == 3 || MODE == 4) {
#pragma unroll
      for (int g = 0; g < 16; g += 2) {
        const f2 av = {a[g], a[g + 1]}, lv = {l[g], l[g + 1]}, hv = {h[g], h[g + 1]};
        const f2 z1 = __builtin_elementwise_fma(av, av, -lv);
        const f2 z2 = __builtin_elementwise_fma(-av, av, hv);
        s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(z1[0]), 31);
        s1[g + 1] = __builtin_amdgcn_alignbit(s1[g + 1], __float_as_uint(z1[1]), 31);
        s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(z2[0]), 31);
        s2[g + 1] = __builtin_amdgcn_alignbit(s2[g + 1], __float_as_uint(z2[1]), 31);
      }
    } else if (MODE == 5) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float z1 = __builtin_fmaf(a[g], a[g], -l[g]);
        const float z2 = __builtin_fmaf(-a[g], a[g], h[g]);
        s1[g] = (s1[g] << 1) | (__float_as_uint(z1) >> 31);
        s2[g] = (s2[g] << 1) | (__float_as_uint(z2) >> 31);
      }
    } else {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float z1 = __builtin_fmaf(a[g], a[g], -l[g]);
        const float z2 = __builtin_fmaf(-a[g], a[g], h[g]);
        s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(z1), 31);
        s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(z2), 31);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned r = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g) r += s1[g] ^ s2[g] ^ __float_as_uint(l[g] + h[g]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (lane == 0) cyc[blockIdx.x * kWaves + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int iters = 20000;
  _Float16* in;
  unsigned* out;
  unsigned long long* cyc;
  hipMalloc(&in, 4096 * 2);
  hipMemset(in, 0, 4096 * 2);
  hipMalloc(&out, (size_t)cus * kWaves * 64 * 4);
  hipMalloc(&cyc, (size_t)cus * kWaves * 8);
  void (*ks[11])(const _Float16*, unsigned*, unsigned long long*, int) = {
      k_tile<0>, k_tile<1>, k_tile<2>, k_tile<3>, k_tile<4>, k_tile<5>, k_tile<6>, k_tile<7>,
      k_tile<8>, k_tile<9>, k_tile<10>};
  const char* names[11] = {"MFMA only", "decisions only", "MFMA + decisions", "MFMA + decisions, pk_fma",
                          "decisions only, pk_fma", "decisions only, shift+or", "split order",
                          "two accumulator sets", "64 v_fma_f32", "64 v_alignbit_b32", "64 v_lshl_add_u32"};
  unsigned long long* h = new unsigned long long[cus * kWaves];
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int v = 0; v < 11; ++v) {
    hipLaunchKernelGGL(ks[v], dim3(cus), dim3(kWaves * 64), 0, 0, in, out, cyc, 100);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[v], dim3(cus), dim3(kWaves * 64), 0, 0, in, out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, cyc, (size_t)cus * kWaves * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < cus * kWaves; ++i) mean += (double)h[i];
    mean /= cus * kWaves;
    // 3 waves share a SIMD: SIMD cycles per tile = wave cycles per tile / 3
    printf("%-28s %8.3f ms  %7.1f cycles per tile per wave  -> %6.1f SIMD cycles per tile  (clock %.2f GHz)\n",
           names[v], ms, mean / iters, mean / iters / 3.0, mean / (ms * 1e6));
  }
  return 0;
}
