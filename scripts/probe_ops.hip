// Probe: issue cost of single VALU instructions on gfx950 at the scorer's
// occupancy (3 waves per SIMD, 12 waves per block, one block per CU), for
// choosing the decision encoding of k_score_mf2's tile loop
// (scripts/probe_ops.hip; profiles/r04_probe_ops.txt).  Each variant runs 16
// independent accumulators through 4 dependent applications of one
// instruction per iteration (64 instructions per wave-iteration); the result
// is SIMD cycles per wave64 instruction = wave cycles / (64 x 3 waves).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -o probe_ops probe_ops.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kWaves = 12;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

#define ASM3(ins) asm volatile(ins " %0, %1, %2" : "=v"(r) : "v"(s), "v"(x))
#define ASM4(ins) asm volatile(ins " %0, %1, %2, %3" : "=v"(r) : "v"(s), "v"(x), "v"(y))
template <int MODE>
__device__ __forceinline__ unsigned op(unsigned s, unsigned x, unsigned y) {
  unsigned r;
  switch (MODE) {
    case 0: ASM4("v_fma_f32"); break;
    case 1: ASM3("v_mul_f32"); break;
    case 2: asm volatile("v_alignbit_b32 %0, %1, %2, 31" : "=v"(r) : "v"(s), "v"(x)); break;
    case 3: asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xf2" : "=v"(r) : "v"(s), "v"(x), "v"(y)); break;
    case 4: ASM4("v_bfi_b32"); break;
    case 5: ASM4("v_lshl_or_b32"); break;
    case 6: ASM4("v_perm_b32"); break;
    case 7: ASM3("v_add_u32"); break;
    case 8: ASM3("v_lshrrev_b32"); break;
    case 9: ASM4("v_and_or_b32"); break;
    case 10: ASM4("v_or3_b32"); break;
    case 11: ASM3("v_xor_b32"); break;
    case 12: ASM4("v_med3_f32"); break;
    case 13: ASM4("v_bfe_u32"); break;
    case 14: ASM3("v_cvt_pkrtz_f16_f32"); break;
    case 15: ASM4("v_add3_u32"); break;
    case 16: ASM3("v_pk_add_u16"); break;
    case 17: ASM4("v_lshl_add_u32"); break;
    default: r = s;
  }
  return r;
}

template <int MODE>
__global__ __launch_bounds__(kWaves * 64) __attribute__((amdgpu_waves_per_eu(3, 3)))
void k_ops(const unsigned* __restrict__ in, unsigned* __restrict__ out, unsigned long long* __restrict__ cyc,
           int iters) {
  const int lane = threadIdx.x & 63;
  unsigned s[16], x[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) { s[g] = in[(lane + g) & 63]; x[g] = in[64 + ((lane + 3 * g) & 63)]; }
  unsigned y = in[128 + lane];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    y += 0x9E3779B9u;                  // one op per iteration keeps the loop body live
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int g = 0; g < 16; ++g) s[g] = op<MODE>(s[g], x[(g + k) & 15], y);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned r = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g) r ^= s[g];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (lane == 0) cyc[blockIdx.x * kWaves + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int iters = 20000;
  unsigned *in, *out;
  unsigned long long* cyc;
  hipMalloc(&in, 4096 * 4);
  unsigned hin[4096];
  for (int i = 0; i < 4096; ++i) hin[i] = 0x3f800000u + (unsigned)i * 977u;   // finite floats near 1
  hipMemcpy(in, hin, sizeof(hin), hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)cus * kWaves * 64 * 4);
  hipMalloc(&cyc, (size_t)cus * kWaves * 8);
  constexpr int kN = 18;
  void (*ks[kN])(const unsigned*, unsigned*, unsigned long long*, int) = {
      k_ops<0>, k_ops<1>, k_ops<2>, k_ops<3>, k_ops<4>, k_ops<5>, k_ops<6>, k_ops<7>,
      k_ops<8>, k_ops<9>, k_ops<10>, k_ops<11>, k_ops<12>, k_ops<13>, k_ops<14>, k_ops<15>, k_ops<16>, k_ops<17>};
  const char* names[kN] = {"v_fma_f32", "v_mul_f32", "v_alignbit_b32", "v_bitop3_b32", "v_bfi_b32",
                           "v_lshl_or_b32", "v_perm_b32", "v_add_u32", "v_lshrrev_b32", "v_and_or_b32",
                           "v_or3_b32", "v_xor_b32", "v_med3_f32", "v_bfe_u32", "v_cvt_pkrtz_f16_f32",
                           "v_add3_u32", "v_pk_add_u16", "v_lshl_add_u32"};
  unsigned long long* h = new unsigned long long[cus * kWaves];
  for (int v = 0; v < kN; ++v) {
    hipLaunchKernelGGL(ks[v], dim3(cus), dim3(kWaves * 64), 0, 0, in, out, cyc, 100);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
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
    printf("%-22s %8.3f ms  %6.2f SIMD cycles per wave64 instruction  (s_memtime clock %.2f GHz)\n", names[v], ms,
           mean / iters / (64.0 * 3.0), mean / (ms * 1e6));
  }
  return 0;
}
