// Probe (round 3): what bounds k_score_mf's tile loop on gfx950.
// One tile = 4 v_mfma_f32_32x32x16_f16 (a: two chained, Ylo / Yhi: one each)
// on B fragments read from LDS (3 ds_read_b128, one tile ahead) + the
// decisions on the 16 outputs per lane.  Cycles from s_memtime per wave,
// reported per tile per SIMD (wave cycles / waves per SIMD).
//
// Variants (template MODE):
//   0  the kernel's loop: one accumulator set, decisions fma + v_alignbit
//   1  two accumulator sets, loop unrolled by 2: tile t+1's MFMAs issue
//      before tile t's decisions (no register copies)
//   2  MFMA only (+ 4 VALU per tile to keep the results live)
//   3  decisions only (fma + alignbit; inputs perturbed by one add)
//   4  decisions only, sign shift-in as v_lshrrev + v_lshl_or_b32
//   5  decisions only, aa = a*a, then sign(aa - Ylo) via v_sub (z1 = aa - lo, z2 = hi - aa)
//   6  like 0 with the decisions as mode 4
//   7  like 1 with the decisions as mode 4
//   8  decisions only, 64 v_alignbit_b32 (independent chains)
//   9  decisions only, 64 v_lshl_or_b32
//  10  decisions only, 64 v_fma_f32
// W = waves per SIMD (block = 4 W waves, one block per CU).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-slp-vectorize -o probe_tile probe_tile.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kTiles = 24;

struct Acc { f16v a, l, h; };

__device__ __forceinline__ Acc tile_mfma(h8 A1, h8 A2, h8 AL, h8 AH, h8 b1, h8 b2, h8 bd) {
  f16v z = {};
  Acc r;
  r.a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, b1, z, 0, 0, 0);
  r.l = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL, bd, z, 0, 0, 0);
  r.h = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH, bd, z, 0, 0, 0);
  r.a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, b2, r.a, 0, 0, 0);
  return r;
}

template <int ENC>
__device__ __forceinline__ void decide(const Acc& r, uint32_t (&s1)[16], uint32_t (&s2)[16]) {
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    if (ENC == 0) {
      const float z1 = __builtin_fmaf(r.a[g], r.a[g], -r.l[g]);
      const float z2 = __builtin_fmaf(-r.a[g], r.a[g], r.h[g]);
      s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(z1), 31);
      s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(z2), 31);
    } else if (ENC == 1) {
      const float z1 = __builtin_fmaf(r.a[g], r.a[g], -r.l[g]);
      const float z2 = __builtin_fmaf(-r.a[g], r.a[g], r.h[g]);
      s1[g] = (s1[g] << 1) | (__float_as_uint(z1) >> 31);
      s2[g] = (s2[g] << 1) | (__float_as_uint(z2) >> 31);
    } else {
      const float aa = r.a[g] * r.a[g];
      const float z1 = aa - r.l[g];
      const float z2 = r.h[g] - aa;
      s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(z1), 31);
      s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(z2), 31);
    }
  }
}

template <int W, int MODE>
__global__ __launch_bounds__(256 * W) __attribute__((amdgpu_waves_per_eu(W, W)))
void k_probe(const _Float16* __restrict__ in, uint32_t* __restrict__ out, unsigned long long* __restrict__ cyc,
             int iters) {
  __shared__ __attribute__((aligned(16))) _Float16 frag[kTiles][3][64][8];
  const int tid = threadIdx.x, lane = tid & 63;
  for (int i = tid; i < kTiles * 3 * 64 * 8; i += blockDim.x) (&frag[0][0][0][0])[i] = in[4096 + (i & 4095)];
  h8 A1, A2, AL, AH;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    A1[i] = in[lane * 8 + i];
    A2[i] = in[512 + lane * 8 + i];
    AL[i] = in[1024 + lane * 8 + i];
    AH[i] = in[1536 + lane * 8 + i];
  }
  uint32_t s1[16], s2[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) { s1[g] = g; s2[g] = 3 * g; }
  Acc r0, r1;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    r0.a[g] = (float)in[2048 + g]; r0.l[g] = (float)in[2080 + g]; r0.h[g] = (float)in[2112 + g];
  }
  r1 = r0;
  __syncthreads();
  const h8* fr = reinterpret_cast<const h8*>(&frag[0][0][0][0]);
  auto ld = [&](int t, h8& b1, h8& b2, h8& bd) {
    b1 = fr[(t * 3 + 0) * 64 + lane];
    b2 = fr[(t * 3 + 1) * 64 + lane];
    bd = fr[(t * 3 + 2) * 64 + lane];
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (MODE == 0 || MODE == 6) {
    h8 b1, b2, bd;
    ld(0, b1, b2, bd);
    for (int it = 0; it < iters; ++it) {
      const int t = it % kTiles;
      h8 c1 = b1, c2 = b2, cd = bd;
      ld(t + 1 < kTiles ? t + 1 : 0, b1, b2, bd);
      const Acc r = tile_mfma(A1, A2, AL, AH, c1, c2, cd);
      if (MODE == 0) decide<0>(r, s1, s2); else decide<1>(r, s1, s2);
    }
  } else if (MODE == 1 || MODE == 7) {
    h8 b1, b2, bd;
    ld(0, b1, b2, bd);
    r0 = tile_mfma(A1, A2, AL, AH, b1, b2, bd);
    for (int it = 0; it < iters; it += 2) {
      const int t = it % kTiles;
      ld(t + 1, b1, b2, bd);
      r1 = tile_mfma(A1, A2, AL, AH, b1, b2, bd);
      if (MODE == 1) decide<0>(r0, s1, s2); else decide<1>(r0, s1, s2);
      ld(t + 2 < kTiles ? t + 2 : 0, b1, b2, bd);
      r0 = tile_mfma(A1, A2, AL, AH, b1, b2, bd);
      if (MODE == 1) decide<0>(r1, s1, s2); else decide<1>(r1, s1, s2);
    }
  } else if (MODE == 2) {
    h8 b1, b2, bd;
    ld(0, b1, b2, bd);
    for (int it = 0; it < iters; ++it) {
      const int t = it % kTiles;
      h8 c1 = b1, c2 = b2, cd = bd;
      ld(t + 1 < kTiles ? t + 1 : 0, b1, b2, bd);
      const Acc r = tile_mfma(A1, A2, AL, AH, c1, c2, cd);
#pragma unroll
      for (int g = 0; g < 16; g += 4) s1[g] ^= __float_as_uint(r.a[g] + r.l[g] + r.h[g]);
    }
  } else if (MODE >= 3 && MODE <= 5) {
    for (int it = 0; it < iters; ++it) {
      r0.a[it & 15] += 1.0f;
      if (MODE == 3) decide<0>(r0, s1, s2);
      else if (MODE == 4) decide<1>(r0, s1, s2);
      else decide<2>(r0, s1, s2);
    }
  } else {
    for (int it = 0; it < iters; ++it) {
      r0.a[it & 15] += 1.0f;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        if (MODE == 8) {
          s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(r0.a[g]), 31);
          s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(r0.l[g]), 31);
          s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(r0.h[g]), 31);
          s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(r0.a[g]), 30);
        } else if (MODE == 9) {
          s1[g] = (s1[g] << 1) | __float_as_uint(r0.a[g]);
          s2[g] = (s2[g] << 1) | __float_as_uint(r0.l[g]);
          s1[g] = (s1[g] << 2) | __float_as_uint(r0.h[g]);
          s2[g] = (s2[g] << 2) | __float_as_uint(r0.a[g]);
        } else {
          r0.l[g] = __builtin_fmaf(r0.a[g], r0.a[g], -r0.l[g]);
          r0.h[g] = __builtin_fmaf(-r0.a[g], r0.a[g], r0.h[g]);
          r0.l[g] = __builtin_fmaf(r0.a[g], r0.l[g], -r0.h[g]);
          r0.h[g] = __builtin_fmaf(-r0.a[g], r0.h[g], r0.l[g]);
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int g = 0; g < 16; ++g)
    acc += s1[g] ^ s2[g] ^ __float_as_uint(r0.l[g] + r0.h[g] + r1.a[g]);
  out[blockIdx.x * blockDim.x + tid] = acc;
  if (lane == 0) cyc[blockIdx.x * 16 + (tid >> 6)] = t1 - t0;
}

typedef void (*KFn)(const _Float16*, uint32_t*, unsigned long long*, int);

struct V { const char* name; int w; KFn fn; };

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int iters = 24 * 800;
  std::vector<_Float16> hin(8192);
  srand(7);
  for (auto& v : hin) v = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.25f);
  _Float16* in;
  uint32_t* out;
  unsigned long long* cyc;
  hipMalloc(&in, hin.size() * 2);
  hipMemcpy(in, hin.data(), hin.size() * 2, hipMemcpyHostToDevice);
  hipMalloc(&out, (size_t)cus * 1024 * 4);
  hipMalloc(&cyc, (size_t)cus * 16 * 8);
#define VV(W, M, N) {N, W, k_probe<W, M>}
  V vs[] = {
      VV(3, 0, "loop (1 acc set, alignbit)"), VV(2, 0, "loop (1 acc set, alignbit)"),
      VV(4, 0, "loop (1 acc set, alignbit)"),
      VV(2, 1, "loop, 2 acc sets, alignbit"), VV(3, 1, "loop, 2 acc sets, alignbit"),
      VV(3, 6, "loop (1 acc set, shl|shr)"), VV(3, 7, "loop, 2 acc sets, shl|shr"),
      VV(2, 7, "loop, 2 acc sets, shl|shr"), VV(4, 6, "loop (1 acc set, shl|shr)"),
      VV(3, 2, "MFMA only"), VV(2, 2, "MFMA only"),
      VV(3, 3, "decisions only (fma+alignbit)"), VV(3, 4, "decisions only (fma+shl|shr)"),
      VV(3, 5, "decisions only (mul, 2 sub, alignbit)"),
      VV(3, 8, "64 alignbit"), VV(3, 9, "64 lshl_or"), VV(3, 10, "64 fma"),
      VV(2, 8, "64 alignbit"), VV(2, 10, "64 fma"),
  };
  std::vector<unsigned long long> h(cus * 16);
  for (const V& v : vs) {
    const int threads = 256 * v.w;
    hipLaunchKernelGGL(v.fn, dim3(cus), dim3(threads), 0, 0, in, out, cyc, 240);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(v.fn, dim3(cus), dim3(threads), 0, 0, in, out, cyc, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h.data(), cyc, (size_t)cus * 16 * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    const int nw = 4 * v.w;
    for (int b = 0; b < cus; ++b)
      for (int w = 0; w < nw; ++w) mean += (double)h[b * 16 + w];
    mean /= (double)cus * nw;
    printf("W=%d %-40s %8.3f ms  %7.1f wave cyc/tile  %6.1f SIMD cyc/tile  clock %.2f GHz\n", v.w, v.name, ms,
           mean / iters, mean / iters / v.w, mean / (ms * 1e6));
  }
  return 0;
}
