// Probe: HBM write bandwidth of the cost-volume store shapes on gfx950.
// Writes a [B=8][64][128][94*311] fp32 volume (7.66 GB) with
//   A) per-thread 2 px x 64 rows, float2 non-temporal stores (current sweep)
//   B) same with plain stores
//   C) per-thread 4 px, float4 stores, 16-B aligned windows (rows aligned per plane parity)
//   D) flat contiguous float4 grid-stride memset-like stream (ceiling)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int B = 8, CH = 64, L = 128, HW = 94 * 311;

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void kA(float* out) {
  const int pix_blocks = (HW + 511) / 512;
  int bid = blockIdx.x;
  const int b = bid % B; bid /= B;
  const int pg = bid % (L / 16); const int pb = bid / (L / 16);
  const int p0 = (pb * 256 + threadIdx.x) * 2;
  if (pb >= pix_blocks || p0 >= HW) return;
  float* O = out + (size_t)b * CH * L * HW + p0;
  for (int l = pg * 16; l < pg * 16 + 16; ++l)
    for (int c = 0; c < CH; ++c) {
      f2 v = {(float)c, (float)l};
      f2* d = (f2*)(O + ((size_t)c * L + l) * HW);
      if (NT) __builtin_nontemporal_store(v, d); else *d = v;
    }
}

// float4 windows: row base parity decides a 2-element shift
__global__ __launch_bounds__(256) void kC(float* out) {
  const int win = (HW + 3 + 1023) / 1024;   // 1024 px per block (256 thr x 4)
  int bid = blockIdx.x;
  const int b = bid % B; bid /= B;
  const int pg = bid % (L / 16); const int pb = bid / (L / 16);
  if (pb >= win) return;
  for (int l = pg * 16; l < pg * 16 + 16; ++l) {
    const size_t rb0 = ((size_t)(b * CH) * L + l) * HW;
    const int shift = (int)(rb0 & 3);              // same for every channel row of plane l (L even)
    const int p = (pb * 256 + threadIdx.x) * 4 - shift;
    for (int c = 0; c < CH; ++c) {
      float* row = out + ((size_t)(b * CH + c) * L + l) * HW;
      f4 v = {(float)c, (float)l, 1.f, 2.f};
      if (p >= 0 && p + 3 < HW) __builtin_nontemporal_store(v, (f4*)(row + p));
      else for (int k = 0; k < 4; ++k) if (p + k >= 0 && p + k < HW) row[p + k] = v[k];
    }
  }
}

// float4 windows, c outer / l inner (consecutive planes of one channel are contiguous)
template <bool NT, int LG>
__global__ __launch_bounds__(256) void kG(float* out) {
  const int win = (HW + 3 + 1023) / 1024;
  int bid = blockIdx.x;
  const int b = bid % B; bid /= B;
  const int pg = bid % (L / LG); const int pb = bid / (L / LG);
  if (pb >= win) return;
  for (int c = 0; c < CH; ++c) {
    for (int l = pg * LG; l < pg * LG + LG; ++l) {
      const size_t rb = ((size_t)(b * CH + c) * L + l) * HW;
      const int p = (pb * 256 + threadIdx.x) * 4 - (int)(rb & 3);
      float* row = out + rb;
      f4 v = {(float)c, (float)l, 1.f, 2.f};
      if (p >= 0 && p + 3 < HW) { if (NT) __builtin_nontemporal_store(v, (f4*)(row + p)); else *(f4*)(row + p) = v; }
      else for (int k = 0; k < 4; ++k) if (p + k >= 0 && p + k < HW) row[p + k] = v[k];
    }
  }
}

// C with plain stores
__global__ __launch_bounds__(256) void kE(float* out) {
  const int win = (HW + 3 + 1023) / 1024;
  int bid = blockIdx.x;
  const int b = bid % B; bid /= B;
  const int pg = bid % (L / 16); const int pb = bid / (L / 16);
  if (pb >= win) return;
  for (int l = pg * 16; l < pg * 16 + 16; ++l) {
    const size_t rb0 = ((size_t)(b * CH) * L + l) * HW;
    const int shift = (int)(rb0 & 3);
    const int p = (pb * 256 + threadIdx.x) * 4 - shift;
    for (int c = 0; c < CH; ++c) {
      float* row = out + ((size_t)(b * CH + c) * L + l) * HW;
      f4 v = {(float)c, (float)l, 1.f, 2.f};
      if (p >= 0 && p + 3 < HW) *(f4*)(row + p) = v;
      else for (int k = 0; k < 4; ++k) if (p + k >= 0 && p + k < HW) row[p + k] = v[k];
    }
  }
}

// item order (b, g, l, pw) with pw fastest; each item writes RPI rows x 1024 px
template <int RPI, int IPB, int CSTRIDE = 1>
__global__ __launch_bounds__(256) void kItems(float* out) {
  constexpr int NPW = (HW + 3 + 1023) / 1024;
  constexpr int G = CH / RPI;
  const int total = B * G * L * NPW;
  for (int it = 0; it < IPB; ++it) {
    const int item = blockIdx.x * IPB + it;
    if (item >= total) return;
    const int pw = item % NPW; int r = item / NPW;
    const int l = r % L; r /= L;
    const int g = r % G; const int b = r / G;
    const int p = pw * 1024 - 2 * (l & 1) + threadIdx.x * 4;
    for (int k = 0; k < RPI; ++k) {
      const int c = CSTRIDE == 1 ? g * RPI + k : g + k * (CH / RPI);
      float* row = out + ((size_t)(b * CH + c) * L + l) * HW;
      f4 v = {(float)k, (float)l, 1.f, 2.f};
      if (p >= 0 && p + 3 < HW) *(f4*)(row + p) = v;
      else for (int j = 0; j < 4; ++j) if (p + j >= 0 && p + j < HW) row[p + j] = v[j];
    }
  }
}

// flat 1-row items copying a source row (re-read for every plane, L2-resident)
// LD: 0 = no load (constant), 1 = 4 scalar loads, 2 = 2 x float2 loads
template <int LD, int IPB>
__global__ __launch_bounds__(256) void kCopy(const float* __restrict__ src, float* out) {
  constexpr int NPW = (HW + 3 + 1023) / 1024;
  const int total = B * CH * L * NPW;
  for (int it = 0; it < IPB; ++it) {
    const int item = blockIdx.x * IPB + it;
    if (item >= total) return;
    const int pw = item % NPW; int r = item / NPW;
    const int l = r % L; r /= L;
    const int c = r % CH; const int b = r / CH;
    const int p = pw * 1024 - 2 * (l & 1) + threadIdx.x * 4;
    const float* S = src + ((size_t)b * 32 + (c & 31)) * HW;
    f4 v;
    if (LD == 0) {
      v = f4{(float)c, (float)l, 1.f, 2.f};
    } else if (LD == 1) {
      for (int j = 0; j < 4; ++j) v[j] = S[min(max(p + j, 0), HW - 1)];
    } else {
      const int q = min(max(p, 0), HW - 4);
      const f2 a = *(const f2*)(S + (q & ~1)), bb = *(const f2*)(S + (q & ~1) + 2);
      v = f4{a[0], a[1], bb[0], bb[1]};
    }
    float* row = out + ((size_t)(b * CH + c) * L + l) * HW;
    if (p >= 0 && p + 3 < HW) *(f4*)(row + p) = v;
    else for (int j = 0; j < 4; ++j) if (p + j >= 0 && p + j < HW) row[p + j] = v[j];
  }
}

__global__ void kD(f4* out, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    f4 v = {1.f, 2.f, 3.f, 4.f};
    __builtin_nontemporal_store(v, out + i);
  }
}

int main() {
  const size_t n = (size_t)B * CH * L * HW;
  float* out;
  CK(hipMalloc(&out, n * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  auto run = [&](const char* name, auto launch) {
    launch(); CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(a)); launch(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
    }
    printf("%-40s %8.3f ms  %8.1f GB/s\n", name, best, n * 4 / (best * 1e-3) / 1e9);
    return 0;
  };
  const int gA = ((HW + 511) / 512) * (L / 16) * B;
  const int gC = ((HW + 3 + 1023) / 1024) * (L / 16) * B;
  run("E float4 plain aligned windows", [&] { hipLaunchKernelGGL(kE, dim3(gC), dim3(256), 0, 0, out); });
  constexpr int NPW = (HW + 3 + 1023) / 1024;
  run("P1 items 4 rows, ipb 4", [&] { hipLaunchKernelGGL((kItems<4, 4>), dim3((B * 16 * L * NPW + 3) / 4), dim3(256), 0, 0, out); });
  run("P1s items 4 rows stride 16 ch, ipb 4", [&] { hipLaunchKernelGGL((kItems<4, 4, 16>), dim3((B * 16 * L * NPW + 3) / 4), dim3(256), 0, 0, out); });
  run("P3 items 1 row (flat), ipb 4", [&] { hipLaunchKernelGGL((kItems<1, 4>), dim3((B * 64 * L * NPW + 3) / 4), dim3(256), 0, 0, out); });
  run("P4 items 2 rows, ipb 4", [&] { hipLaunchKernelGGL((kItems<2, 4>), dim3((B * 32 * L * NPW + 3) / 4), dim3(256), 0, 0, out); });
  run("D float4 nt flat stream", [&] { hipLaunchKernelGGL(kD, dim3(8192), dim3(256), 0, 0, (f4*)out, n / 4); });
  float* src;
  CK(hipMalloc(&src, (size_t)B * 32 * HW * 4));
  {
    std::vector<float> h((size_t)B * 32 * HW);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.001f + 0.5f;
    CK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  }
  run("C0 copy items, no load, ipb 4", [&] { hipLaunchKernelGGL((kCopy<0, 4>), dim3((B * 64 * L * NPW + 3) / 4), dim3(256), 0, 0, src, out); });
  run("C1 copy items, 4 scalar loads, ipb 4", [&] { hipLaunchKernelGGL((kCopy<1, 4>), dim3((B * 64 * L * NPW + 3) / 4), dim3(256), 0, 0, src, out); });
  run("C2 copy items, 2 float2 loads, ipb 4", [&] { hipLaunchKernelGGL((kCopy<2, 4>), dim3((B * 64 * L * NPW + 3) / 4), dim3(256), 0, 0, src, out); });
  CK(hipFree(src));
  CK(hipFree(out));
  return 0;
}
