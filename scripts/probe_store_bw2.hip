// Probe 2: pure HBM write bandwidth on gfx950 by store width, cache policy,
// per-block span and grid shape.  Writes a flat 7.72 GB fp32 buffer (the
// KITTI L=128 B=8 cost-volume size) so every byte goes to HBM.
//   S<V,NT,U>  : block of 256 threads writes one contiguous span of
//                256*V*U floats with U unrolled stores of V floats per lane
//                (each store instruction covers 256*V*4 contiguous bytes)
//   G<V,NT>    : grid-stride loop, grid = nblk blocks
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int V> struct Vec;
template <> struct Vec<1> { typedef float T; };
template <> struct Vec<2> { typedef f2 T; };
template <> struct Vec<4> { typedef f4 T; };

template <int V, bool NT, int U>
__global__ __launch_bounds__(256) void kS(float* out, size_t n) {
  typedef typename Vec<V>::T T;
  const size_t base = (size_t)blockIdx.x * (256 * V * U);
  T v;
  for (int k = 0; k < V; ++k) ((float*)&v)[k] = (float)k;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t i = base + ((size_t)u * 256 + threadIdx.x) * V;
    if (i + V <= n) {
      T* d = (T*)(out + i);
      if (NT) __builtin_nontemporal_store(v, d); else *d = v;
    }
  }
}

template <int V, bool NT>
__global__ __launch_bounds__(256) void kG(float* out, size_t n) {
  typedef typename Vec<V>::T T;
  T v;
  for (int k = 0; k < V; ++k) ((float*)&v)[k] = (float)k;
  const size_t nv = n / V;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < nv; i += (size_t)gridDim.x * 256) {
    T* d = (T*)out + i;
    if (NT) __builtin_nontemporal_store(v, d); else *d = v;
  }
}


// The cost-volume's own item shapes: [8][64 rows][128 planes][94*311] fp32,
// items (b, grp, l, pw) in address order, grp < 32: one row, else a quad of
// rows; a 1024-pixel window per item, lane-consecutive 4-byte stores
// (sweep_lane_pixels=0) or 4 pixels per lane with 16-byte stores (LP4).
template <int IPB, bool LP4, int QROWS>
__global__ __launch_bounds__(256) void kVol(float* out) {
  constexpr int HW = 94 * 311, L = 128, ROWS = 64, REF = 32;
  constexpr int GROUPS = REF + (ROWS - REF) / QROWS;
  constexpr int NPW = (HW + 3 + 1023) / 1024;
  const int total = 8 * GROUPS * L * NPW;
  for (int it = 0; it < IPB; ++it) {
    const int item = blockIdx.x * IPB + it;
    if (item >= total) return;
    const int pw = item % NPW; int r = item / NPW;
    const int l = r % L; r /= L;
    const int grp = r % GROUPS; const int b = r / GROUPS;
    const int nrow = grp < REF ? 1 : QROWS;
    const int row0 = grp < REF ? grp : REF + (grp - REF) * QROWS;
    const int shift = 2 * (l & 1);
    for (int k = 0; k < nrow; ++k) {
      float* row = out + (((size_t)b * ROWS + row0 + k) * L + l) * HW;
      if (LP4) {
        const int p = pw * 1024 - shift + threadIdx.x * 4;
        f4 v = {1.f, 2.f, 3.f, (float)k};
        if (p >= 0 && p + 3 < HW) *(f4*)(row + p) = v;
        else for (int j = 0; j < 4; ++j) if (p + j >= 0 && p + j < HW) row[p + j] = v[j];
      } else {
        const int wb = pw * 1024 - shift + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int p = wb + 64 * j;
          if (p >= 0 && p < HW) row[p] = (float)k;
        }
      }
    }
  }
}


// Same volume, but items are 256-byte-aligned 1024-float windows of each
// channel slab [b][row][L*hw] (a window may straddle two planes): every
// wave store is one aligned 256-B segment.  QROWS rows share a window.
template <int IPB, int QROWS, int REF>
__global__ __launch_bounds__(256) void kVolA(float* out) {
  constexpr int HW = 94 * 311, L = 128, ROWS = 64;
  constexpr int GROUPS = REF + (ROWS - REF) / QROWS;
  constexpr int SLAB = L * HW;
  constexpr int NW = (SLAB + 1023) / 1024;
  const int total = 8 * GROUPS * NW;
  for (int it = 0; it < IPB; ++it) {
    const int item = blockIdx.x * IPB + it;
    if (item >= total) return;
    const int wi = item % NW; const int r = item / NW;
    const int grp = r % GROUPS; const int b = r / GROUPS;
    const int nrow = grp < REF ? 1 : QROWS;
    const int row0 = grp < REF ? grp : REF + (grp - REF) * QROWS;
    const int wb = wi * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
    for (int k = 0; k < nrow; ++k) {
      float* slab = out + ((size_t)b * ROWS + row0 + k) * SLAB;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = wb + 64 * j;
        if (p < SLAB) slab[p] = (float)k;
      }
    }
  }
}

template <typename F>
static int timeit(const char* name, F launch, double bytes) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  launch(); launch();
  CK(hipDeviceSynchronize());
  const int reps = 5;
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= reps;
  printf("%-40s %8.3f ms  %8.1f GB/s\n", name, ms, bytes / (ms * 1e6));
  fflush(stdout);
  CK(hipGetLastError());
  return 0;
}

int main() {
  const size_t n = (size_t)8 * 64 * 128 * 94 * 311;   // 1.93e9 floats = 7.72 GB
  float* out;
  CK(hipMalloc(&out, n * 4 + 4096));
  const double bytes = (double)n * 4;
#define RUN_S(V, NT, U)                                                                   \
  {                                                                                       \
    const size_t span = (size_t)256 * V * U;                                              \
    const unsigned g = (unsigned)((n + span - 1) / span);                                 \
    char nm[64]; snprintf(nm, 64, "span V=%d nt=%d U=%d", V, (int)NT, U);                  \
    if (timeit(nm, [&] { kS<V, NT, U><<<g, 256>>>(out, n); }, bytes)) return 1;           \
  }
#define RUN_G(V, NT, NB)                                                                  \
  {                                                                                       \
    char nm[64]; snprintf(nm, 64, "gridstride V=%d nt=%d blocks=%d", V, (int)NT, NB);       \
    if (timeit(nm, [&] { kG<V, NT><<<NB, 256>>>(out, n); }, bytes)) return 1;             \
  }

#define RUN_V(IPB, LP4, Q)                                                                \
  {                                                                                       \
    constexpr int GROUPS = 32 + 32 / Q, NPW = (94 * 311 + 3 + 1023) / 1024;               \
    const unsigned g = (unsigned)((8 * GROUPS * 128 * NPW + IPB - 1) / IPB);              \
    char nm[64]; snprintf(nm, 64, "volume ipb=%d lp4=%d quad=%d", IPB, (int)LP4, Q);        \
    if (timeit(nm, [&] { kVol<IPB, LP4, Q><<<g, 256>>>(out); }, bytes)) return 1;         \
  }

#define RUN_A(IPB, Q, REF)                                                                \
  {                                                                                       \
    constexpr int GROUPS = REF + (64 - REF) / Q, NW = (128 * 94 * 311 + 1023) / 1024;     \
    const unsigned g = (unsigned)((8 * GROUPS * NW + IPB - 1) / IPB);                     \
    char nm[64]; snprintf(nm, 64, "aligned ipb=%d quad=%d ref=%d", IPB, Q, REF);           \
    if (timeit(nm, [&] { kVolA<IPB, Q, REF><<<g, 256>>>(out); }, bytes)) return 1;        \
  }
  RUN_A(1, 1, 32) RUN_A(2, 1, 32) RUN_A(1, 4, 32) RUN_A(2, 4, 32) RUN_A(4, 4, 32) RUN_A(1, 8, 32) RUN_A(1, 2, 32)
  RUN_A(1, 4, 0) RUN_A(1, 8, 0) RUN_A(1, 16, 0)
  RUN_V(1, false, 4) RUN_V(2, false, 4) RUN_V(4, false, 4) RUN_V(1, true, 4) RUN_V(4, true, 4)
  RUN_V(1, false, 1) RUN_V(4, false, 1) RUN_V(1, false, 2) RUN_V(1, false, 8)
  RUN_S(1, false, 4) RUN_S(1, false, 16) RUN_S(1, true, 16)
  RUN_S(2, false, 4) RUN_S(2, false, 16) RUN_S(2, true, 16)
  RUN_S(4, false, 1) RUN_S(4, false, 4) RUN_S(4, false, 16) RUN_S(4, true, 4) RUN_S(4, true, 16)
  RUN_G(1, false, 2048) RUN_G(1, false, 8192) RUN_G(1, true, 8192)
  RUN_G(2, false, 2048) RUN_G(2, false, 8192)
  RUN_G(4, false, 1024) RUN_G(4, false, 2048) RUN_G(4, false, 4096) RUN_G(4, false, 8192) RUN_G(4, true, 2048)
  CK(hipFree(out));
  return 0;
}
