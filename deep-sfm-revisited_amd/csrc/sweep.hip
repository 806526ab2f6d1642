// Plane-sweep cost volume and inverse warp on CDNA4 (gfx950).
//
// Replaces the per-plane Python loop of models/PSNet.py:144-158 (L iterations
// of ~10 ATen launches: bmm, elementwise, grid_sample, two strided copies)
// with one launch that writes the whole [B, 2C, L, h, w] volume (plus a tiny
// channel-quad relayout of the target features).  HBM-write-bound.
//
// Arithmetic: warp.h (the reference's float32 expression order).
#include <algorithm>
#include <string>
#include "warp.h"

namespace sfm {

// ---------------------------------------------------------------------------
// Cost volume: the output is produced in address order.
//
// The [B, 2C, L, h, w] volume is cut into work items of 1024 consecutive
// pixels (256 threads x 4, one 16-byte store per thread per row):
//   * reference rows c < C: one item = one row segment (pure copy)
//   * warped rows: one item = the same segment of a channel QUAD (4 rows),
//     so the sampling position, mask and bilinear taps of a pixel are computed
//     once for 4 channels and each tap is one 16-byte load from the
//     channel-quad layout tq[B][C4][h*w][4] of the target features.
// Items are enumerated in the volume's memory order (window fastest, then
// plane, then row / quad, then pair) and each block takes `ipb` consecutive
// items, so the resident blocks sweep one contiguous window of the volume.
// MI355X write bandwidth drops with the number of interleaved store streams
// (git-history scripts/probe_store_bw.hip: 1 stream 4.9 TB/s, 2 -> 4.5, 4 -> 4.0, many
// scattered row chunks -> 3.7): the copy half therefore runs as a single
// stream, the warped half as 4 (the price of sharing the taps; one row per
// item would need ~45 VALU ops and 5 vector loads per output element).
//
// 16-byte alignment: a row starts at element ((b*rows + r)*L + l)*h*w.  With
// h*w = 2 (mod 4) and L even, that is 2*(l & 1) (mod 4) for every row of the
// plane, so the pixel windows of odd planes are shifted by 2.  Other shapes
// take the element-wise store path (correct, slower).
// ---------------------------------------------------------------------------
constexpr int kSwThreads = 256;
constexpr int kSwPix = 4;
constexpr int kSwWin = kSwThreads * kSwPix;

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float plane_depth(float dmax, float dstep, int l) {
  // PSNet.py:150-153: depth planes (i+1)*MIN_DEPTH, or disp2depth / (i+1)
  return dstep > 0.0f ? (float)(l + 1) * dstep : dmax / (float)(l + 1);
}

// The tensor preparation of PSNet.forward before its sweep loop, one thread per
// pair (run by k_tgt_quads, before that pair's Proj), in the reference's float32 operations (PSNet.py:130-133 and the
// RESCALE_DEPTH branch): P.float() (RNE from float64), translation * t_scale,
// K rows 0-1 / 4, K^-1[:2,:2] * 4.  Division by 4 and multiplication by 4
// are exact, and the conversion and the one multiply are correctly rounded,
// so the results equal the torch ops bit for bit.
struct PsnetPrep {          // sfm_plane_sweep_psnet's inputs (PSNet.py:130-133 + RESCALE_DEPTH)
  const void* pose;
  int pose_f64;
  const float* K;
  const float* Kinv;
  float t_scale;
  float* out;               // planar: B poses (12), then B K4 (9), then B K4inv (9)
};

// one pair's preparation into P[12], K4[9], Ki4[9] (registers), also stored
// to the workspace for the sweep kernels that read them from there
__device__ __forceinline__ void psnet_prep_pair(const PsnetPrep& q, int B, int b, float (&P)[12], float (&K4)[9],
                                                float (&Ki4)[9]) {
#pragma unroll
  for (int e = 0; e < 12; ++e) {
    float v = q.pose_f64 ? (float)static_cast<const double*>(q.pose)[(size_t)b * 12 + e]
                         : static_cast<const float*>(q.pose)[(size_t)b * 12 + e];
    if (q.t_scale > 0.0f && (e & 3) == 3) v = v * q.t_scale;
    P[e] = v;
    q.out[(size_t)b * 12 + e] = v;
  }
#pragma unroll
  for (int e = 0; e < 9; ++e) {
    const float k = q.K[(size_t)b * 9 + e], ki = q.Kinv[(size_t)b * 9 + e];
    K4[e] = e < 6 ? k / 4.0f : k;
    Ki4[e] = (e == 0 || e == 1 || e == 3 || e == 4) ? ki * 4.0f : ki;
    q.out[(size_t)B * 12 + (size_t)b * 9 + e] = K4[e];
    q.out[(size_t)B * 21 + (size_t)b * 9 + e] = Ki4[e];
  }
}

// tgt [B][C][hw] -> tq [B][C4][hw] float4 (channels >= C are zero).  With
// `projs`, threads 0..B-1 also write each pair's Proj (K.pose rows and K^-1,
// load_proj's float32 expression order), so the sweep's waves read it with
// scalar loads instead of each recomputing the uniform 3x3.3x4 product on the
// VALU (~80 instructions per wave item); threads 0..L-1 the plane depths
// (two IEEE divisions per wave item otherwise).
__global__ void k_tgt_quads(const float* __restrict__ tgt, int B, int C, int C4, int hw, f32x4* __restrict__ tq,
                            const float* __restrict__ pose, const float* __restrict__ K4,
                            const float* __restrict__ K4inv, Proj* __restrict__ projs, int L, float dmax,
                            float dstep, float* __restrict__ depths, PsnetPrep prep) {
  // grid (pixels, quads, pairs): no integer division per thread; the uniform
  // per-pair and per-plane tables from the first quad row of pair 0
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int q = (int)blockIdx.y, b = (int)blockIdx.z;
  if (q == 0 && b == 0) {
    if (projs && i < B) {
      // sfm_plane_sweep_psnet: the pair's PSNet preparation first (the sweep's
      // other paths read it from the workspace), then its Proj from those values
      Proj pr;
      if (prep.out) {
        float P[12], Kq[9], Kqi[9];
        psnet_prep_pair(prep, B, i, P, Kq, Kqi);
        load_proj(P, Kq, Kqi, 0, pr);
      } else {
        load_proj(pose, K4, K4inv, i, pr);
      }
      projs[i] = pr;
    }
    if (depths && i < L) depths[i] = plane_depth(dmax, dstep, i);
  }
  if (i >= hw) return;
  f32x4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * q + k;
    v[k] = c < C ? tgt[((size_t)b * C + c) * hw + i] : 0.0f;
  }
  tq[((size_t)b * C4 + q) * hw + i] = v;
}

static dim3 quads_grid(int B, int C4, int hw, int extra) {
  return dim3((unsigned)((std::max(hw, extra) + 255) / 256), (unsigned)C4, (unsigned)B);
}

void launch_channel_quads(const float* feat, int B, int C, int hw, f32x4* quads, hipStream_t s) {
  const int C4 = (C + 3) / 4;
  hipLaunchKernelGGL(k_tgt_quads, quads_grid(B, C4, hw, 0), dim3(256), 0, s, feat, B, C, C4, hw, quads,
                     nullptr, nullptr, nullptr, nullptr, 0, 0.0f, 0.0f, nullptr, PsnetPrep{});
}

__device__ __forceinline__ void store4(float* dst, const float (&v)[4]) {
  *reinterpret_cast<f32x4*>(dst) = f32x4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ void store4(unsigned short* dst, const float (&v)[4]) {
  u32x2 u;
  u[0] = (unsigned int)to_bf16(v[0]) | ((unsigned int)to_bf16(v[1]) << 16);
  u[1] = (unsigned int)to_bf16(v[2]) | ((unsigned int)to_bf16(v[3]) << 16);
  *reinterpret_cast<u32x2*>(dst) = u;
}
__device__ __forceinline__ void store1(float* dst, float v) { *dst = v; }
__device__ __forceinline__ void store1(unsigned short* dst, float v) { *dst = to_bf16(v); }

// VEC: rows are 16-byte aligned at the (shifted) window starts (see above)
template <typename OutT, bool VEC>
__device__ __forceinline__ void store_row(OutT* row, int p0, int hw, const float (&v)[4]) {
  if (VEC && p0 >= 0 && p0 + 3 < hw) {
    store4(row + p0, v);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (p0 + j >= 0 && p0 + j < hw) store1(row + p0 + j, v[j]);
  }
}

struct SweepGeom {
  int B, C, C4, h, w, L;
  int ref_rows;    // C (full volume) or 0 (warped half only)
  int rows;        // output rows per plane: ref_rows + C
  int groups;      // row groups per pair: ref_rows single rows + C4 quads
  int npw;         // pixel windows per row
  int shift_mode;  // 1: odd planes' windows shifted by 2 elements
  float dmax;      // MIN_DEPTH * L
  float dstep;     // > 0: PREDICT_BY_DEPTH planes d_i = (i + 1) * dstep
};

// one warped item: 4 channels of the window at plane l
template <typename OutT> __device__ __forceinline__ void store1_nt(OutT* dst, float v);
template <> __device__ __forceinline__ void store1_nt<float>(float* dst, float v) { __builtin_nontemporal_store(v, dst); }
template <> __device__ __forceinline__ void store1_nt<unsigned short>(unsigned short* dst, float v) {
  __builtin_nontemporal_store(to_bf16(v), dst);
}

template <typename OutT, bool VEC, bool LANE_PIX, bool NT = false>
__device__ __forceinline__ void warp_quad(const f32x4* __restrict__ tq, const float* __restrict__ pose,
                                          const float* __restrict__ K4, const float* __restrict__ K4inv,
                                          const SweepGeom& g, int b, int q, int l, int p0, OutT* plane,
                                          size_t rstride) {
  const int hw = g.h * g.w;
  Proj pr;
  load_proj(pose, K4, K4inv, b, pr);
  // PSNet.py:150-153: depth planes (i+1)*MIN_DEPTH, or disp2depth / (i+1)
  const float d = g.dstep > 0.0f ? (float)(l + 1) * g.dstep : g.dmax / (float)(l + 1);
  const f32x4* T = tq + ((size_t)b * g.C4 + q) * hw;
  f32x4 acc[4];
  // LANE_PIX: pixel j of this lane is p0 + j (one 16-byte store per row);
  // otherwise the window's pixels are lane-consecutive (w0 + 64 j + lane, with
  // w0 = the wave's 256-pixel span), so each gather instruction reads
  // neighbouring source pixels, at the price of 4-byte stores.
  const int wave_base = p0 - 4 * (int)(threadIdx.x & 63);
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int pj = LANE_PIX ? p0 + j : wave_base + 64 * j + lane;
    const int p = min(max(pj, 0), hw - 1);
    const float x = (float)(p % g.w), y = (float)(p / g.w);
    float ray[3];
    ray[0] = (pr.ki[0] * x + pr.ki[1] * y) + pr.ki[2];
    ray[1] = (pr.ki[3] * x + pr.ki[4] * y) + pr.ki[5];
    ray[2] = (pr.ki[6] * x + pr.ki[7] * y) + pr.ki[8];
    float ix, iy;
    acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (sample_pos(pr, ray, d, g.h, g.w, ix, iy)) {
      Taps tp;
      make_taps(ix, iy, g.h, g.w, tp);
      const f32x4 t0 = T[tp.off[0]], t1 = T[tp.off[1]], t2 = T[tp.off[2]], t3 = T[tp.off[3]];
      f32x4 a = tp.wt[0] * t0;
      a = a + tp.wt[1] * t1;
      a = a + tp.wt[2] * t2;
      a = a + tp.wt[3] * t3;
      acc[j] = a;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * q + k;
    if (c >= g.C) break;
    OutT* row = plane + (size_t)(g.ref_rows + c) * rstride;
    if (LANE_PIX) {
      const float v[4] = {acc[0][k], acc[1][k], acc[2][k], acc[3][k]};
      store_row<OutT, VEC>(row, p0, hw, v);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int pj = wave_base + 64 * j + lane;
        if (pj >= 0 && pj < hw) {
          if (NT) store1_nt(row + pj, acc[j][k]);
          else store1(row + pj, acc[j][k]);
        }
      }
    }
  }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// 4 reference pixels p0..p0+3 of a row starting at element `row_off` of `ref`.
// Even-aligned interior windows use two 8-byte loads (4 scalar loads per
// thread cap the copy at ~3.6 TB/s on MI355X: the address unit, not HBM, is
// the limit); edges and odd alignments load element-wise with clamping.
__device__ __forceinline__ void load_ref4(const float* __restrict__ ref, size_t row_off, int p0, int hw,
                                          float (&v)[4]) {
  if (p0 >= 0 && p0 + 3 < hw && ((row_off + (size_t)p0) & 1) == 0) {
    const f32x2 a = *reinterpret_cast<const f32x2*>(ref + row_off + p0);
    const f32x2 b = *reinterpret_cast<const f32x2*>(ref + row_off + p0 + 2);
    v[0] = a[0]; v[1] = a[1]; v[2] = b[0]; v[3] = b[1];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = ref[row_off + min(max(p0 + j, 0), hw - 1)];
  }
}

struct ItemPos {
  int pw, l, grp, b;
  __device__ __forceinline__ void decode(int item, const SweepGeom& g) {
    pw = item % g.npw;
    int r = item / g.npw;
    l = r % g.L;
    r /= g.L;
    grp = r % g.groups;
    b = r / g.groups;
  }
  __device__ __forceinline__ void next(const SweepGeom& g) {
    if (++pw == g.npw) {
      pw = 0;
      if (++l == g.L) {
        l = 0;
        if (++grp == g.groups) { grp = 0; ++b; }
      }
    }
  }
};

template <typename OutT, bool VEC, int IPB, bool LANE_PIX = true, bool NT = false>
__global__ __launch_bounds__(kSwThreads) void k_sweep(const float* __restrict__ ref, const f32x4* __restrict__ tq,
                                                      const float* __restrict__ pose, const float* __restrict__ K4,
                                                      const float* __restrict__ K4inv, SweepGeom g,
                                                      OutT* __restrict__ out) {
  const int hw = g.h * g.w;
  const int total = g.B * g.groups * g.L * g.npw;   // < 2^31 (checked by the launcher)
  const int first = blockIdx.x * IPB;
  if (first >= total) return;
  const size_t rstride = (size_t)g.L * hw;
  ItemPos ip;
  ip.decode(first, g);
  ItemPos last;
  last.decode(min(first + IPB, total) - 1, g);
  if (first + IPB <= total && last.b == ip.b && last.grp < g.ref_rows) {
    // copy block: every item is a reference row of pair b.  Issue all loads
    // first (IPB x 16 bytes in flight per thread), then the stores.
    float v[IPB][4];
    int p0s[IPB];
    OutT* dst[IPB];
#pragma unroll
    for (int it = 0; it < IPB; ++it) {
      const int shift = g.shift_mode ? 2 * (ip.l & 1) : 0;
      const int p0 = ip.pw * kSwWin - shift + (int)threadIdx.x * kSwPix;
      p0s[it] = p0;
      dst[it] = out + (((size_t)ip.b * g.rows + ip.grp) * g.L + ip.l) * hw;
      load_ref4(ref, ((size_t)ip.b * g.C + ip.grp) * hw, p0, hw, v[it]);
      ip.next(g);
    }
#pragma unroll
    for (int it = 0; it < IPB; ++it)
      if (p0s[it] < hw) store_row<OutT, VEC>(dst[it], p0s[it], hw, v[it]);
    return;
  }
  for (int it = 0, item = first; it < IPB && item < total; ++it, ++item, ip.next(g)) {
    const int shift = g.shift_mode ? 2 * (ip.l & 1) : 0;
    const int p0 = ip.pw * kSwWin - shift + (int)threadIdx.x * kSwPix;
    OutT* plane = out + ((size_t)ip.b * g.rows * g.L + ip.l) * hw;   // row c at plane + c * rstride
    if (ip.grp < g.ref_rows) {
      if (p0 >= hw) continue;
      float v[4];
      load_ref4(ref, ((size_t)ip.b * g.C + ip.grp) * hw, p0, hw, v);
      store_row<OutT, VEC>(plane + (size_t)ip.grp * rstride, p0, hw, v);
    } else {
      warp_quad<OutT, VEC, LANE_PIX, NT>(tq, pose, K4, K4inv, g, ip.b, ip.grp - g.ref_rows, ip.l, p0, plane, rstride);
    }
  }
}


// ---------------------------------------------------------------------------
// Cost volume, aligned-slab form (default, tuning key sweep_flat = 1).
//
// Each output row (b, r) of the [B, rows, L, h, w] volume is one contiguous
// slab of L*h*w elements.  A work item is a 1024-element window of the slabs
// of one channel group: G = 4*NQ warped rows (channels 4*NQ*k ..) and, for
// the full volume, the G reference rows of the same channels.  Window starts
// are 256-byte aligned in absolute address (a window may straddle two
// planes), so every wave store is one aligned 256-byte segment.
//   * git-history scripts/probe_store_bw2.hip (profiles/r01_probe_store_bw2.txt): stores
//     of this shape run at 6.3-7.0 TB/s on MI355X for 1-8 rows per item, the
//     per-row windows above at 4.0-5.0 (their 256-byte wave segments straddle
//     cache lines: rows start at arbitrary 4-byte offsets).
//   * Pairing the copy rows with the warped rows in one item keeps every
//     block half store-bound, half VALU-bound, so the two overlap on every
//     CU instead of alternating between all-copy and all-warp phases.
//   * One item per block, items in address order (window fastest): the
//     resident blocks sweep a narrow front of the 2G slabs.
//   * Every vector-memory byte passes the CU's 64 B/clk L1 path: per 4-byte
//     output ~8 B of tap gathers (16 B per warped output), 2 B of reference
//     loads and the 4 B store.  Rays K^-1 (x, y, 1) are therefore recomputed
//     (18 VALU) rather than read from a per-pixel table (16 B per pixel and
//     plane; measured 1.36 vs 1.32 ms at KITTI B=8, L=128).
// Arithmetic: the reference's float32 expression order (warp.h
// sample_pos_nr: the same bits as sample_pos with Newton-Raphson divisions),
// the bilinear taps in the in-image form (make_taps_inside), and FMA in the
// 4-tap sum (within 1 ulp of the per-row kernel's mul/add chain).  Uniform
// integer divisions use magic numbers.
// ---------------------------------------------------------------------------
constexpr int kFlatWin = 1024;

struct Magic {   // floor(n / d) = (n * m) >> s for 0 <= n < 2^31
  unsigned m, s;
};
static Magic make_magic(unsigned d) {
  unsigned l = 0;
  while ((1ull << l) < d) ++l;
  const unsigned long long two = 1ull << (31 + l);
  return Magic{(unsigned)((two + d - 1) / d), 31 + l};
}
__device__ __forceinline__ unsigned magic_div(unsigned n, Magic mg) {
  return (unsigned)(((unsigned long long)n * mg.m) >> mg.s);
}

struct FlatGeom {
  int B, C, C4, h, w, L, hw;
  int ref_rows, rows;
  int G;           // channels per group (4 * NQ)
  int groups;      // ceil(C / G) per pair
  int slab;        // L * hw elements
  int nwin;        // windows per slab
  int amask;       // elements per 256 bytes - 1
  int out_mis;     // element offset of the output pointer modulo amask + 1
  int pair_ok;     // bf16: every row starts at an even element (4-byte pair stores)
  int buf_ok;      // k_sweep_tile fast path: per-pair volume, ref and quad ranges < 2^32 bytes, pair_ok
  int share;       // k_sweep_tile fast path: neighbour-lane tap sharing (tuning key sweep_share)
  int store_nt;    // k_sweep_tile fast path: non-temporal volume stores (tuning key sweep_store_nt)
  int write_ref;   // k_sweep_tile: write the reference rows too (0: the warped half only, the reference
                   // half comes from k_ref_planes, e.g. on a side stream beside RANSAC)
  int store_px;    // bf16 fast path: consecutive pixels per lane store (tuning key sweep_store_px; 0: pairs)
  unsigned pair_bytes;   // one pair's output volume in bytes (buffer range)
  Magic mwin, mgrp, mhw;
  float inv_w;
  float dmax, dstep;
  const float* depths;   // plane depths (k_tgt_quads), or null
  int wpol;        // 16-byte stores' cache policy when not -1 (16 sc1, 17 sc0 sc1, 18 nt sc1; sweep_store_wt)
};

template <typename OutT> struct FlatLanes;   // pixels per lane per store, stores per lane per row
template <> struct FlatLanes<float> { static constexpr int PXL = 1, NS = 4; };
template <> struct FlatLanes<unsigned short> { static constexpr int PXL = 2, NS = 2; };


template <typename OutT, int PXL>
__device__ __forceinline__ void store_px(OutT* row, int f0, int slab, bool pair_ok, const float* v) {
  if (PXL == 1) {
    if (f0 >= 0 && f0 < slab) store1(row + f0, v[0]);
  } else {
    if (pair_ok && f0 >= 0 && f0 + 1 < slab) {
      const unsigned int u = (unsigned int)to_bf16(v[0]) | ((unsigned int)to_bf16(v[1]) << 16);
      *reinterpret_cast<unsigned int*>(row + f0) = u;
    } else {
#pragma unroll
      for (int k = 0; k < PXL; ++k)
        if (f0 + k >= 0 && f0 + k < slab) store1(row + f0 + k, v[k]);
    }
  }
}

// Bilinear taps of an in-image sample (sample_pos returned true): then
// ix in [0, w-1] and iy in [0, h-1] exactly (monotone rounding of
// ((xn + 1) / 2) (w - 1) with |xn| <= 1), so x0, y0 are valid and x1 = w
// (y1 = h) only when ix = w - 1 exactly, where its weight ix - x0 is +0: the
// taps and weights equal make_taps' (invalid taps there weigh 0), without
// the validity tests.  Addresses of such taps are clamped.
struct TapsIn {
  unsigned off[4];
  float wt[4];
};
__device__ __forceinline__ void make_taps_inside(float ix, float iy, int h, int w, TapsIn& t) {
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy;
  const float wx1 = ix - fx, wx0 = (fx + 1.0f) - ix;
  const float wy1 = iy - fy, wy0 = (fy + 1.0f) - iy;
  t.wt[0] = wx0 * wy0;
  t.wt[1] = wx1 * wy0;
  t.wt[2] = wx0 * wy1;
  t.wt[3] = wx1 * wy1;
  const unsigned o0 = (unsigned)__mul24(y0, w) + (unsigned)x0;
  const unsigned dx = x0 < w - 1 ? 1u : 0u, dy = y0 < h - 1 ? (unsigned)w : 0u;
  t.off[0] = o0;
  t.off[1] = o0 + dx;
  t.off[2] = o0 + dy;
  t.off[3] = o0 + dy + dx;
}

// base + a 32-bit byte offset: uniform base pointers stay in SGPRs and the
// accesses use the saddr + 32-bit voffset form (no 64-bit address VALU).
template <typename T>
__device__ __forceinline__ T* at_u32(T* base, unsigned byte_off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + byte_off);
}
template <typename T>
__device__ __forceinline__ const T* at_u32(const T* base, unsigned byte_off) {
  return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + byte_off);
}

// One item's body.  INTERIOR: the window lies inside the slab (every lane
// pixel valid; unguarded stores), else edge windows with per-pixel guards.
template <typename OutT, int NQ, bool INTERIOR>
__device__ __forceinline__ void sweep_flat_item(const float* __restrict__ ref, const f32x4* __restrict__ tq,
                                                const float* __restrict__ pose,
                                                const float* __restrict__ K4, const float* __restrict__ K4inv,
                                                const FlatGeom& g, OutT* __restrict__ out, int b, int k,
                                                int start, size_t wbase) {
  constexpr int PXL = FlatLanes<OutT>::PXL, NS = FlatLanes<OutT>::NS, NPX = PXL * NS;
  constexpr int G = 4 * NQ;
  const int c0 = k * G;
  const int l0 = (int)magic_div((unsigned)max(start, 0), g.mhw);
  const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
  // lane pixels: slab index f = start + 256 wave + 64 PXL s + PXL lane + e
  int fs[NS], ps[NPX], ls[NPX];
  const int pbase = start - l0 * g.hw;         // in-plane index of the window start (< 0 only at an edge)
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    fs[s] = start + 256 * wave + 64 * PXL * s + PXL * lane;
#pragma unroll
    for (int e = 0; e < PXL; ++e) {
      int p = pbase + 256 * wave + 64 * PXL * s + PXL * lane + e, l = l0;
      if (!INTERIOR) {
        const int f = fs[s] + e;
        if (f < 0 || f >= g.slab) p = 0;
      }
      while (p >= g.hw) { p -= g.hw; ++l; }
      ps[s * PXL + e] = p;
      ls[s * PXL + e] = l;
    }
  }
  const int nc = min(G, g.C - c0);
  // reference rows of the group: loads first (in flight during the warp)
  float cp[G][NPX];
  if (g.ref_rows) {
#pragma unroll
    for (int c = 0; c < G; ++c) {
      if (c >= nc) break;
      const float* R = ref + ((size_t)b * g.C + c0 + c) * g.hw;
#pragma unroll
      for (int j = 0; j < NPX; ++j) cp[c][j] = *at_u32(R, (unsigned)ps[j] * 4u);
    }
  }
  Proj pr;
  load_proj(pose, K4, K4inv, b, pr);
  const SampleK sk = sample_consts(g.h, g.w);
  const float dA = plane_depth(g.dmax, g.dstep, l0), dB = plane_depth(g.dmax, g.dstep, l0 + 1);
  const f32x4* Tb = tq + ((size_t)b * g.C4 + k * NQ) * g.hw;
  f32x4 acc[NQ][NPX];
#pragma unroll
  for (int j = 0; j < NPX; ++j) {
    const int p = ps[j], l = ls[j];
    float d = l == l0 ? dA : dB;
    if (l > l0 + 1) d = plane_depth(g.dmax, g.dstep, l);   // feature maps under 1024 pixels
    // pixel (x, y) = (p % w, p / w): float reciprocal and one correction (p < 2^24),
    // then the ray K^-1 (x, y, 1) in the reference's order (pixel2cam)
    int y = (int)((float)p * g.inv_w);
    int x = p - y * g.w;
    if (x < 0) { --y; x += g.w; }
    if (x >= g.w) { ++y; x -= g.w; }
    const float xf = (float)x, yf = (float)y;
    float ray[3];
    ray[0] = (pr.ki[0] * xf + pr.ki[1] * yf) + pr.ki[2];
    ray[1] = (pr.ki[3] * xf + pr.ki[4] * yf) + pr.ki[5];
    ray[2] = (pr.ki[6] * xf + pr.ki[7] * yf) + pr.ki[8];
    float ix, iy;
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[n][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (sample_pos_nr(pr, ray, d, sk, ix, iy)) {
      TapsIn tp;
      make_taps_inside(ix, iy, g.h, g.w, tp);
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        if (4 * n >= nc) break;
        const f32x4* T = Tb + (size_t)n * g.hw;
        const f32x4 t0 = *at_u32(T, tp.off[0] * 16u), t1 = *at_u32(T, tp.off[1] * 16u);
        const f32x4 t2 = *at_u32(T, tp.off[2] * 16u), t3 = *at_u32(T, tp.off[3] * 16u);
        f32x4 a;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = tp.wt[0] * t0[e];
          v = __builtin_fmaf(tp.wt[1], t1[e], v);
          v = __builtin_fmaf(tp.wt[2], t2[e], v);
          a[e] = __builtin_fmaf(tp.wt[3], t3[e], v);
        }
        acc[n][j] = a;
      }
    }
  }
  // stores: row base + 32-bit byte offset of the window (slab < 2^30 elements)
  auto store_row = [&](OutT* row, const float* v) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (INTERIOR) {
        OutT* dst = at_u32(row, (unsigned)fs[s] * (unsigned)sizeof(OutT));
        if (PXL == 1) {
          store1(dst, v[s]);
        } else {
          const unsigned int u = (unsigned int)to_bf16(v[2 * s]) | ((unsigned int)to_bf16(v[2 * s + 1]) << 16);
          if (g.pair_ok) *reinterpret_cast<unsigned int*>(dst) = u;
          else { store1(dst, v[2 * s]); store1(dst + 1, v[2 * s + 1]); }
        }
      } else {
        store_px<OutT, PXL>(row, fs[s], g.slab, g.pair_ok, v + s * PXL);
      }
    }
  };
  if (g.ref_rows) {
#pragma unroll
    for (int c = 0; c < G; ++c) {
      if (c >= nc) break;
      store_row(out + ((size_t)b * g.rows + c0 + c) * (size_t)g.slab, cp[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < G; ++c) {
    if (c >= nc) break;
    float v[NPX];
#pragma unroll
    for (int j = 0; j < NPX; ++j) v[j] = acc[c >> 2][j][c & 3];
    store_row(out + wbase + (size_t)c * g.slab, v);
  }
}

template <typename OutT, int NQ>
__global__ __launch_bounds__(kSwThreads) void k_sweep_flat(const float* __restrict__ ref,
                                                           const f32x4* __restrict__ tq,
                                                           const float* __restrict__ pose,
                                                           const float* __restrict__ K4,
                                                           const float* __restrict__ K4inv, FlatGeom g,
                                                           OutT* __restrict__ out) {
  const unsigned item = blockIdx.x;            // grid = B * groups * nwin
  const unsigned r = magic_div(item, g.mwin);
  const int win = (int)(item - r * (unsigned)g.nwin);
  const int b = (int)magic_div(r, g.mgrp);
  const int k = (int)(r - (unsigned)b * (unsigned)g.groups);
  const size_t wbase = ((size_t)b * g.rows + g.ref_rows + k * 4 * NQ) * (size_t)g.slab;   // first warped row
  const int start = win * kFlatWin - (int)((wbase + (size_t)g.out_mis) & (size_t)g.amask);
  if (start >= g.slab) return;
  if (start >= 0 && start + kFlatWin <= g.slab)
    sweep_flat_item<OutT, NQ, true>(ref, tq, pose, K4, K4inv, g, out, b, k, start, wbase);
  else
    sweep_flat_item<OutT, NQ, false>(ref, tq, pose, K4, K4inv, g, out, b, k, start, wbase);
}

// ---------------------------------------------------------------------------
// Cost volume, narrow-window form (tuning key sweep_flat = 2).
//
// The same aligned slab windows as k_sweep_flat, but a window is 256 * NJ
// elements and every lane owns NJ lane-consecutive pixels (wave pixel
// 64 j + lane), for both output types:
//   * HBM write rate on MI355X falls with the bytes that the resident
//     workgroups have in flight at once (profiles/r01_probe_store_bw2.txt:
//     items of 1 / 4 / 8 / 16 rows x 4 KB: 6.7 / 6.5 / 6.3 / 5.7 TB/s; one
//     contiguous span of 4 KB vs 64 KB per block: 7.0 vs 6.0 TB/s).  An item
//     writes 2G rows; NJ = 1 keeps it at 2G x 1 KB.
//   * bf16: neighbouring lanes' pixels are packed into 4-byte pairs with one
//     DPP quad swap (lane 2k stores pixels 64 j + 2k, +1 of register j = 2s,
//     lane 2k + 1 those of register 2s + 1), so the gathers stay
//     lane-consecutive and each wave store is still one 256-byte segment.
// ---------------------------------------------------------------------------
template <typename OutT> struct TileLanes;
template <> struct TileLanes<float> { static constexpr int AM = 63; };
template <> struct TileLanes<unsigned short> { static constexpr int AM = 127; };

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
// a wave's LDS stage handed between its lanes: the compiler keeps every
// memory access on its side (the "memory" clobber; wavefront-scope fences do
// not order plain accesses) and the LDS operations before it have completed
__device__ __forceinline__ void sweep_wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ unsigned bf16_pair_swap(unsigned a, unsigned b, bool odd) {
  // a, b: this lane's bf16 of pixel registers 2s and 2s+1; returns the pair
  // (lo, hi) this lane stores: even lane (a_self, a_next), odd (b_prev, b_self)
  const unsigned send = odd ? a : b;
  const unsigned r = (unsigned)__builtin_amdgcn_update_dpp(0, (int)send, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  return odd ? (r | (b << 16)) : (a | (r << 16));
}

template <typename OutT, int NQ, int NJ, bool INTERIOR>
__device__ __forceinline__ void sweep_tile_item(const float* __restrict__ ref, const f32x4* __restrict__ tq,
                                                const float* __restrict__ pose,
                                                const float* __restrict__ K4, const float* __restrict__ K4inv,
                                                const FlatGeom& g, OutT* __restrict__ out, int b, int k,
                                                int start, size_t wbase) {
  constexpr bool BF = sizeof(OutT) == 2;
  static_assert(!BF || NJ % 2 == 0, "bf16 windows pack register pairs");
  constexpr int G = 4 * NQ, WW = 64 * NJ;
  const int c0 = k * G;
  const int l0 = (int)magic_div((unsigned)max(start, 0), g.mhw);
  const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
  const int woff = start + WW * wave;                 // slab index of the wave's first pixel
  int ps[NJ], ls[NJ];
  bool okf[NJ];
  const int pbase = start - l0 * g.hw;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int f = woff + 64 * j + lane;
    int p = pbase + WW * wave + 64 * j + lane, l = l0;
    okf[j] = true;
    if (!INTERIOR) {
      okf[j] = f >= 0 && f < g.slab;
      if (!okf[j]) p = 0;
    }
    while (p >= g.hw) { p -= g.hw; ++l; }
    ps[j] = p;
    ls[j] = l;
  }
  const int nc = min(G, g.C - c0);
  constexpr bool LATE = NJ >= 8;                      // reference rows loaded at their stores (registers)
  float cp[LATE ? 1 : G][NJ];
  auto load_ref_row = [&](int c, float* v) {
    const float* R = ref + ((size_t)b * g.C + c0 + c) * g.hw;
#pragma unroll
    for (int j = 0; j < NJ; ++j) v[j] = *at_u32(R, (unsigned)ps[j] * 4u);
  };
  if (!LATE && g.ref_rows && g.write_ref) {
#pragma unroll
    for (int c = 0; c < G; ++c) {
      if (c >= nc) break;
      load_ref_row(c, cp[LATE ? 0 : c]);
    }
  }
  Proj pr;
  load_proj(pose, K4, K4inv, b, pr);
  const SampleK sk = sample_consts(g.h, g.w);
  const float dA = plane_depth(g.dmax, g.dstep, l0), dB = plane_depth(g.dmax, g.dstep, l0 + 1);
  const f32x4* Tb = tq + ((size_t)b * g.C4 + k * NQ) * g.hw;
  f32x4 acc[NQ][NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = ps[j], l = ls[j];
    float d = l == l0 ? dA : dB;
    if (l > l0 + 1) d = plane_depth(g.dmax, g.dstep, l);
    int y = (int)((float)p * g.inv_w);
    int x = p - y * g.w;
    if (x < 0) { --y; x += g.w; }
    if (x >= g.w) { ++y; x -= g.w; }
    const float xf = (float)x, yf = (float)y;
    float ray[3];
    ray[0] = (pr.ki[0] * xf + pr.ki[1] * yf) + pr.ki[2];
    ray[1] = (pr.ki[3] * xf + pr.ki[4] * yf) + pr.ki[5];
    ray[2] = (pr.ki[6] * xf + pr.ki[7] * yf) + pr.ki[8];
    float ix, iy;
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[n][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (sample_pos_nr(pr, ray, d, sk, ix, iy)) {
      TapsIn tp;
      make_taps_inside(ix, iy, g.h, g.w, tp);
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        if (4 * n >= nc) break;
        const f32x4* T = Tb + (size_t)n * g.hw;
        const f32x4 t0 = *at_u32(T, tp.off[0] * 16u), t1 = *at_u32(T, tp.off[1] * 16u);
        const f32x4 t2 = *at_u32(T, tp.off[2] * 16u), t3 = *at_u32(T, tp.off[3] * 16u);
        f32x4 a;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = tp.wt[0] * t0[e];
          v = __builtin_fmaf(tp.wt[1], t1[e], v);
          v = __builtin_fmaf(tp.wt[2], t2[e], v);
          a[e] = __builtin_fmaf(tp.wt[3], t3[e], v);
        }
        acc[n][j] = a;
      }
    }
  }
  const bool odd = (lane & 1) != 0;
  auto store_row = [&](OutT* row, const float* v) {
    if (!BF) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int f = woff + 64 * j + lane;
        if (INTERIOR || okf[j]) store1(at_u32(row, (unsigned)f * 4u), v[j]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < NJ / 2; ++s) {
        const unsigned a = to_bf16(v[2 * s]), bb = to_bf16(v[2 * s + 1]);
        const unsigned u = bf16_pair_swap(a, bb, odd);
        // even lane 2k: pixels 128 s + 2k, +1; odd lane 2k+1: 128 s + 64 + 2k, +1
        const int f = woff + 128 * s + lane + (odd ? 63 : 0);
        if (INTERIOR && g.pair_ok) {
          *reinterpret_cast<unsigned int*>(at_u32(row, (unsigned)f * 2u)) = u;
        } else {
          const bool okl = f >= 0 && f < g.slab, okh = f + 1 >= 0 && f + 1 < g.slab;
          if (g.pair_ok && okl && okh) {
            *reinterpret_cast<unsigned int*>(row + f) = u;
          } else {
            if (okl) row[f] = (unsigned short)(u & 0xffffu);
            if (okh) row[f + 1] = (unsigned short)(u >> 16);
          }
        }
      }
    }
  };
  if (g.ref_rows && g.write_ref) {
#pragma unroll
    for (int c = 0; c < G; ++c) {
      if (c >= nc) break;
      if (LATE) load_ref_row(c, cp[0]);
      store_row(out + ((size_t)b * g.rows + c0 + c) * (size_t)g.slab, cp[LATE ? 0 : c]);
    }
  }
#pragma unroll
  for (int c = 0; c < G; ++c) {
    if (c >= nc) break;
    float v[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) v[j] = acc[c >> 2][j][c & 3];
    store_row(out + wbase + (size_t)c * g.slab, v);
  }
}

// Interior windows of a full channel group (the bulk of the volume), with
// buffer addressing: one SGPR resource per pair and tensor, the per-lane
// pixel byte offset in one VGPR shared by every row, each row's offset in an
// SGPR (soffset).  The generic body above spends ~200 VALU per wave item on
// 64-bit address arithmetic, partial-group branches and their zero moves
// (SQ_INSTS_VALU 324 per item at KITTI, ~110 of them the sampling itself);
// here stores and loads need no VALU address work.  Same arithmetic, so the
// same bits.  Requires every per-pair byte range below 2^32 (g.buf_ok).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

// Lane i + 1's value in lane i (DPP wave_shl:1; lane 63 reads 0).
__device__ __forceinline__ unsigned next_lane_u(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, true);
}
__device__ __forceinline__ float next_lane_f(float v) { return __uint_as_float(next_lane_u(__float_as_uint(v))); }

template <typename OutT, int NQ, int NJ, bool SHARE, bool NT, bool WIDE = false, int WPOL = -1>
__device__ __forceinline__ void sweep_tile_fast(const float* __restrict__ ref, const f32x4* __restrict__ tq,
                                                const Proj* __restrict__ projs, const FlatGeom& g,
                                                OutT* __restrict__ out, int b, int k, int start) {
  constexpr bool BF = sizeof(OutT) == 2;
  constexpr int G = 4 * NQ, WW = 64 * NJ;
  const int c0 = k * G;
  const int l0 = (int)magic_div((unsigned)start, g.mhw);
  const int lane = (int)(threadIdx.x & 63), wave = (int)(threadIdx.x >> 6);
  const int woff = start + WW * wave;
  const int pbase = start - l0 * g.hw;
  int ps[NJ], ls[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    int p = pbase + WW * wave + 64 * j + lane, l = l0;
    if (g.hw >= 256 * NJ) {                    // a window spans at most two planes
      if (p >= g.hw) { p -= g.hw; ++l; }
    } else {
      while (p >= g.hw) { p -= g.hw; ++l; }
    }
    ps[j] = p;
    ls[j] = l;
  }
  const __amdgpu_buffer_rsrc_t rout = buf_rsrc(out + (size_t)b * g.rows * g.slab, g.pair_bytes);
  const unsigned row_bytes = (unsigned)g.slab * (unsigned)sizeof(OutT);
  // the reference rows: loaded up front (their latency under the sampling),
  // or, with wide stores (more pixels per lane), row by row at their stores
  const __amdgpu_buffer_rsrc_t rref = buf_rsrc(ref + ((size_t)b * g.C + c0) * g.hw, (unsigned)G * g.hw * 4u);
  auto load_ref_row = [&](int c, float* v) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      v[j] = __uint_as_float(
          __builtin_amdgcn_raw_buffer_load_b32(rref, (unsigned)ps[j] * 4u, (unsigned)c * g.hw * 4u, 0));
  };
  constexpr bool LATE = WIDE && NJ == 8;        // registers: the reference rows at their stores
  float cp[LATE ? 1 : G][NJ];
  if (!LATE && g.ref_rows && g.write_ref) {
#pragma unroll
    for (int c = 0; c < G; ++c) load_ref_row(c, cp[LATE ? 0 : c]);
  }
  const Proj pr = projs[b];                    // uniform: scalar loads
  const SampleK sk = sample_consts(g.h, g.w);
  float dA, dB;
  if (g.depths) {
    dA = g.depths[l0];
    dB = l0 + 1 < g.L ? g.depths[l0 + 1] : dA;
  } else {
    dA = plane_depth(g.dmax, g.dstep, l0);
    dB = plane_depth(g.dmax, g.dstep, l0 + 1);
  }
  const __amdgpu_buffer_rsrc_t rtq =
      buf_rsrc(tq + ((size_t)b * g.C4 + k * NQ) * g.hw, (unsigned)NQ * g.hw * 16u);
  f32x4 acc[NQ][NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int p = ps[j], l = ls[j];
    float d = l == l0 ? dA : dB;
    if (l > l0 + 1) d = plane_depth(g.dmax, g.dstep, l);
    int y = (int)((float)p * g.inv_w);
    int x = p - y * g.w;
    if (x < 0) { --y; x += g.w; }
    if (x >= g.w) { ++y; x -= g.w; }
    const float xf = (float)x, yf = (float)y;
    float ray[3];
    ray[0] = (pr.ki[0] * xf + pr.ki[1] * yf) + pr.ki[2];
    ray[1] = (pr.ki[3] * xf + pr.ki[4] * yf) + pr.ki[5];
    ray[2] = (pr.ki[6] * xf + pr.ki[7] * yf) + pr.ki[8];
    float ix, iy;
#pragma unroll
    for (int n = 0; n < NQ; ++n) acc[n][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    if (SHARE) {
      // Lanes hold consecutive pixels, and a fronto-parallel plane maps
      // neighbouring pixels ~one source pixel apart: lane i's right-hand taps
      // (off[1], off[3]) are usually lane i + 1's left-hand taps (off[0],
      // off[2]).  Each lane gathers its left-hand taps, takes the right-hand
      // ones from the next lane where the offsets are equal (then the values
      // are the same memory words), and gathers them itself elsewhere: half
      // the tap gathers through the texture path, the same bits.
      const bool in = sample_pos_nr(pr, ray, d, sk, ix, iy);
      TapsIn tp;
      if (in) {
        make_taps_inside(ix, iy, g.h, g.w, tp);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) { tp.off[e] = 0u; tp.wt[e] = 0.0f; }
      }
      const unsigned n0 = next_lane_u(tp.off[0]), n2 = next_lane_u(tp.off[2]);
      const unsigned nin = next_lane_u(in ? 1u : 0u);
      const bool own = in && !(nin != 0u && n0 == tp.off[1] && n2 == tp.off[3]);
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        const unsigned so = (unsigned)n * g.hw * 16u;
        f32x4 t[4];
        t[0] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        t[2] = t[0];
        if (in) {
          t[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtq, tp.off[0] * 16u, so, 0));
          t[2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtq, tp.off[2] * 16u, so, 0));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          t[1][e] = next_lane_f(t[0][e]);
          t[3][e] = next_lane_f(t[2][e]);
        }
        if (own) {
          t[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtq, tp.off[1] * 16u, so, 0));
          t[3] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtq, tp.off[3] * 16u, so, 0));
        }
        f32x4 a;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = tp.wt[0] * t[0][e];
          v = __builtin_fmaf(tp.wt[1], t[1][e], v);
          v = __builtin_fmaf(tp.wt[2], t[2][e], v);
          a[e] = __builtin_fmaf(tp.wt[3], t[3][e], v);
        }
        if (in) acc[n][j] = a;
      }
    } else if (sample_pos_nr(pr, ray, d, sk, ix, iy)) {
      TapsIn tp;
      make_taps_inside(ix, iy, g.h, g.w, tp);
#pragma unroll
      for (int n = 0; n < NQ; ++n) {
        const unsigned so = (unsigned)n * g.hw * 16u;
        f32x4 t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          t[e] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtq, tp.off[e] * 16u, so, 0));
        f32x4 a;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = tp.wt[0] * t[0][e];
          v = __builtin_fmaf(tp.wt[1], t[1][e], v);
          v = __builtin_fmaf(tp.wt[2], t[2][e], v);
          a[e] = __builtin_fmaf(tp.wt[3], t[3][e], v);
        }
        acc[n][j] = a;
      }
    }
  }
  const bool odd = (lane & 1) != 0;
  // volume stores: with NT the cache policy is sc0 nt (non-temporal, the
  // volume is never re-read by this kernel), so the 7.7 GB of streaming
  // writes do not evict the reference rows and target quads that every plane
  // re-reads from L2 (tuning key sweep_store_nt, profiles/r02_sweep_nt_ab.txt:
  // bf16 0.474 -> 0.442 ms; fp32 1.255 -> 1.265, so by default bf16 only)
  auto bstore = [&](unsigned v, __amdgpu_buffer_rsrc_t r, unsigned off, unsigned so) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off, so, NT ? 3 : 0);
  };
  // row r of the pair: soffset r * row_bytes; per-lane byte offset(s) of the window
  auto store_row = [&](unsigned r, const float* v) {
    const unsigned so = r * row_bytes;
    if (!BF) {                                  // (wide stores: put / flush below)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bstore(__float_as_uint(v[j]), rout, (unsigned)(woff + 64 * j + lane) * 4u, so);
    } else {
#pragma unroll
      for (int s = 0; s < NJ / 2; ++s) {
        const unsigned u = bf16_pair_swap(to_bf16(v[2 * s]), to_bf16(v[2 * s + 1]), odd);
        const int f = woff + 128 * s + lane + (odd ? 63 : 0);
        bstore(u, rout, (unsigned)f * 2u, so);
      }
    }
  };
  if constexpr (WIDE) {
    // 16-byte lane stores (sweep_store_px): a 16-byte store holds EPL pixels
    // (8 bf16 / 4 fp32) and the wave's window of a row, 64 NJ pixels, takes
    // LPR = 64 NJ / EPL lanes, so one store instruction covers RPS = 64 / LPR
    // consecutive rows.  The pixels go through a per-wave LDS stage of RPS
    // rows (1 KB) at their window positions and come back as EPL consecutive
    // pixels per lane; the tap gathers stay lane-consecutive.
    constexpr int EPL = 16 / (int)sizeof(OutT), LPR = 64 * NJ / EPL, RPS = 64 / LPR;
    // the 16-byte stores' cache policy: sc0 nt / plain by NT, or WPOL (sc1:
    // write-through, the line is not kept in the XCD's L2 -- tuning key
    // sweep_store_wt)
    constexpr int POL = WPOL >= 0 ? WPOL : (NT ? 3 : 0);
    static_assert(NJ <= EPL && EPL % NJ == 0, "wide stores: NJ divides the pixels of a 16-byte store");
    __shared__ __attribute__((aligned(16))) uint32_t s_rows[kSwThreads / 64][RPS][16 * LPR / 4];
    const int rr = lane / LPR, cl = lane - rr * LPR;
    const unsigned voff = (unsigned)(woff + EPL * cl) * (unsigned)sizeof(OutT) + (unsigned)rr * row_bytes;
    // (per-pixel LDS writes; the DPP-packed pairs staged as 4-byte writes are
    // equally correct since the store-hazard fix below, profiles/r05_store_hazard.txt)
    auto put = [&](int slot, const float* v) {
      OutT* st = reinterpret_cast<OutT*>(s_rows[wave][slot]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if constexpr (BF) st[64 * j + lane] = (unsigned short)to_bf16(v[j]);
        else st[64 * j + lane] = v[j];
      }
    };
    auto flush = [&](unsigned r0) {             // rows r0 .. r0 + RPS - 1
      sweep_wave_sync();
      const u32x4 x = *reinterpret_cast<const u32x4*>(&s_rows[wave][rr][4 * cl]);
      // the row offset in voffset with a literal-0 soffset, not an SGPR
      // soffset: a 128-bit store's data VGPRs must not be overwritten by the
      // next instruction (gfx950 stores the new value for lanes 16r+12..15
      // otherwise, scripts/probe_store_hazard.hip), and LLVM's hazard
      // recognizer inserts that wait state only for stores without an SGPR
      // soffset -- the round-4 "4-byte staging miscompute" was this pair
      // (profiles/r05_store_hazard.txt)
      __builtin_amdgcn_raw_buffer_store_b128(x, rout, voff + r0 * row_bytes, 0, POL);
      sweep_wave_sync();                        // the stage's reads before the next rows' writes
    };
    static_assert(G % RPS == 0, "row groups");
#pragma unroll
    for (int c = 0; c < G; c += RPS) {
#pragma unroll
      for (int t = 0; t < RPS; ++t) {
        float v[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) v[j] = acc[(c + t) >> 2][j][(c + t) & 3];
        put(t, v);
      }
      flush((unsigned)(g.ref_rows + c0 + c));
    }
    if (g.ref_rows && g.write_ref) {
#pragma unroll
      for (int c = 0; c < G; c += RPS) {
#pragma unroll
        for (int t = 0; t < RPS; ++t) {
          if (LATE) {
            float v[NJ];
            load_ref_row(c + t, v);
            put(t, v);
          } else {
            put(t, cp[LATE ? 0 : c + t]);
          }
        }
        flush((unsigned)(c0 + c));
      }
    }
  } else {
    if (g.ref_rows && g.write_ref) {
#pragma unroll
      for (int c = 0; c < G; ++c) store_row((unsigned)(c0 + c), cp[LATE ? 0 : c]);
    }
#pragma unroll
    for (int c = 0; c < G; ++c) {
      float v[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) v[j] = acc[c >> 2][j][c & 3];
      store_row((unsigned)(g.ref_rows + c0 + c), v);
    }
  }
}

// bf16 volumes at NJ = 2 (the default; round 6): 8 waves per SIMD instead of the 6 the allocator
// picks (76 -> 64 VGPRs, a 48-byte spill outside the fast path): the tap
// gathers' latency is what the extra waves hide -- the C3 sweep 0.363-0.368
// -> 0.351-0.355 ms in three alternating rounds on one box
// (profiles/r06_sweep_occupancy_ab.txt); fp32 kernels already run at 8.
template <typename OutT, int NQ, int NJ>
__global__ __launch_bounds__(kSwThreads) __attribute__((amdgpu_waves_per_eu(sizeof(OutT) == 2 && NJ == 2 ? 8 : 1)))
void k_sweep_tile(const float* __restrict__ ref,
                                                           const f32x4* __restrict__ tq,
                                                           const float* __restrict__ pose,
                                                           const float* __restrict__ K4,
                                                           const float* __restrict__ K4inv, FlatGeom g,
                                                           OutT* __restrict__ out, const Proj* __restrict__ projs) {
  constexpr int WIN = 256 * NJ;
  const unsigned item = blockIdx.x;            // grid = B * groups * nwin
  const unsigned r = magic_div(item, g.mwin);
  const int win = (int)(item - r * (unsigned)g.nwin);
  const int b = (int)magic_div(r, g.mgrp);
  const int k = (int)(r - (unsigned)b * (unsigned)g.groups);
  const size_t wbase = ((size_t)b * g.rows + g.ref_rows + k * 4 * NQ) * (size_t)g.slab;
  const int start = win * WIN - (int)((wbase + (size_t)g.out_mis) & (size_t)g.amask);
  if (start >= g.slab) return;
  if (g.buf_ok && start >= 0 && start + WIN <= g.slab && (k + 1) * 4 * NQ <= g.C)
  {
    if constexpr (NJ <= 16 / (int)sizeof(OutT)) {
      if (NJ == 8 || (g.store_px == NJ && !g.share)) {     // NJ = 8 is launched for wide stores only
        if (g.wpol == 16) sweep_tile_fast<OutT, NQ, NJ, false, false, true, 16>(ref, tq, projs, g, out, b, k, start);
        else if (g.wpol == 17) sweep_tile_fast<OutT, NQ, NJ, false, false, true, 17>(ref, tq, projs, g, out, b, k, start);
        else if (g.wpol == 18) sweep_tile_fast<OutT, NQ, NJ, false, false, true, 18>(ref, tq, projs, g, out, b, k, start);
        else if (g.store_nt) sweep_tile_fast<OutT, NQ, NJ, false, true, true>(ref, tq, projs, g, out, b, k, start);
        else sweep_tile_fast<OutT, NQ, NJ, false, false, true>(ref, tq, projs, g, out, b, k, start);
        return;
      }
    }
    if constexpr (NJ == 8) return;
    else if (g.store_nt) {
      if (g.share) sweep_tile_fast<OutT, NQ, NJ, true, true>(ref, tq, projs, g, out, b, k, start);
      else sweep_tile_fast<OutT, NQ, NJ, false, true>(ref, tq, projs, g, out, b, k, start);
    } else {
      if (g.share) sweep_tile_fast<OutT, NQ, NJ, true, false>(ref, tq, projs, g, out, b, k, start);
      else sweep_tile_fast<OutT, NQ, NJ, false, false>(ref, tq, projs, g, out, b, k, start);
    }
  }
  else if (start >= 0 && start + WIN <= g.slab)
    sweep_tile_item<OutT, NQ, NJ, true>(ref, tq, pose, K4, K4inv, g, out, b, k, start, wbase);
  else
    sweep_tile_item<OutT, NQ, NJ, false>(ref, tq, pose, K4, K4inv, g, out, b, k, start, wbase);
}

template <typename OutT, int NQ>
static void launch_k_sweep_tile_nj(int nj, unsigned blocks, hipStream_t s, const float* ref, const f32x4* tq,
                                   const float* pose, const float* K4, const float* K4inv, const FlatGeom& g,
                                   void* out, const Proj* projs) {
  const dim3 grid(blocks), block(kSwThreads);
  constexpr bool BF = sizeof(OutT) == 2;
  if (nj >= 8 && BF)
    hipLaunchKernelGGL((k_sweep_tile<OutT, NQ, (BF ? 8 : 4)>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g,
                       (OutT*)out, projs);
  else if (nj >= 4)
    hipLaunchKernelGGL((k_sweep_tile<OutT, NQ, 4>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g, (OutT*)out, projs);
  else if (nj == 2 || BF)
    hipLaunchKernelGGL((k_sweep_tile<OutT, NQ, 2>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g, (OutT*)out, projs);
  else
    hipLaunchKernelGGL((k_sweep_tile<OutT, NQ, (BF ? 2 : 1)>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g,
                       (OutT*)out, projs);
}

template <typename OutT>
static void launch_k_sweep_flat(int nq, unsigned blocks, hipStream_t s, const float* ref, const f32x4* tq,
                                const float* pose, const float* K4, const float* K4inv, const FlatGeom& g,
                                void* out) {
  if (nq == 2)
    hipLaunchKernelGGL((k_sweep_flat<OutT, 2>), dim3(blocks), dim3(kSwThreads), 0, s, ref, tq, pose, K4, K4inv, g,
                       (OutT*)out);
  else
    hipLaunchKernelGGL((k_sweep_flat<OutT, 1>), dim3(blocks), dim3(kSwThreads), 0, s, ref, tq, pose, K4, K4inv, g,
                       (OutT*)out);
}

// ---------------------------------------------------------------------------
// Cost volume, plane-run form with the target band in LDS (sweep_flat = 3).
//
// k_sweep_tile is bound by the texture address/data units, not by HBM: per
// pixel and channel quad a lane issues four 16-byte tap gathers (64 B through
// the L1 path for 16 B of output), and re-reads the same target pixels at
// every plane (PMC: 1.8 GB of reads per launch against 0.06 GB algorithmic).
// Here one block produces a run of R consecutive planes of one 256*NJ-pixel
// tile for one channel quad:
//   * the source rows every tap of the run touches are found first (the same
//     sample positions, computed twice), and that band of full target rows --
//     contiguous in tq -- is copied once into LDS; the taps are then ds_read
//     from it (lanes whose taps fall outside a band clipped to the LDS budget
//     gather from global memory, same values);
//   * the tile's reference pixels (the same at every plane) are staged once
//     and stored R times;
//   * the windows stay 256-byte aligned per plane: at plane l the tile covers
//     pixels [WIN n - ph_l, WIN n - ph_l + WIN), ph_l the row's misalignment
//     at that plane, so every full wave store is one aligned segment.
// On KITTI (94x311 features, |t| 0.6) the band of a 16-plane run is 6 rows at
// the median, 14 at p99: ~15 B of staged reads per 4 channels of a pixel
// and plane instead of 64 B of gathers.  Same arithmetic as k_sweep_tile
// (bit-identical volumes).
// ---------------------------------------------------------------------------
struct BandGeom {
  int C, C4, h, w, hw, L;
  int ref_rows, rows;
  int slab;        // L * hw elements
  int ntiles;      // tiles per plane: ceil((hw + A - 1) / WIN)
  int nruns;       // plane runs per quad: ceil(L / run)
  int run;         // planes per block
  int amask;       // A - 1, A = elements per 256 bytes
  int out_mis;     // element offset of the output pointer modulo A
  int hwmod;       // hw mod A
  int pair_ok;     // bf16: every row starts at an even element
  int cap_rows;    // band rows the LDS holds
  Magic mtile, mrun, mgrp;
  float inv_w, dmax, dstep;
};

template <int NJ>
__device__ __forceinline__ int band_pixel(int ws, int wave, int lane, int j) {
  return ws + 64 * NJ * wave + 64 * j + lane;
}

constexpr int kBandThreads = 1024;   // 16 waves: 4 wave groups x 4 waves over the tile

template <typename OutT, int NJ>
__global__ __launch_bounds__(kBandThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_sweep_band(const float* __restrict__ ref,
                                                             const f32x4* __restrict__ tq,
                                                             const float* __restrict__ pose,
                                                             const float* __restrict__ K4,
                                                             const float* __restrict__ K4inv, BandGeom g,
                                                             OutT* __restrict__ out) {
  constexpr bool BF = sizeof(OutT) == 2;
  static_assert(!BF || NJ % 2 == 0, "bf16 windows pack register pairs");
  constexpr int WIN = 256 * NJ;
  extern __shared__ f32x4 s_band[];            // cap_rows * w quads, then the reference tile
  __shared__ int s_ylo, s_yhi;
  const unsigned item = blockIdx.x;            // ((b * C4 + k) * nruns + run) * ntiles + n
  const unsigned r1 = magic_div(item, g.mtile);
  const int n = (int)(item - r1 * (unsigned)g.ntiles);
  const unsigned r2 = magic_div(r1, g.mrun);
  const int run = (int)(r1 - r2 * (unsigned)g.nruns);
  const int b = (int)magic_div(r2, g.mgrp);
  const int k = (int)(r2 - (unsigned)b * (unsigned)g.C4);
  const int tid = (int)threadIdx.x;
  const int lane = tid & 63, wave = (tid >> 6) & 3, grp = tid >> 8;   // wave group grp takes planes l0 + grp + 4 i
  const int A = g.amask + 1;
  const int l0 = run * g.run, l1 = min(g.L, l0 + g.run);
  const int nc = min(4, g.C - 4 * k);
  const size_t wrow = ((size_t)b * g.rows + g.ref_rows + 4 * k) * (size_t)g.slab;   // first warped row
  const int wmis = (int)((wrow + (size_t)g.out_mis) & (size_t)g.amask);
  auto phase = [&](int l) { return (wmis + (int)(((unsigned)l * (unsigned)g.hwmod) & (unsigned)g.amask)) & g.amask; };
  const int rbase = WIN * n - A;               // reference tile: pixels [rbase, rbase + WIN + A)
  const int RW = WIN + A;                      // <= 640 < kBandThreads
  float* s_ref = reinterpret_cast<float*>(s_band + g.cap_rows * g.w);

  if (tid == 0) { s_ylo = 0x7fffffff; s_yhi = -1; }
  // reference tile loads first: in flight during the band estimate
  float rv[4];
  if (g.ref_rows) {
    const int p = rbase + tid;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float* R = ref + ((size_t)b * g.C + 4 * k + min(c, nc - 1)) * g.hw;
      rv[c] = (tid < RW && p >= 0 && p < g.hw) ? R[p] : 0.0f;
    }
  }
  Proj pr;
  load_proj(pose, K4, K4inv, b, pr);
  const SampleK sk = sample_consts(g.h, g.w);
  auto pixel_ray = [&](int p, float (&ray)[3]) {
    int y = (int)((float)p * g.inv_w);
    int x = p - y * g.w;
    if (x < 0) { --y; x += g.w; }
    if (x >= g.w) { ++y; x -= g.w; }
    const float xf = (float)x, yf = (float)y;
    ray[0] = (pr.ki[0] * xf + pr.ki[1] * yf) + pr.ki[2];
    ray[1] = (pr.ki[3] * xf + pr.ki[4] * yf) + pr.ki[5];
    ray[2] = (pr.ki[6] * xf + pr.ki[7] * yf) + pr.ki[8];
  };

  // Band estimate: the tap rows of the tile at four planes of the run (its
  // first and last, and two between; one per wave group).  A pixel's sample
  // moves monotonically along its epipolar line with the plane, so the run's
  // taps lie between the end planes' almost everywhere; the exceptions (and
  // bands clipped to cap_rows) take the global path below, so the estimate
  // changes only speed, never values.
  int ylo = 0x7fffffff, yhi = -1;
  {
    const int l = l0 + (grp * (l1 - 1 - l0) + 1) / 3;
    const float d = plane_depth(g.dmax, g.dstep, l);
    const int ws = WIN * n - phase(l);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int p = band_pixel<NJ>(ws, wave, lane, j);
      if (p >= 0 && p < g.hw) {
        float ray[3], ix, iy;
        pixel_ray(p, ray);
        if (sample_pos_nr(pr, ray, d, sk, ix, iy)) {
          const int y0 = (int)floorf(iy);
          ylo = min(ylo, y0);
          yhi = max(yhi, y0 + (y0 < g.h - 1 ? 1 : 0));
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    ylo = min(ylo, __shfl_xor(ylo, o));
    yhi = max(yhi, __shfl_xor(yhi, o));
  }
  __syncthreads();   // s_ylo / s_yhi initialised
  if (lane == 0) { atomicMin(&s_ylo, ylo); atomicMax(&s_yhi, yhi); }
  if (g.ref_rows && tid < RW) {
#pragma unroll
    for (int c = 0; c < 4; ++c) s_ref[c * RW + tid] = rv[c];
  }
  __syncthreads();
  int by0 = s_ylo, nb = 0;
  if (s_yhi >= by0) {
    // a little slack around the estimate, inside the image and the LDS
    const int want_lo = max(by0 - 1, 0), want_hi = min(s_yhi + 1, g.h - 1);
    nb = min(want_hi - want_lo + 1, g.cap_rows);
    by0 = want_lo;
  } else {
    by0 = 0;
  }
  const f32x4* T = tq + ((size_t)b * g.C4 + k) * g.hw;   // this quad's target plane
  {
    const f32x4* src = T + (size_t)by0 * g.w;
    const int cnt = nb * g.w;
    int i = tid;
    for (; i + kBandThreads < cnt; i += 2 * kBandThreads) {
      const f32x4 a0 = src[i], a1 = src[i + kBandThreads];
      s_band[i] = a0; s_band[i + kBandThreads] = a1;
    }
    if (i < cnt) s_band[i] = src[i];
  }
  __syncthreads();
  const unsigned lo = (unsigned)(by0 * g.w), span = (unsigned)(nb * g.w);
  const bool odd = (lane & 1) != 0;

  for (int l = l0 + grp; l < l1; l += 4) {
    const float d = plane_depth(g.dmax, g.dstep, l);
    const int ws = WIN * n - phase(l);
    const int fl = l * g.hw;                   // slab index of the plane's pixel 0
    float acc[4][NJ], cp[4][NJ];
    bool ok[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int p = band_pixel<NJ>(ws, wave, lane, j);
      ok[j] = p >= 0 && p < g.hw;
      const int pp = ok[j] ? p : max(rbase, 0);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        acc[c][j] = 0.0f;
        cp[c][j] = g.ref_rows ? s_ref[c * RW + (pp - rbase)] : 0.0f;
      }
      float ray[3], ix, iy;
      pixel_ray(pp, ray);
      if (ok[j] && sample_pos_nr(pr, ray, d, sk, ix, iy)) {
        TapsIn tp;
        make_taps_inside(ix, iy, g.h, g.w, tp);
        f32x4 t0, t1, t2, t3;
        if (tp.off[0] - lo < span && tp.off[3] - lo < span) {
          t0 = s_band[tp.off[0] - lo]; t1 = s_band[tp.off[1] - lo];
          t2 = s_band[tp.off[2] - lo]; t3 = s_band[tp.off[3] - lo];
        } else {
          t0 = *at_u32(T, tp.off[0] * 16u); t1 = *at_u32(T, tp.off[1] * 16u);
          t2 = *at_u32(T, tp.off[2] * 16u); t3 = *at_u32(T, tp.off[3] * 16u);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = tp.wt[0] * t0[e];
          v = __builtin_fmaf(tp.wt[1], t1[e], v);
          v = __builtin_fmaf(tp.wt[2], t2[e], v);
          acc[e][j] = __builtin_fmaf(tp.wt[3], t3[e], v);
        }
      }
    }
    auto store_row = [&](OutT* row, const float* v) {
      if (!BF) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const int p = band_pixel<NJ>(ws, wave, lane, j);
          if (ok[j]) store1(at_u32(row, (unsigned)(fl + p) * 4u), v[j]);
        }
      } else {
#pragma unroll
        for (int s = 0; s < NJ / 2; ++s) {
          const unsigned a = to_bf16(v[2 * s]), bb = to_bf16(v[2 * s + 1]);
          const unsigned u = bf16_pair_swap(a, bb, odd);
          // even lane 2m: pixels 128 s + 2m, +1; odd lane 2m+1: 128 s + 64 + 2m, +1
          const int p = ws + 64 * NJ * wave + 128 * s + lane + (odd ? 63 : 0);
          const bool okl = p >= 0 && p < g.hw, okh = p + 1 >= 0 && p + 1 < g.hw;
          if (g.pair_ok && okl && okh) {
            *reinterpret_cast<unsigned int*>(at_u32(row, (unsigned)(fl + p) * 2u)) = u;
          } else {
            if (okl) row[fl + p] = (unsigned short)(u & 0xffffu);
            if (okh) row[fl + p + 1] = (unsigned short)(u >> 16);
          }
        }
      }
    };
    if (g.ref_rows) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        if (c >= nc) break;
        store_row(out + ((size_t)b * g.rows + 4 * k + c) * (size_t)g.slab, cp[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= nc) break;
      store_row(out + wrow + (size_t)c * g.slab, acc[c]);
    }
  }
}

// LDS bytes of one k_sweep_band block holding `rows` band rows
static size_t band_lds_bytes(int rows, int w, int nj) {
  return (size_t)rows * w * sizeof(f32x4) + 4 * (size_t)(256 * nj + 128) * sizeof(float);   // band + ref tile
}

// inverse_warp for an arbitrary depth map (models/inverse_warp.py:121-153)
__global__ __launch_bounds__(kSweepThreads) void k_inverse_warp(const float* __restrict__ feat, int C, int h, int w,
                                                                const float* __restrict__ depth,
                                                                const float* __restrict__ pose,
                                                                const float* __restrict__ K,
                                                                const float* __restrict__ Kinv,
                                                                float* __restrict__ out) {
  const int b = blockIdx.y;
  const int hw = h * w;
  const int p = blockIdx.x * kSweepThreads + threadIdx.x;
  if (p >= hw) return;
  Proj pr;
  load_proj(pose, K, Kinv, b, pr);
  const float x = (float)(p % w), y = (float)(p / w);
  float ray[3];
  ray[0] = (pr.ki[0] * x + pr.ki[1] * y) + pr.ki[2];
  ray[1] = (pr.ki[3] * x + pr.ki[4] * y) + pr.ki[5];
  ray[2] = (pr.ki[6] * x + pr.ki[7] * y) + pr.ki[8];
  float ix, iy;
  const bool ok = sample_pos(pr, ray, depth[(size_t)b * hw + p], h, w, ix, iy);
  Taps tp;
  if (ok) make_taps(ix, iy, h, w, tp);
  const float* F = feat + (size_t)b * C * hw;
  float* O = out + (size_t)b * C * hw + p;
  for (int c = 0; c < C; ++c) {
    const float* Fc = F + (size_t)c * hw;
    float acc = 0.0f;
    if (ok) {
      acc = tp.wt[0] * Fc[tp.off[0]];
      acc = acc + tp.wt[1] * Fc[tp.off[1]];
      acc = acc + tp.wt[2] * Fc[tp.off[2]];
      acc = acc + tp.wt[3] * Fc[tp.off[3]];
    }
    O[(size_t)c * hw] = acc;
  }
}

template <typename OutT, bool VEC, bool LP, bool NT>
static void launch_k_sweep_lp(int ipb, int64_t blocks, hipStream_t s, const float* ref, const f32x4* tq, const float* pose,
                           const float* K4, const float* K4inv, const SweepGeom& g, void* out) {
  const dim3 grid((unsigned)blocks), block(kSwThreads);
  switch (ipb) {
    case 1: hipLaunchKernelGGL((k_sweep<OutT, VEC, 1, LP, NT>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g, (OutT*)out); break;
    case 2: hipLaunchKernelGGL((k_sweep<OutT, VEC, 2, LP, NT>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g, (OutT*)out); break;
    case 4: hipLaunchKernelGGL((k_sweep<OutT, VEC, 4, LP, NT>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g, (OutT*)out); break;
    default: hipLaunchKernelGGL((k_sweep<OutT, VEC, 8, LP, NT>), grid, block, 0, s, ref, tq, pose, K4, K4inv, g, (OutT*)out);
  }
}

template <typename OutT, bool VEC>
static void launch_k_sweep(int ipb, int64_t blocks, hipStream_t s, const float* ref, const f32x4* tq, const float* pose,
                           const float* K4, const float* K4inv, const SweepGeom& g, void* out) {
  // sweep_lane_pixels: 0 lane-consecutive pixels (default), 1 four pixels per
  // lane (16-byte stores), 2 lane-consecutive with non-temporal stores
  const int m = tuning().sweep_lane_pixels;
  if (m == 1) launch_k_sweep_lp<OutT, VEC, true, false>(ipb, blocks, s, ref, tq, pose, K4, K4inv, g, out);
  else if (m == 2) launch_k_sweep_lp<OutT, VEC, false, true>(ipb, blocks, s, ref, tq, pose, K4, K4inv, g, out);
  else launch_k_sweep_lp<OutT, VEC, false, false>(ipb, blocks, s, ref, tq, pose, K4, K4inv, g, out);
}

// workspace: channel quads tq [B][C4][hw] float4
static size_t sweep_quads_bytes(int B, int C, int h, int w) {
  const int C4 = (C + 3) / 4;
  return (size_t)B * C4 * (size_t)h * w * sizeof(f32x4);
}
// workspace: channel quads, then the per-pair Proj table
constexpr int kDepthTable = 1024;   // plane depths kept in the workspace for L <= this
static size_t sweep_proj_bytes(int B) { return ((size_t)B * sizeof(Proj) + 255) & ~(size_t)255; }
// sfm_plane_sweep_psnet: float32 pose, K4, K4inv per pair (12 + 9 + 9 floats)
static size_t sweep_psnet_bytes(int B) { return ((size_t)B * 30 * sizeof(float) + 255) & ~(size_t)255; }
// what launch_sweep uses: quads, Proj table, plane depths
static size_t sweep_core_bytes(int B, int C, int h, int w) {
  return sweep_quads_bytes(B, C, h, w) + sweep_proj_bytes(B) + kDepthTable * sizeof(float);
}
// the public size: the core plus the sfm_plane_sweep_psnet operands at its end
static size_t sweep_ws_bytes(int B, int C, int h, int w) { return sweep_core_bytes(B, C, h, w) + sweep_psnet_bytes(B); }

static int launch_sweep(bool with_ref, const float* ref, const float* tgt, int B, int C, int h, int w,
                        const float* pose, const float* K4, const float* K4inv, int L, float min_depth,
                        int depth_mode, int out_dtype, void* out, void* ws, size_t ws_bytes, hipStream_t s,
                        const PsnetPrep& prep = PsnetPrep{}, bool write_ref = true) {
  SFM_REQUIRE(tgt && pose && K4 && K4inv && out && (!with_ref || ref), "null pointer argument");
  SFM_REQUIRE(B >= 1 && B <= 65535 && C >= 1 && C <= 4 * 65535 && h >= 2 && w >= 2 && L >= 1,
              "invalid sweep shape");   // k_tgt_quads' grid: quads in y, pairs in z
  SFM_REQUIRE(out_dtype == 0 || out_dtype == 1, "out_dtype must be 0 (float32) or 1 (bfloat16)");
  SFM_REQUIRE(depth_mode == 0 || depth_mode == 1, "depth_mode must be 0 (inverse depth) or 1 (depth)");
  SFM_REQUIRE(min_depth > 0.0f, "min_depth must be positive");
  SFM_REQUIRE((int64_t)h * w < ((int64_t)1 << 30), "feature map too large");
  const size_t need = sweep_core_bytes(B, C, h, w);
  if (!ws || ws_bytes < need) {
    set_error("plane sweep workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  const int hw = h * w;
  SweepGeom g;
  g.B = B; g.C = C; g.C4 = (C + 3) / 4; g.h = h; g.w = w; g.L = L;
  g.ref_rows = with_ref ? C : 0;
  g.rows = g.ref_rows + C;
  g.groups = g.ref_rows + g.C4;
  g.npw = (hw + 3 + kSwWin - 1) / kSwWin;
  // 16-byte row alignment (see k_sweep): every row aligned if hw % 4 == 0; rows of
  // plane l shifted by 2*(l&1) if hw % 4 == 2 and L even; element stores otherwise
  g.shift_mode = (hw % 4 == 2 && L % 2 == 0) ? 1 : 0;
  const bool vec = (hw % 4 == 0) || g.shift_mode;
  const int ipb = tuning().sweep_items_per_block >= 8 ? 8 : tuning().sweep_items_per_block >= 4 ? 4
                  : tuning().sweep_items_per_block >= 2 ? 2 : 1;
  g.dmax = min_depth * (float)L;   // disp2depth = ones * MIN_DEPTH * nlabel (fp32)
  g.dstep = depth_mode ? min_depth : 0.0f;
  const int64_t items = (int64_t)B * g.groups * L * g.npw;
  SFM_REQUIRE(items < ((int64_t)1 << 31), "sweep too large for one launch");
  const int64_t blocks = (items + ipb - 1) / ipb;
  f32x4* tq = (f32x4*)ws;
  Proj* projs = reinterpret_cast<Proj*>((char*)ws + sweep_quads_bytes(B, C, h, w));
  float* depths = L <= kDepthTable ? reinterpret_cast<float*>((char*)projs + sweep_proj_bytes(B)) : nullptr;
  {
    ProfScope ps("sweep_tgt_quads", s);
    hipLaunchKernelGGL(k_tgt_quads, quads_grid(B, g.C4, hw, std::max(B, L)), dim3(256), 0, s, tgt, B, C, g.C4, hw, tq,
                       pose, K4, K4inv, projs, L, g.dmax, g.dstep, depths, prep);
  }
  SFM_LAUNCHED();
  const char* pname = with_ref ? "plane_sweep" : "plane_sweep_warped";
  // aligned-slab form: int slab offsets, 31-bit magic-number decode
  const int nq = tuning().sweep_group == 8 ? 2 : 1;
  const int64_t slab = (int64_t)L * hw;
  const int fgroups = (C + 4 * nq - 1) / (4 * nq);
  // the warped half alone (write_ref = 0): only k_sweep_tile honours write_ref
  // (the other forms would also write the reference rows, racing the side
  // stream's k_ref_planes with the same values), so it always takes that form
  const int mode = write_ref ? tuning().sweep_flat : 2;
  // k_sweep_tile: 256 * nj elements per window (bf16 packs register pairs: nj even)
  int nj = tuning().sweep_nj;
  if (out_dtype == 1 && nj < 2) nj = 2;
  // 16-byte lane stores: NJ = the tuned pixels per lane (bf16: 2, 4, 8;
  // fp32: 1, 2, 4); rows keep 16-byte alignment from window to window (slab
  // a multiple of a store's pixels)
  // default (-1): bf16 volumes 2 pixels per lane (the C3 sweep 0.454 -> 0.347 ms
  // in the bench step, profiles/r04_sweep_wide_ab.txt), fp32 1 pixel per lane
  // (with the nt sc1 policy below; 2 pixels per lane are slower)
  int store_px = tuning().sweep_store_px;
  if (store_px < 0) store_px = out_dtype == 1 ? 2 : 1;
  if (out_dtype == 1 && store_px == 1) store_px = 2;
  if (out_dtype == 0 && store_px == 8) store_px = 0;
  if (!(mode == 2 && slab % (out_dtype == 1 ? 8 : 4) == 0 && (uintptr_t)out % 16 == 0 && !tuning().sweep_share))
    store_px = 0;
  if (store_px) nj = store_px;
  if (mode == 3 && hw < (1 << 24) && slab < ((int64_t)1 << 30)) {
    const int bnj = out_dtype == 1 ? 2 : 1;
    const int esz = out_dtype == 0 ? 4 : 2;
    BandGeom bg;
    bg.C = C; bg.C4 = g.C4; bg.h = h; bg.w = w; bg.hw = hw; bg.L = L;
    bg.ref_rows = g.ref_rows; bg.rows = g.rows; bg.slab = (int)slab;
    bg.amask = 256 / esz - 1;
    bg.ntiles = (hw + bg.amask + 256 * bnj - 1) / (256 * bnj);
    bg.run = std::min(tuning().sweep_run, L);
    bg.nruns = (L + bg.run - 1) / bg.run;
    bg.out_mis = (int)(((uintptr_t)out / esz) & (uintptr_t)bg.amask);
    bg.hwmod = hw & bg.amask;
    bg.pair_ok = (slab % 2 == 0) && ((uintptr_t)out % 4 == 0);
    // two blocks per CU: <= 80 KB of LDS each
    const size_t lds_cap = 80 * 1024 - 64;
    const size_t row_bytes = (size_t)w * sizeof(f32x4);
    const size_t fixed = band_lds_bytes(0, w, bnj);
    const int rows_fit = lds_cap > fixed ? (int)((lds_cap - fixed) / row_bytes) : 0;
    bg.cap_rows = std::min(std::min(tuning().sweep_band_rows, rows_fit), h);
    const int64_t nblk = (int64_t)B * g.C4 * bg.nruns * bg.ntiles;
    if (bg.cap_rows >= 2 && nblk < ((int64_t)1 << 31)) {
      bg.mtile = make_magic((unsigned)bg.ntiles);
      bg.mrun = make_magic((unsigned)bg.nruns);
      bg.mgrp = make_magic((unsigned)bg.C4);
      bg.inv_w = 1.0f / (float)w;
      bg.dmax = g.dmax; bg.dstep = g.dstep;
      const unsigned lds = (unsigned)band_lds_bytes(bg.cap_rows, w, bnj);
      ProfScope ps(pname, s);
      if (out_dtype == 0) {
        SFM_HIP(hipFuncSetAttribute((const void*)k_sweep_band<float, 1>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((k_sweep_band<float, 1>), dim3((unsigned)nblk), dim3(kBandThreads), lds, s, ref, tq, pose,
                           K4, K4inv, bg, (float*)out);
      } else {
        SFM_HIP(hipFuncSetAttribute((const void*)k_sweep_band<unsigned short, 2>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL((k_sweep_band<unsigned short, 2>), dim3((unsigned)nblk), dim3(kBandThreads), lds, s, ref,
                           tq, pose, K4, K4inv, bg, (unsigned short*)out);
      }
      SFM_LAUNCHED();
      return SFM_OK;
    }
  }
  const int64_t win_el = mode == 2 ? 256 * (int64_t)nj : kFlatWin;
  const int64_t nwin = (slab + 127 + win_el - 1) / win_el;
  if (mode && hw < (1 << 24) && slab < ((int64_t)1 << 30) && (int64_t)B * fgroups * nwin < ((int64_t)1 << 31)) {
    FlatGeom fg;
    fg.B = B; fg.C = C; fg.C4 = g.C4; fg.h = h; fg.w = w; fg.L = L; fg.hw = hw;
    fg.ref_rows = g.ref_rows; fg.rows = g.rows; fg.G = 4 * nq; fg.groups = fgroups;
    fg.slab = (int)slab; fg.nwin = (int)nwin;
    const int esz = out_dtype == 0 ? 4 : 2;
    fg.amask = 256 / esz - 1;
    fg.out_mis = (int)(((uintptr_t)out / esz) & (uintptr_t)fg.amask);
    fg.pair_ok = (slab % 2 == 0) && ((uintptr_t)out % 4 == 0);
    const int64_t pair_bytes = (int64_t)g.rows * slab * esz;
    fg.buf_ok = pair_bytes < ((int64_t)1 << 32) && (out_dtype == 0 || fg.pair_ok) && tuning().sweep_buffer;
    fg.share = tuning().sweep_share;
    // auto (2): bf16 volumes always; fp32 volumes when a channel slab (L x h x w
    // floats) is at most 6 MiB.  Measured, not derived (profiles/r05_sweep_store_shapes.txt):
    // non-temporal fp32 stores are faster at 120x160 L=64 (the indoor c4 volume:
    // 0.73 vs 0.69 of HBM inside the bench step), 120x161 L=64, and equal at
    // 128x128 L=64 (slabs 4.2-4.9 MiB), slower at every slab of 7.5 MiB or more
    // (KITTI 94x311 at L = 64 and 128, 120x160 L=128, 100x300 L=64, 96x320)
    fg.store_nt = tuning().sweep_store_nt == 2 ? (out_dtype != 0 || slab * 4 <= ((int64_t)6 << 20))
                                               : tuning().sweep_store_nt;
    fg.write_ref = write_ref ? 1 : 0;
    fg.store_px = store_px;
    fg.pair_bytes = fg.buf_ok ? (unsigned)pair_bytes : 0u;
    fg.mwin = make_magic((unsigned)nwin);
    fg.mgrp = make_magic((unsigned)fgroups);
    fg.mhw = make_magic((unsigned)hw);
    fg.inv_w = 1.0f / (float)w;
    fg.dmax = g.dmax; fg.dstep = g.dstep;
    fg.depths = depths;
    {
      // auto (-1): fp32 volumes nt sc1 (write-through: the volume's lines do
      // not stay in the XCD's L2, where plain / nt stores keep them), bf16 by
      // sweep_store_nt.  Measured (profiles/r05_sweep_store_wt.txt): inside the
      // bench step the fp32 sweep 1.275 -> 1.245 ms (c2) and 0.440 -> 0.422 ms
      // (c4); bf16 slower with sc1 (0.359 -> 0.384 ms, c3)
      int wt = tuning().sweep_store_wt;
      if (wt < 0) wt = out_dtype == 0 ? 3 : 0;
      fg.wpol = wt == 1 ? 16 : wt == 2 ? 17 : wt == 3 ? 18 : -1;
    }
    const unsigned blocks = (unsigned)((int64_t)B * fgroups * nwin);
    ProfScope ps(pname, s);
    if (mode == 2) {
      if (out_dtype == 0) {
        if (nq == 2) launch_k_sweep_tile_nj<float, 2>(nj, blocks, s, ref, tq, pose, K4, K4inv, fg, out, projs);
        else launch_k_sweep_tile_nj<float, 1>(nj, blocks, s, ref, tq, pose, K4, K4inv, fg, out, projs);
      } else {
        if (nq == 2) launch_k_sweep_tile_nj<unsigned short, 2>(nj, blocks, s, ref, tq, pose, K4, K4inv, fg, out, projs);
        else launch_k_sweep_tile_nj<unsigned short, 1>(nj, blocks, s, ref, tq, pose, K4, K4inv, fg, out, projs);
      }
    } else if (out_dtype == 0) launch_k_sweep_flat<float>(nq, blocks, s, ref, tq, pose, K4, K4inv, fg, out);
    else launch_k_sweep_flat<unsigned short>(nq, blocks, s, ref, tq, pose, K4, K4inv, fg, out);
    SFM_LAUNCHED();
    return SFM_OK;
  }
  SFM_REQUIRE(write_ref, "warped-half sweep: the shape is outside k_sweep_tile's range");
  ProfScope ps(pname, s);
  if (out_dtype == 0) {
    if (vec) launch_k_sweep<float, true>(ipb, blocks, s, ref, tq, pose, K4, K4inv, g, out);
    else launch_k_sweep<float, false>(ipb, blocks, s, ref, tq, pose, K4, K4inv, g, out);
  } else {
    if (vec) launch_k_sweep<unsigned short, true>(ipb, blocks, s, ref, tq, pose, K4, K4inv, g, out);
    else launch_k_sweep<unsigned short, false>(ipb, blocks, s, ref, tq, pose, K4, K4inv, g, out);
  }
  SFM_LAUNCHED();
  return SFM_OK;
}

// ---------------------------------------------------------------------------
// The volume's reference half on its own (round 4).  cost[b][c][l] =
// ref[b][c] for every plane l (PSNet.py:155) does not depend on the pose, so
// the hot path writes it on a side stream while RANSAC runs and the sweep
// after RANSAC writes only the warped half (k_sweep_tile with write_ref = 0).
// The scorer is compute-bound and leaves the memory system idle, but it holds
// 3 waves x 168 VGPRs per SIMD: k_ref_planes is built to fit the remaining 8
// VGPRs (one wave per SIMD beside the scorer's three).
//   k_ref_pad:    ref [B*C][hw] -> rp [B*C][hw + kRefPad], rp[i] = ref[i mod hw]
//                 (a row and its first kRefPad elements again, so that six
//                 consecutive 64-element chunks never wrap)
//   k_ref_planes: persistent; wave w copies the w-th contiguous range of the
//                 64-element chunks of every pair's reference half (C slabs of
//                 L * hw elements, chunks never straddle a slab: L * hw % 64
//                 == 0); lane i of a chunk at slab element e reads rp[c][e mod
//                 hw] (one dword, L2-resident) and writes it, so a wave store
//                 is one aligned 256-byte segment.  Six chunks per iteration.
// Same values as the full sweep's reference rows (a copy; bf16 by the same
// RNE conversion).  Shapes outside the fast path take k_ref_planes_generic.
// ---------------------------------------------------------------------------
constexpr int kRefUnroll = 4;   // dwords in flight per lane: 8 VGPRs in all
constexpr int kRefPad = 64 * kRefUnroll;

__global__ __launch_bounds__(256) void k_ref_pad(const float* __restrict__ ref, int hw, float* __restrict__ rp) {
  const size_t row = blockIdx.y;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < hw + kRefPad; i += gridDim.x * 256)
    rp[row * (size_t)(hw + kRefPad) + i] = ref[row * (size_t)hw + (i < hw ? i : (i - hw) % hw)];
}

template <typename OutT>
__device__ __forceinline__ void ref_bstore(__amdgpu_buffer_rsrc_t r, float v, unsigned voff, unsigned soff);
template <>
__device__ __forceinline__ void ref_bstore<float>(__amdgpu_buffer_rsrc_t r, float v, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff * 4u, soff * 4u, 0);
}
template <>
__device__ __forceinline__ void ref_bstore<unsigned short>(__amdgpu_buffer_rsrc_t r, float v, unsigned voff,
                                                           unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b16(to_bf16(v), r, voff * 2u, soff * 2u, 0);
}
template <typename OutT>
__device__ __forceinline__ void ref_store(OutT* dst, float v);
template <>
__device__ __forceinline__ void ref_store<float>(float* dst, float v) { *dst = v; }
template <>
__device__ __forceinline__ void ref_store<unsigned short>(unsigned short* dst, float v) { *dst = to_bf16(v); }

// One wave's share of the chunks, and the uniform decode constants (host-made:
// no integer division on the device, whose VALU expansion would hold VGPRs).
struct RefPlanes {
  unsigned cps;        // 64-element chunks per slab (L * hw / 64)
  unsigned q, r;       // total chunks / waves, remainder: wave w takes q (+1 if w < r)
  int C, hw, L;
  Magic mcps, mC, mhw;
};

// grid: one 256-thread block per CU (one wave per SIMD).  Buffer addressing
// keeps the per-lane state to the source offset and the lane's element: every
// uniform part of an address is an SGPR (resource base, soffset).
template <typename OutT>
__global__ __launch_bounds__(256) void k_ref_planes(const float* __restrict__ rp, RefPlanes g,
                                                    OutT* __restrict__ out) {
  const unsigned lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const unsigned w = blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  unsigned m = w * g.q + min(w, g.r);
  const unsigned hi = m + g.q + (w < g.r ? 1u : 0u);
  const unsigned slab_bytes = (unsigned)g.L * (unsigned)g.hw * (unsigned)sizeof(OutT);
  const unsigned hw = (unsigned)g.hw;
  while (m < hi) {
    // uniform: slab (pair b, channel c) and chunk j of m
    const unsigned sl = magic_div(m, g.mcps);
    const unsigned j = m - sl * g.cps;
    const unsigned b = magic_div(sl, g.mC), c = sl - b * (unsigned)g.C;
    unsigned n = min(hi - m, g.cps - j);
    const __amdgpu_buffer_rsrc_t rsrc = buf_rsrc(rp + ((size_t)b * g.C + c) * (size_t)(hw + kRefPad),
                                                 (hw + kRefPad) * 4u);
    const __amdgpu_buffer_rsrc_t rdst = buf_rsrc(out + ((size_t)b * 2 * g.C + c) * (size_t)g.L * hw, slab_bytes);
    unsigned e = j * 64u;                                      // slab element of the chunk (uniform)
    const unsigned e0 = e - magic_div(e, g.mhw) * hw;          // e mod hw
    unsigned p = e0 + lane;                                    // source element of this lane
    p = min(p, p - hw);                                        // mod hw (unsigned wrap: the smaller is it)
    m += n;
    for (; n >= (unsigned)kRefUnroll; n -= kRefUnroll) {
      float v[kRefUnroll];
#pragma unroll
      for (int k = 0; k < kRefUnroll; ++k)
        v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, p * 4u, 256u * k, 0));
#pragma unroll
      for (int k = 0; k < kRefUnroll; ++k) ref_bstore<OutT>(rdst, v[k], lane, e + 64u * k);
      e += 64u * kRefUnroll;
      p += 64u * kRefUnroll;
      p = min(p, p - hw);
    }
    for (; n > 0; --n) {
      ref_bstore<OutT>(rdst, __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, p * 4u, 0u, 0)), lane, e);
      e += 64u;
      p += 64u;
      p = min(p, p - hw);
    }
  }
}

// any shape: one thread per element of the reference half
template <typename OutT>
__global__ __launch_bounds__(256) void k_ref_planes_generic(const float* __restrict__ ref, int C, int hw, int L,
                                                            OutT* __restrict__ out) {
  const size_t slab = (size_t)L * hw;
  const size_t bc = blockIdx.y;                              // b * C + c
  const size_t b = bc / C, c = bc - b * C;
  OutT* dst = out + (b * 2 * C + c) * slab;
  const float* src = ref + bc * hw;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < slab; e += (size_t)gridDim.x * 256)
    ref_store<OutT>(dst + e, src[e % hw]);
}

static size_t ref_planes_ws_bytes(int B, int C, int h, int w) {
  return (((size_t)B * C * ((size_t)h * w + kRefPad) * sizeof(float)) + 255) & ~(size_t)255;
}

}  // namespace sfm

using namespace sfm;

extern "C" {

size_t sfm_plane_sweep_workspace_bytes(int batch, int channels, int h, int w) {
  if (batch < 1 || channels < 1 || h < 1 || w < 1) return 0;
  return sweep_ws_bytes(batch, channels, h, w);
}

int sfm_plane_sweep_ex(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                       const float* pose, const float* K4, const float* K4inv, int nlabel, float min_depth,
                       int depth_mode, int out_dtype, void* cost, void* workspace, size_t workspace_bytes,
                       void* stream) {
  return launch_sweep(ref != nullptr, ref, tgt, batch, channels, h, w, pose, K4, K4inv, nlabel, min_depth,
                      depth_mode, out_dtype, cost, workspace, workspace_bytes, (hipStream_t)stream);
}

int sfm_plane_sweep(const float* ref, const float* tgt, int batch, int channels, int h, int w, const float* pose,
                    const float* K4, const float* K4inv, int nlabel, float min_depth, int out_dtype, void* cost,
                    void* workspace, size_t workspace_bytes, void* stream) {
  SFM_REQUIRE(ref, "null pointer argument");
  return launch_sweep(true, ref, tgt, batch, channels, h, w, pose, K4, K4inv, nlabel, min_depth, 0, out_dtype, cost,
                      workspace, workspace_bytes, (hipStream_t)stream);
}

int sfm_plane_sweep_psnet(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                          const void* pose, int pose_dtype, const float* K, const float* Kinv, float t_scale,
                          int nlabel, float min_depth, int depth_mode, int out_dtype, void* cost, void* workspace,
                          size_t workspace_bytes, void* stream) {
  SFM_REQUIRE(tgt && pose && K && Kinv && cost && workspace, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && channels >= 1 && h >= 2 && w >= 2, "invalid sweep shape");
  SFM_REQUIRE(pose_dtype == 0 || pose_dtype == 1, "pose_dtype must be 0 (float32) or 1 (float64)");
  // every argument launch_sweep checks, before the preparation kernel runs
  SFM_REQUIRE(nlabel >= 1, "invalid sweep shape");
  SFM_REQUIRE(out_dtype == 0 || out_dtype == 1, "out_dtype must be 0 (float32) or 1 (bfloat16)");
  SFM_REQUIRE(depth_mode == 0 || depth_mode == 1, "depth_mode must be 0 (inverse depth) or 1 (depth)");
  SFM_REQUIRE(min_depth > 0.0f, "min_depth must be positive");
  SFM_REQUIRE((int64_t)h * w < ((int64_t)1 << 30), "feature map too large");
  const size_t need = sweep_ws_bytes(batch, channels, h, w);
  if (workspace_bytes < need) {
    set_error("plane sweep workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  hipStream_t s = (hipStream_t)stream;
  float* prep = reinterpret_cast<float*>((char*)workspace + sweep_core_bytes(batch, channels, h, w));
  // the preparation runs inside the sweep's first kernel (k_tgt_quads, one
  // thread per pair before its Proj), not as a launch of its own; the sweep's
  // own scratch excludes the prep region at the workspace's end
  return launch_sweep(ref != nullptr, ref, tgt, batch, channels, h, w, prep, prep + (size_t)batch * 12,
                      prep + (size_t)batch * 21, nlabel, min_depth, depth_mode, out_dtype, cost, workspace,
                      sweep_core_bytes(batch, channels, h, w), s,
                      PsnetPrep{pose, pose_dtype, K, Kinv, t_scale, prep});
}

size_t sfm_plane_sweep_ref_planes_workspace_bytes(int batch, int channels, int h, int w) {
  if (batch < 1 || channels < 1 || h < 1 || w < 1) return 0;
  return ref_planes_ws_bytes(batch, channels, h, w);
}

int sfm_plane_sweep_ref_planes(const float* ref, int batch, int channels, int h, int w, int nlabel, int out_dtype,
                               void* cost, void* workspace, size_t workspace_bytes, void* stream) {
  SFM_REQUIRE(ref && cost, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && batch <= 65535 && channels >= 1 && channels <= 65535 && h >= 1 && w >= 1 && nlabel >= 1,
              "invalid sweep shape");
  SFM_REQUIRE(out_dtype == 0 || out_dtype == 1, "out_dtype must be 0 (float32) or 1 (bfloat16)");
  SFM_REQUIRE((int64_t)h * w < ((int64_t)1 << 30), "feature map too large");
  // k_ref_pad / k_ref_planes_generic take one (pair, channel) row per grid y
  SFM_REQUIRE((int64_t)batch * channels <= 65535, "batch * channels must be <= 65535");
  hipStream_t s = (hipStream_t)stream;
  const int hw = h * w;
  const int64_t slab = (int64_t)nlabel * hw;
  const int esz = out_dtype == 0 ? 4 : 2;
  // fast path: chunks within slabs, a padded row that six chunks never wrap, 256-byte aligned slabs
  // (magic_div needs n < 2^31: chunk counts and slab elements)
  const bool fast = slab % 64 == 0 && hw >= kRefPad && ((uintptr_t)cost % 256) == 0 && (slab * esz) % 256 == 0 &&
                    (int64_t)batch * channels * (slab / 64) < ((int64_t)1 << 31) && slab < ((int64_t)1 << 31) &&
                    slab * esz < ((int64_t)1 << 32) && workspace &&
                    workspace_bytes >= ref_planes_ws_bytes(batch, channels, h, w);
  ProfScope ps("ref_planes", s);
  if (fast) {
    float* rp = (float*)workspace;
    hipLaunchKernelGGL(k_ref_pad, dim3((hw + kRefPad + 255) / 256, (unsigned)(batch * channels)), dim3(256), 0, s,
                       ref, hw, rp);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    cus = std::max(1, cus);
    RefPlanes g;
    g.cps = (unsigned)(slab / 64);
    const unsigned waves = (unsigned)cus * 4u;
    const int64_t total = (int64_t)batch * channels * g.cps;
    g.q = (unsigned)(total / waves);
    g.r = (unsigned)(total % waves);
    g.C = channels; g.hw = hw; g.L = nlabel;
    g.mcps = make_magic(g.cps); g.mC = make_magic((unsigned)channels); g.mhw = make_magic((unsigned)hw);
    if (out_dtype == 0)
      hipLaunchKernelGGL(k_ref_planes<float>, dim3(cus), dim3(256), 0, s, rp, g, (float*)cost);
    else
      hipLaunchKernelGGL(k_ref_planes<unsigned short>, dim3(cus), dim3(256), 0, s, rp, g, (unsigned short*)cost);
  } else {
    const unsigned gx = (unsigned)std::min<int64_t>((slab + 255) / 256, 4096);
    if (out_dtype == 0)
      hipLaunchKernelGGL(k_ref_planes_generic<float>, dim3(gx, (unsigned)(batch * channels)), dim3(256), 0, s, ref,
                         channels, hw, nlabel, (float*)cost);
    else
      hipLaunchKernelGGL(k_ref_planes_generic<unsigned short>, dim3(gx, (unsigned)(batch * channels)), dim3(256), 0,
                         s, ref, channels, hw, nlabel, (unsigned short*)cost);
  }
  SFM_LAUNCHED();
  return SFM_OK;
}

int sfm_plane_sweep_psnet_warped_half(const float* ref, const float* tgt, int batch, int channels, int h, int w, const void* pose,
                                      int pose_dtype, const float* K, const float* Kinv, float t_scale, int nlabel,
                                      float min_depth, int depth_mode, int out_dtype, void* cost, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  SFM_REQUIRE(ref && tgt && pose && K && Kinv && cost && workspace, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && channels >= 1 && h >= 2 && w >= 2, "invalid sweep shape");
  SFM_REQUIRE(pose_dtype == 0 || pose_dtype == 1, "pose_dtype must be 0 (float32) or 1 (float64)");
  SFM_REQUIRE(nlabel >= 1, "invalid sweep shape");
  SFM_REQUIRE(out_dtype == 0 || out_dtype == 1, "out_dtype must be 0 (float32) or 1 (bfloat16)");
  SFM_REQUIRE(depth_mode == 0 || depth_mode == 1, "depth_mode must be 0 (inverse depth) or 1 (depth)");
  SFM_REQUIRE(min_depth > 0.0f, "min_depth must be positive");
  SFM_REQUIRE((int64_t)h * w < ((int64_t)1 << 30), "feature map too large");
  const size_t need = sweep_ws_bytes(batch, channels, h, w);
  if (workspace_bytes < need) {
    set_error("plane sweep workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  hipStream_t s = (hipStream_t)stream;
  float* prep = reinterpret_cast<float*>((char*)workspace + sweep_core_bytes(batch, channels, h, w));
  // the full volume's geometry (2C rows per plane) with its reference rows
  // left to sfm_plane_sweep_ref_planes; windows off k_sweep_tile's fast path
  // (edges, other sweep modes) still write them from `ref`: the same values
  return launch_sweep(true, ref, tgt, batch, channels, h, w, prep, prep + (size_t)batch * 12,
                      prep + (size_t)batch * 21, nlabel, min_depth, depth_mode, out_dtype, cost, workspace,
                      sweep_core_bytes(batch, channels, h, w), s,
                      PsnetPrep{pose, pose_dtype, K, Kinv, t_scale, prep}, false);
}

int sfm_plane_sweep_warped(const float* tgt, int batch, int channels, int h, int w, const float* pose,
                           const float* K4, const float* K4inv, int nlabel, float min_depth, int out_dtype,
                           void* out, void* workspace, size_t workspace_bytes, void* stream) {
  return launch_sweep(false, nullptr, tgt, batch, channels, h, w, pose, K4, K4inv, nlabel, min_depth, 0, out_dtype,
                      out, workspace, workspace_bytes, (hipStream_t)stream);
}

int sfm_inverse_warp(const float* feat, int batch, int channels, int h, int w, const float* depth,
                     const float* pose, const float* K, const float* Kinv, float* out, void* stream) {
  SFM_REQUIRE(feat && depth && pose && K && Kinv && out, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && batch <= 65535 && channels >= 1 && h >= 2 && w >= 2, "invalid warp shape");
  const int hw = h * w;
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps("inverse_warp", s);
  hipLaunchKernelGGL(k_inverse_warp, dim3((hw + kSweepThreads - 1) / kSweepThreads, batch), dim3(kSweepThreads), 0,
                     s, feat, channels, h, w, depth, pose, K, Kinv, out);
  SFM_LAUNCHED();
  return SFM_OK;
}

}  // extern "C"
