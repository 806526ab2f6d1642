// Plane-sweep cost volume and inverse warp on CDNA4 (gfx950).
//
// Replaces the per-plane Python loop of models/PSNet.py:144-158 (L iterations
// of ~10 ATen launches: bmm, elementwise, grid_sample, two strided copies)
// with one launch that writes the whole [B, 2C, L, h, w] volume (plus a tiny
// channel-quad relayout of the target features).  HBM-write-bound.
//
// Arithmetic follows the reference's float32 expression order:
//   cam = (Kinv . (x, y, 1)) * d              pixel2cam (27-41)
//   p   = (K.pose)[:, :3] . cam + (K.pose)[:, 3]   cam2pixel (44-75)
//   Z clamped at 1e-3, xn = 2 (X/Z)/(w-1) - 1, |xn| > 1 -> 2 (zero sample)
//   grid_sample bilinear, zeros padding, align_corners=True
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <string>
#include "common.h"

namespace sfm {

constexpr int kSweepThreads = 256;

struct Proj {   // (K . pose) rows and Kinv
  float m[12];
  float ki[9];
};

__device__ __forceinline__ void load_proj(const float* __restrict__ pose, const float* __restrict__ K,
                                          const float* __restrict__ Kinv, int b, Proj& pr) {
  const float* Pb = pose + b * 12;
  const float* Kb = K + b * 9;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c)
      pr.m[4 * r + c] = (Kb[3 * r + 0] * Pb[c] + Kb[3 * r + 1] * Pb[4 + c]) + Kb[3 * r + 2] * Pb[8 + c];
#pragma unroll
  for (int e = 0; e < 9; ++e) pr.ki[e] = Kinv[b * 9 + e];
}

// Sampling position for a pixel ray `ray` (K^-1 (x,y,1)) at depth d.
// Returns false when the sample is outside the image (the reference pushes the
// normalised coordinate to 2 and grid_sample returns 0 for every channel).
__device__ __forceinline__ bool sample_pos(const Proj& pr, const float ray[3], float d, int h, int w,
                                           float& ix, float& iy) {
  const float c0 = ray[0] * d, c1 = ray[1] * d, c2 = ray[2] * d;
  const float X = ((pr.m[0] * c0 + pr.m[1] * c1) + pr.m[2] * c2) + pr.m[3];
  const float Y = ((pr.m[4] * c0 + pr.m[5] * c1) + pr.m[6] * c2) + pr.m[7];
  float Z = ((pr.m[8] * c0 + pr.m[9] * c1) + pr.m[10] * c2) + pr.m[11];
  Z = Z < 1e-3f ? 1e-3f : Z;
  const float xn = 2.0f * (X / Z) / (float)(w - 1) - 1.0f;
  const float yn = 2.0f * (Y / Z) / (float)(h - 1) - 1.0f;
  if (!(xn <= 1.0f && xn >= -1.0f && yn <= 1.0f && yn >= -1.0f)) return false;
  ix = ((xn + 1.0f) / 2.0f) * (float)(w - 1);
  iy = ((yn + 1.0f) / 2.0f) * (float)(h - 1);
  return true;
}

struct Taps {
  int off[4];
  float wt[4];
};

__device__ __forceinline__ void make_taps(float ix, float iy, int h, int w, Taps& t) {
  const float fx = floorf(ix), fy = floorf(iy);
  const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
  const float wx1 = ix - fx, wx0 = (fx + 1.0f) - ix;
  const float wy1 = iy - fy, wy0 = (fy + 1.0f) - iy;
  const bool vx0 = x0 >= 0 && x0 < w, vx1 = x1 >= 0 && x1 < w;
  const bool vy0 = y0 >= 0 && y0 < h, vy1 = y1 >= 0 && y1 < h;
  // nw, ne, sw, se (grid_sampler_2d order); invalid taps weight 0, clamped address
  t.wt[0] = (vx0 && vy0) ? wx0 * wy0 : 0.0f;
  t.wt[1] = (vx1 && vy0) ? wx1 * wy0 : 0.0f;
  t.wt[2] = (vx0 && vy1) ? wx0 * wy1 : 0.0f;
  t.wt[3] = (vx1 && vy1) ? wx1 * wy1 : 0.0f;
  const int cx0 = min(max(x0, 0), w - 1), cx1 = min(max(x1, 0), w - 1);
  const int cy0 = min(max(y0, 0), h - 1), cy1 = min(max(y1, 0), h - 1);
  t.off[0] = cy0 * w + cx0;
  t.off[1] = cy0 * w + cx1;
  t.off[2] = cy1 * w + cx0;
  t.off[3] = cy1 * w + cx1;
}

__device__ __forceinline__ unsigned short to_bf16(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return *reinterpret_cast<unsigned short*>(&b);
}

// ---------------------------------------------------------------------------
// Cost volume, v2: the output is produced in address order.
//
// Work item = (pair b, 4-row channel group g, plane l, 1024-pixel window):
// 256 threads x 4 consecutive pixels write four 4 KB row segments with
// 16-byte stores.  Items are enumerated with the window fastest, then the
// plane, then the group, then the pair, and each block takes kSwItems
// consecutive items, so the chip streams through the [B, 2C, L, h, w] volume
// roughly in address order (a volume written as thousands of scattered row
// chunks tops out ~20% lower on MI355X: scripts/probe_store_bw.hip).
//
// Groups [0, C4) copy the reference features (rows c < C, identical for every
// plane); groups [C4, 2 C4) are the warped target features: the 4 bilinear
// taps of each pixel are read as float4 from the channel-quad layout
// tq[B][C4][h*w][4] (one 16-byte load per tap per 4 channels).
//
// 16-byte alignment: a row starts at element ((b*rows + r)*L + l)*h*w.  With
// h*w = 2 (mod 4) and L even, that is 2*(l & 1) (mod 4) for every row of the
// plane, so the pixel windows of odd planes are shifted by 2.  Other shapes
// take the element-wise store path (correct, slower).
// ---------------------------------------------------------------------------
constexpr int kSwThreads = 256;
constexpr int kSwPix = 4;
constexpr int kSwWin = kSwThreads * kSwPix;
constexpr int kSwItems = 8;

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// tgt [B][C][hw] -> tq [B][C4][hw] float4 (channels >= C are zero)
__global__ void k_tgt_quads(const float* __restrict__ tgt, int B, int C, int C4, int hw, f32x4* __restrict__ tq) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)B * C4 * hw;
  if (i >= total) return;
  const int p = (int)(i % hw);
  const int64_t bq = i / hw;
  const int q = (int)(bq % C4), b = (int)(bq / C4);
  f32x4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = 4 * q + k;
    v[k] = c < C ? tgt[((size_t)b * C + c) * hw + p] : 0.0f;
  }
  tq[i] = v;
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

template <typename OutT, bool VEC>
__global__ __launch_bounds__(kSwThreads) void k_sweep(const float* __restrict__ ref, const f32x4* __restrict__ tq,
                                                      int B, int C, int C4, int h, int w,
                                                      const float* __restrict__ pose, const float* __restrict__ K4,
                                                      const float* __restrict__ K4inv, int L, float dmax,
                                                      int with_ref, int shift_mode, OutT* __restrict__ out) {
  const int hw = h * w;
  const int npw = (hw + 3 + kSwWin - 1) / kSwWin;
  const int groups = with_ref ? 2 * C4 : C4;
  const int rows = with_ref ? 2 * C : C;
  const int64_t per_group = (int64_t)L * npw;
  const int64_t total = (int64_t)B * groups * per_group;
  const int64_t first = (int64_t)blockIdx.x * kSwItems;
  for (int it = 0; it < kSwItems; ++it) {
    const int64_t item = first + it;
    if (item >= total) return;
    const int pw = (int)(item % npw);
    int64_t r = item / npw;
    const int l = (int)(r % L);
    r /= L;
    const int g = (int)(r % groups);
    const int b = (int)(r / groups);
    const int shift = shift_mode ? 2 * (l & 1) : 0;
    const int p0 = pw * kSwWin - shift + threadIdx.x * kSwPix;
    if (p0 >= hw) continue;
    OutT* plane = out + ((size_t)b * rows * L + l) * hw;    // row r at plane + r * L * hw
    const size_t rstride = (size_t)L * hw;
    if (with_ref && g < C4) {
      // reference half: rows 4g .. 4g+3
      const float* R = ref + (size_t)b * C * hw;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = 4 * g + k;
        if (c >= C) break;
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int p = min(max(p0 + j, 0), hw - 1);
          v[j] = R[(size_t)c * hw + p];
        }
        store_row<OutT, VEC>(plane + (size_t)c * rstride, p0, hw, v);
      }
      continue;
    }
    const int q = with_ref ? g - C4 : g;
    Proj pr;
    load_proj(pose, K4, K4inv, b, pr);
    const float d = dmax / (float)(l + 1);
    const f32x4* T = tq + ((size_t)b * C4 + q) * hw;
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = min(max(p0 + j, 0), hw - 1);
      const float x = (float)(p % w), y = (float)(p / w);
      float ray[3];
      ray[0] = (pr.ki[0] * x + pr.ki[1] * y) + pr.ki[2];
      ray[1] = (pr.ki[3] * x + pr.ki[4] * y) + pr.ki[5];
      ray[2] = (pr.ki[6] * x + pr.ki[7] * y) + pr.ki[8];
      float ix, iy;
      acc[j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      if (sample_pos(pr, ray, d, h, w, ix, iy)) {
        Taps tp;
        make_taps(ix, iy, h, w, tp);
        const f32x4 t0 = T[tp.off[0]], t1 = T[tp.off[1]], t2 = T[tp.off[2]], t3 = T[tp.off[3]];
        f32x4 a = tp.wt[0] * t0;
        a = a + tp.wt[1] * t1;
        a = a + tp.wt[2] * t2;
        a = a + tp.wt[3] * t3;
        acc[j] = a;
      }
    }
    const int cbase = with_ref ? C : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = 4 * q + k;
      if (c >= C) break;
      const float v[4] = {acc[0][k], acc[1][k], acc[2][k], acc[3][k]};
      store_row<OutT, VEC>(plane + (size_t)(cbase + c) * rstride, p0, hw, v);
    }
  }
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

static size_t sweep_ws_bytes(int B, int C, int h, int w) {
  const int C4 = (C + 3) / 4;
  return (size_t)B * C4 * (size_t)h * w * 16;
}

static int launch_sweep(bool with_ref, const float* ref, const float* tgt, int B, int C, int h, int w,
                        const float* pose, const float* K4, const float* K4inv, int L, float min_depth,
                        int out_dtype, void* out, void* ws, size_t ws_bytes, hipStream_t s) {
  SFM_REQUIRE(tgt && pose && K4 && K4inv && out && (!with_ref || ref), "null pointer argument");
  SFM_REQUIRE(B >= 1 && C >= 1 && h >= 2 && w >= 2 && L >= 1, "invalid sweep shape");
  SFM_REQUIRE(out_dtype == 0 || out_dtype == 1, "out_dtype must be 0 (float32) or 1 (bfloat16)");
  SFM_REQUIRE((int64_t)h * w < ((int64_t)1 << 30), "feature map too large");
  const size_t need = sweep_ws_bytes(B, C, h, w);
  if (!ws || ws_bytes < need) {
    set_error("plane sweep workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  const int hw = h * w, C4 = (C + 3) / 4;
  const int npw = (hw + 3 + kSwWin - 1) / kSwWin;
  const int groups = with_ref ? 2 * C4 : C4;
  const int64_t items = (int64_t)B * groups * L * npw;
  const int64_t blocks = (items + kSwItems - 1) / kSwItems;
  SFM_REQUIRE(blocks < ((int64_t)1 << 31), "sweep grid too large");
  // 16-byte row alignment (see k_sweep): every row aligned if hw % 4 == 0; rows of
  // plane l shifted by 2*(l&1) if hw % 4 == 2 and L even; element stores otherwise
  const bool vec = (hw % 4 == 0) || (hw % 4 == 2 && L % 2 == 0);
  const int shift_mode = (hw % 4 == 2 && L % 2 == 0) ? 1 : 0;
  const float dmax = min_depth * (float)L;   // disp2depth = ones * MIN_DEPTH * nlabel (fp32)
  f32x4* tq = (f32x4*)ws;
  {
    ProfScope ps("sweep_tgt_quads", s);
    const int64_t n = (int64_t)B * C4 * hw;
    hipLaunchKernelGGL(k_tgt_quads, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tgt, B, C, C4, hw, tq);
  }
  SFM_LAUNCHED();
  ProfScope ps(with_ref ? "plane_sweep" : "plane_sweep_warped", s);
#define SFM_SWEEP_LAUNCH(OT, V)                                                                              \
  hipLaunchKernelGGL((k_sweep<OT, V>), dim3((unsigned)blocks), dim3(kSwThreads), 0, s, ref, tq, B, C, C4, h, w, \
                     pose, K4, K4inv, L, dmax, with_ref ? 1 : 0, shift_mode, (OT*)out)
  if (out_dtype == 0) { if (vec) SFM_SWEEP_LAUNCH(float, true); else SFM_SWEEP_LAUNCH(float, false); }
  else { if (vec) SFM_SWEEP_LAUNCH(unsigned short, true); else SFM_SWEEP_LAUNCH(unsigned short, false); }
#undef SFM_SWEEP_LAUNCH
  SFM_LAUNCHED();
  return SFM_OK;
}

}  // namespace sfm

using namespace sfm;

extern "C" {

size_t sfm_plane_sweep_workspace_bytes(int batch, int channels, int h, int w) {
  if (batch < 1 || channels < 1 || h < 1 || w < 1) return 0;
  return sweep_ws_bytes(batch, channels, h, w);
}

int sfm_plane_sweep(const float* ref, const float* tgt, int batch, int channels, int h, int w, const float* pose,
                    const float* K4, const float* K4inv, int nlabel, float min_depth, int out_dtype, void* cost,
                    void* workspace, size_t workspace_bytes, void* stream) {
  return launch_sweep(true, ref, tgt, batch, channels, h, w, pose, K4, K4inv, nlabel, min_depth, out_dtype, cost,
                      workspace, workspace_bytes, (hipStream_t)stream);
}

int sfm_plane_sweep_warped(const float* tgt, int batch, int channels, int h, int w, const float* pose,
                           const float* K4, const float* K4inv, int nlabel, float min_depth, int out_dtype,
                           void* out, void* workspace, size_t workspace_bytes, void* stream) {
  return launch_sweep(false, nullptr, tgt, batch, channels, h, w, pose, K4, K4inv, nlabel, min_depth, out_dtype,
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
