// Projection / sampling helpers shared by the plane-sweep kernels
// (sweep.hip: cost volume, inverse warp; depth.hip: correlation cost).
//
// Arithmetic follows the reference's float32 expression order:
//   cam = (Kinv . (x, y, 1)) * d              pixel2cam (inverse_warp.py:27-41)
//   p   = (K.pose)[:, :3] . cam + (K.pose)[:, 3]   cam2pixel (44-75)
//   Z clamped at 1e-3, xn = 2 (X/Z)/(w-1) - 1, |xn| > 1 -> 2 (zero sample)
//   grid_sample bilinear, zeros padding, align_corners=True
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include "common.h"

namespace sfm {

typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// IEEE float32 division a / b (the reference's '/') by the Newton-Raphson
// steps of the compiler's V_DIV_SCALE / V_DIV_FMAS / V_DIV_FIXUP expansion,
// without its range scaling and special-case fixup.  Bit-identical to '/'
// whenever the expansion would not scale or fix up: a, b, 1/b and a/b normal
// and finite, |a| >= 2^-103 and exponent(a) - exponent(b) < 96.  y = rcp_nr(b).
__device__ __forceinline__ float rcp_nr(float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = __builtin_fmaf(-b, y0, 1.0f);
  return __builtin_fmaf(e, y0, y0);
}
__device__ __forceinline__ float div_nr(float a, float b, float y) {
  const float q0 = a * y;
  const float r0 = __builtin_fmaf(-b, q0, a);
  const float q1 = __builtin_fmaf(r0, y, q0);
  const float r1 = __builtin_fmaf(-b, q1, a);
  return __builtin_fmaf(r1, y, q1);
}

// Per-launch constants of sample_pos_nr (uniform).
struct SampleK {
  float cw, ch;     // (float)(w - 1), (float)(h - 1)
  float yw, yh;     // rcp_nr of each
  float hw1, hh1;   // (w - 1) / 2, (h - 1) / 2 (exact)
};
__device__ __forceinline__ SampleK sample_consts(int h, int w) {
  SampleK k;
  k.cw = (float)(w - 1);
  k.ch = (float)(h - 1);
  k.yw = rcp_nr(k.cw);
  k.yh = rcp_nr(k.ch);
  k.hw1 = 0.5f * k.cw;
  k.hh1 = 0.5f * k.ch;
  return k;
}

// sample_pos with its four divisions in the Newton-Raphson form: the same
// decision and the same ix, iy bits.
//  * X / Z and Y / Z: |X|, |Y| <= 2^60 and 1e-3 <= Z <= 2^60 keep div_nr in
//    its exact range, except for |X| < 2^-103 (or a denormal quotient), where
//    the quotient may differ in its last bits but 2 q / (w - 1) - 1 rounds to
//    exactly -1 either way.  Other operands (huge or NaN) take '/'.
//  * 2 q / (w - 1): |2 q| <= 2^71 against w - 1 >= 1; tiny 2 q as above.
//  * ((xn + 1) / 2) (w - 1) = (xn + 1) ((w - 1) / 2): the halving is exact,
//    so both are the one rounding of the same real product.
__device__ __forceinline__ bool sample_pos_nr(const Proj& pr, const float ray[3], float d, const SampleK& k,
                                              float& ix, float& iy) {
  const float c0 = ray[0] * d, c1 = ray[1] * d, c2 = ray[2] * d;
  const float X = ((pr.m[0] * c0 + pr.m[1] * c1) + pr.m[2] * c2) + pr.m[3];
  const float Y = ((pr.m[4] * c0 + pr.m[5] * c1) + pr.m[6] * c2) + pr.m[7];
  float Z = ((pr.m[8] * c0 + pr.m[9] * c1) + pr.m[10] * c2) + pr.m[11];
  Z = Z < 1e-3f ? 1e-3f : Z;
  float qx, qy;
  if (fabsf(X) <= 0x1p60f && fabsf(Y) <= 0x1p60f && Z <= 0x1p60f) {
    const float yz = rcp_nr(Z);
    qx = div_nr(X, Z, yz);
    qy = div_nr(Y, Z, yz);
  } else {
    qx = X / Z;
    qy = Y / Z;
  }
  const float xn = div_nr(2.0f * qx, k.cw, k.yw) - 1.0f;
  const float yn = div_nr(2.0f * qy, k.ch, k.yh) - 1.0f;
  if (!(xn <= 1.0f && xn >= -1.0f && yn <= 1.0f && yn >= -1.0f)) return false;
  ix = (xn + 1.0f) * k.hw1;
  iy = (yn + 1.0f) * k.hh1;
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

// tgt [B][C][hw] -> tq [B][C4][hw] float4 (channels >= C zero); sweep.hip
void launch_channel_quads(const float* feat, int B, int C, int hw, f32x4* quads, hipStream_t s);

}  // namespace sfm
