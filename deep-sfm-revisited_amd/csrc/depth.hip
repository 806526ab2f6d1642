// Depth stage after the plane sweep on CDNA4 (gfx950): SURVEY.md §8(f) row 1.
//
//   k_sweep_corr   parameter-free correlation cost of REG2D.py:103-109:
//                  cost[b, i] = mean_c(ref[b, c] * inverse_warp(tgt, d_i)[b, c])
//                  computed straight from the sweep arithmetic (warp.h), without
//                  materialising the [B, C, L, h, w] warped volume.
//   k_depth_head   soft-argmin head of PSNet.py:191-213: trilinear upsample of
//                  the [B, L, h, w] cost to [L, H, W] (align_corners=False; the
//                  plane axis keeps its size, so it is an identity), softmax over
//                  planes, disparityregression (sum p_i (i+1)) -> depth =
//                  MIN_DEPTH L / (disp + 1e-16), or depthregression
//                  (sum p_i (i+1) step) * MIN_DEPTH under cfg.PREDICT_BY_DEPTH
//                  (submodule.py:57-93).
//
// Both are light: the correlation cost is gather-bound (4 taps x C/4 float4
// loads per pixel and plane, from L2), the head reads the low-resolution cost
// from L2 (15 MB per KITTI pair at L=128) and writes 4 bytes per output pixel.
#include <string>
#include "warp.h"

namespace sfm {

constexpr int kCorrThreads = 256;
constexpr int kCorrPlanes = 8;       // planes per thread (ref quad loads amortised through L1)
constexpr int kHeadThreads = 256;

// grid (ceil(hw / 256), ceil(L / kCorrPlanes), B); thread = pixel
__global__ __launch_bounds__(kCorrThreads) void k_sweep_corr(const f32x4* __restrict__ rq, const f32x4* __restrict__ tq,
                                                             int C, int h, int w, const float* __restrict__ pose,
                                                             const float* __restrict__ K4,
                                                             const float* __restrict__ K4inv, int L, float dmax,
                                                             float dstep, float* __restrict__ out) {
  const int b = blockIdx.z;
  const int hw = h * w;
  const int p = blockIdx.x * kCorrThreads + threadIdx.x;
  if (p >= hw) return;
  const int C4 = (C + 3) / 4;
  Proj pr;
  load_proj(pose, K4, K4inv, b, pr);
  const float x = (float)(p % w), y = (float)(p / w);
  float ray[3];
  ray[0] = (pr.ki[0] * x + pr.ki[1] * y) + pr.ki[2];
  ray[1] = (pr.ki[3] * x + pr.ki[4] * y) + pr.ki[5];
  ray[2] = (pr.ki[6] * x + pr.ki[7] * y) + pr.ki[8];
  const f32x4* R = rq + (size_t)b * C4 * hw + p;
  const f32x4* T = tq + (size_t)b * C4 * hw;
  const int l0 = blockIdx.y * kCorrPlanes;
  const int l1 = min(L, l0 + kCorrPlanes);
  for (int l = l0; l < l1; ++l) {
    // PSNet.py:150-153 / REG2D.py:105: disp2depth / (i+1), or (i+1) MIN_DEPTH
    const float d = dstep > 0.0f ? (float)(l + 1) * dstep : dmax / (float)(l + 1);
    float ix, iy;
    float acc = 0.0f;
    if (sample_pos(pr, ray, d, h, w, ix, iy)) {
      Taps tp;
      make_taps(ix, iy, h, w, tp);
      for (int q = 0; q < C4; ++q) {
        const f32x4* Tq = T + (size_t)q * hw;
        const f32x4 t0 = Tq[tp.off[0]], t1 = Tq[tp.off[1]], t2 = Tq[tp.off[2]], t3 = Tq[tp.off[3]];
        f32x4 wv = tp.wt[0] * t0;
        wv = wv + tp.wt[1] * t1;
        wv = wv + tp.wt[2] * t2;
        wv = wv + tp.wt[3] * t3;
        const f32x4 r = R[(size_t)q * hw];
        // channels c >= C are zero in both quads; ascending channel order
        acc = acc + r[0] * wv[0];
        acc = acc + r[1] * wv[1];
        acc = acc + r[2] * wv[2];
        acc = acc + r[3] * wv[3];
      }
    }
    // outside the image the warped features are 0, so the product is 0
    out[((size_t)b * L + l) * hw + p] = acc / (float)C;
  }
}

struct HeadTaps {
  int o00, o01, o10, o11;
  float wx0, wx1, wy0, wy1;
};

// F.interpolate(..., mode='trilinear', align_corners=False) source index and
// weights along one axis (PyTorch's area_pixel_compute_source_index with
// guard_index_and_lambda; identity when the sizes match)
__device__ __forceinline__ void axis_weights(int dst, int in_size, int out_size, float ratio, int& i0, int& i1,
                                             float& l0, float& l1) {
  if (in_size == out_size) {
    i0 = i1 = dst;
    l0 = 1.0f;
    l1 = 0.0f;
    return;
  }
  float src = ratio * ((float)dst + 0.5f) - 0.5f;
  if (src < 0.0f) src = 0.0f;
  i0 = min((int)floorf(src), in_size - 1);
  l1 = fminf(fmaxf(src - (float)i0, 0.0f), 1.0f);
  i1 = i0 + (i0 < in_size - 1 ? 1 : 0);
  l0 = 1.0f - l1;
}

// interpolated cost of plane l (PyTorch's nested order: ((x00 wx0 + x01 wx1) wy0 + (x10 wx0 + x11 wx1) wy1))
__device__ __forceinline__ float head_value(const float* __restrict__ plane, const HeadTaps& t) {
  const float r0 = plane[t.o00] * t.wx0 + plane[t.o01] * t.wx1;
  const float r1 = plane[t.o10] * t.wx0 + plane[t.o11] * t.wx1;
  return r0 * t.wy0 + r1 * t.wy1;
}

// grid (ceil(W / 256), H, B); thread = output pixel
__global__ __launch_bounds__(kHeadThreads) void k_depth_head(const float* __restrict__ cost, int L, int h, int w,
                                                             int H, int W, float ratio_h, float ratio_w,
                                                             int depth_mode, float min_depth, float step,
                                                             float* __restrict__ depth) {
  const int b = blockIdx.z, Y = blockIdx.y;
  const int X = blockIdx.x * kHeadThreads + threadIdx.x;
  if (X >= W) return;
  HeadTaps t;
  int y0, y1, x0, x1;
  axis_weights(Y, h, H, ratio_h, y0, y1, t.wy0, t.wy1);
  axis_weights(X, w, W, ratio_w, x0, x1, t.wx0, t.wx1);
  t.o00 = y0 * w + x0; t.o01 = y0 * w + x1;
  t.o10 = y1 * w + x0; t.o11 = y1 * w + x1;
  const size_t hw = (size_t)h * w;
  const float* cb = cost + (size_t)b * L * hw;
  // softmax over planes (max, then exp(v - max)), then the weighted sum
  float m = -INFINITY;
  for (int l = 0; l < L; ++l) m = fmaxf(m, head_value(cb + l * hw, t));
  float s = 0.0f, ws = 0.0f;
  for (int l = 0; l < L; ++l) {
    const float e = expf(head_value(cb + l * hw, t) - m);
    s = s + e;
    ws = ws + e * ((float)(l + 1) * step);
  }
  const float reg = ws * (1.0f / s);      // sum_i p_i v_i with p_i = e_i * (1/s)
  float out;
  if (depth_mode) out = reg * min_depth;                          // PSNet.py:209-210
  else out = (min_depth * (float)L) / (reg + 1e-16f);             // PSNet.py:212-213
  depth[((size_t)b * H + Y) * W + X] = out;
}

static size_t corr_ws_bytes(int B, int C, int h, int w) {
  const size_t quads = (size_t)B * ((C + 3) / 4) * h * w * sizeof(f32x4);
  return 2 * ((quads + 255) & ~(size_t)255);
}

// Flow2Depth (models/flow2depth.py:7-41; dead code in the reference, kept
// for the API).  vec_p = (K R) dir_p + K T with dir_p = float32(Ki (j, i, 1))
// formed in float64 as numpy does (float32 Ki times int64 pixel -> float64).
// The reference views the [B, H*W, 3] result as [B, 3, H, W] and returns
// channel 2, i.e. flat element 2HW + k of each batch's buffer: out[b, k] =
// vec_p[c] with p = (2HW + k) / 3, c = (2HW + k) % 3.
constexpr int kF2DThreads = 256;
__global__ __launch_bounds__(kF2DThreads) void k_flow2depth(const float* __restrict__ KR, const float* __restrict__ KT,
                                                            const float* __restrict__ Ki, int H, int W,
                                                            float* __restrict__ out) {
  const int b = blockIdx.y;
  const int64_t hw = (int64_t)H * W;
  const int64_t k = (int64_t)blockIdx.x * kF2DThreads + threadIdx.x;
  if (k >= hw) return;
  const int64_t f = 2 * hw + k;
  const int64_t p = f / 3;
  const int c = (int)(f - 3 * p);
  const int i = (int)(p / W), j = (int)(p - (int64_t)i * W);
  const float* ki = Ki + 9 * b;
  float dir[3];
  for (int r = 0; r < 3; ++r)
    dir[r] = (float)(((double)ki[3 * r] * (double)j + (double)ki[3 * r + 1] * (double)i) + (double)ki[3 * r + 2]);
  const float* kr = KR + 9 * b + 3 * c;
  const float first = (kr[0] * dir[0] + kr[1] * dir[1]) + kr[2] * dir[2];
  out[b * hw + k] = first + KT[3 * b + c];
}

}  // namespace sfm

using namespace sfm;

extern "C" {

size_t sfm_correlation_workspace_bytes(int batch, int channels, int h, int w) {
  if (batch < 1 || channels < 1 || h < 1 || w < 1) return 0;
  return corr_ws_bytes(batch, channels, h, w);
}

int sfm_plane_sweep_correlation(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                                const float* pose, const float* K4, const float* K4inv, int nlabel, float min_depth,
                                int depth_mode, float* cost, void* workspace, size_t workspace_bytes,
                                void* stream) {
  SFM_REQUIRE(ref && tgt && pose && K4 && K4inv && cost, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && batch <= 65535 && channels >= 1 && channels <= 4 * 65535 && h >= 2 && w >= 2 &&
              nlabel >= 1, "invalid correlation shape");
  SFM_REQUIRE(depth_mode == 0 || depth_mode == 1, "depth_mode must be 0 (inverse depth) or 1 (depth)");
  SFM_REQUIRE(min_depth > 0.0f, "min_depth must be positive");
  SFM_REQUIRE((int64_t)h * w < ((int64_t)1 << 30), "feature map too large");
  const size_t need = corr_ws_bytes(batch, channels, h, w);
  if (!workspace || workspace_bytes < need) {
    set_error("correlation workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  const int hw = h * w;
  hipStream_t s = (hipStream_t)stream;
  f32x4* rq = (f32x4*)workspace;
  f32x4* tq = (f32x4*)((char*)workspace + need / 2);
  {
    ProfScope ps("corr_quads", s);
    launch_channel_quads(ref, batch, channels, hw, rq, s);
    launch_channel_quads(tgt, batch, channels, hw, tq, s);
  }
  SFM_LAUNCHED();
  ProfScope ps("sweep_correlation", s);
  const float dmax = min_depth * (float)nlabel;
  const float dstep = depth_mode ? min_depth : 0.0f;
  hipLaunchKernelGGL(k_sweep_corr, dim3((hw + kCorrThreads - 1) / kCorrThreads, (nlabel + kCorrPlanes - 1) / kCorrPlanes,
                                        batch),
                     dim3(kCorrThreads), 0, s, rq, tq, channels, h, w, pose, K4, K4inv, nlabel, dmax, dstep, cost);
  SFM_LAUNCHED();
  return SFM_OK;
}

int sfm_depth_head(const float* cost, int batch, int nlabel, int h, int w, int H, int W, int depth_mode,
                   float min_depth, float depth_step, float* depth, void* stream) {
  SFM_REQUIRE(cost && depth, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && batch <= 65535 && nlabel >= 1 && h >= 1 && w >= 1 && H >= 1 && W >= 1 && H <= 65535,
              "invalid depth-head shape");
  SFM_REQUIRE(depth_mode == 0 || depth_mode == 1, "depth_mode must be 0 (disparity) or 1 (depth)");
  SFM_REQUIRE(depth_mode == 0 || depth_step > 0.0f, "depth regression needs a positive step");
  SFM_REQUIRE((int64_t)nlabel * h * w < ((int64_t)1 << 31), "cost volume too large");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps("depth_head", s);
  // area_pixel_compute_scale: (float)input_size / output_size
  const float ratio_h = (float)h / (float)H, ratio_w = (float)w / (float)W;
  hipLaunchKernelGGL(k_depth_head, dim3((W + kHeadThreads - 1) / kHeadThreads, H, batch), dim3(kHeadThreads), 0, s,
                     cost, nlabel, h, w, H, W, ratio_h, ratio_w, depth_mode, min_depth,
                     depth_mode ? depth_step : 1.0f, depth);
  SFM_LAUNCHED();
  return SFM_OK;
}

}  // extern "C"

extern "C" int sfm_flow2depth(const float* KR, const float* KT, const float* Kinv, int batch, int H, int W, float* out,
                              void* stream) {
  SFM_REQUIRE(KR && KT && Kinv && out, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && batch <= 65535 && H >= 1 && W >= 1 && (int64_t)H * W < ((int64_t)1 << 31) / 3,
              "invalid flow2depth shape");
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps("flow2depth", s);
  const int64_t hw = (int64_t)H * W;
  hipLaunchKernelGGL(k_flow2depth, dim3((unsigned)((hw + kF2DThreads - 1) / kF2DThreads), batch), dim3(kF2DThreads), 0,
                     s, KR, KT, Kinv, H, W, out);
  SFM_LAUNCHED();
  return SFM_OK;
}
