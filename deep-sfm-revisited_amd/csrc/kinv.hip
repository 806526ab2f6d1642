// K^-1 for a batch of 3x3 float32 matrices, bit for bit what
// torch.inverse / torch.linalg.inv_ex return on this ROCm build, in one launch
// (torch's inv_ex: eleven launches, ~61 us per bench step).  SFMnet.forward
// takes intrinsic_inv_gpu = torch.inverse(intrinsic_gpu) (models/SFMnet.py:104).
//
// The operation order is rocsolver's getrf + getrs as torch drives them, found
// by git-history scripts/probe_kinv.hip (64 candidate orders against inv_ex on 20,000
// intrinsic and 20,000 general matrices; one matched every value): the
// row-major buffer is factored as its transpose M = A^T by LU with partial
// pivoting (first maximum |m|, whole rows swapped), multipliers m * (1 / pivot),
// rank-1 updates as one FMA each; then A x = e_k is solved as U^T y = e_k
// (column-oriented, dividing by the diagonal), L^T z = y (column-oriented,
// unit diagonal, separate multiply and subtract) and x = P^T z.  The kernel
// is built with -ffp-contract=off, so every other operation rounds on its own.
// tests/test_gpu_kinv.py compares every bit (signed zeros included) against
// torch.linalg.inv_ex on intrinsic matrices (with and without pivoting) and
// general ones.  A singular matrix gives inf / NaN entries where torch's
// inverse raises; the hot path only ever inverts camera intrinsics.
#include "common.h"

namespace sfm {

// zero / one arrive as kernel arguments: with compile-time constants the
// backend folds the solves' 0 - y into -y, which flips the sign of the exact
// zeros torch returns (+0 - +0 = +0, but -(+0) = -0)
__global__ void k_kinv3(const float* __restrict__ A, int batch, float* __restrict__ X, float zero, float one) {
  const int b = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (b >= batch) return;
  float M[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) M[r][c] = A[(size_t)b * 9 + c * 3 + r];   // M = A^T
  int piv[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    int p = j;
    float best = fabsf(M[j][j]);
#pragma unroll
    for (int r = j + 1; r < 3; ++r)
      if (fabsf(M[r][j]) > best) {
        best = fabsf(M[r][j]);
        p = r;
      }
    piv[j] = p;
#pragma unroll
    for (int r = j + 1; r < 3; ++r)          // swap rows j and p (branch-free: p >= j)
      if (r == p)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float t = M[j][c];
          M[j][c] = M[r][c];
          M[r][c] = t;
        }
    const float rd = one / M[j][j];
#pragma unroll
    for (int r = j + 1; r < 3; ++r) M[r][j] = M[r][j] * rd;
#pragma unroll
    for (int r = j + 1; r < 3; ++r)
#pragma unroll
      for (int c = j + 1; c < 3; ++c) M[r][c] = __builtin_fmaf(-M[r][j], M[j][c], M[r][c]);
  }
  float out[3][3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float x[3] = {k == 0 ? one : zero, k == 1 ? one : zero, k == 2 ? one : zero};
#pragma unroll
    for (int j = 0; j < 3; ++j) {             // U^T y = e_k
      x[j] = x[j] / M[j][j];
#pragma unroll
      for (int r = j + 1; r < 3; ++r) x[r] = x[r] - M[j][r] * x[j];
    }
#pragma unroll
    for (int j = 2; j >= 0; --j)              // L^T z = y
#pragma unroll
      for (int r = 0; r < j; ++r) x[r] = x[r] - M[j][r] * x[j];
#pragma unroll
    for (int j = 2; j >= 0; --j)              // x = P^T z
#pragma unroll
      for (int r = j + 1; r < 3; ++r)
        if (r == piv[j]) {
          const float t = x[j];
          x[j] = x[r];
          x[r] = t;
        }
#pragma unroll
    for (int r = 0; r < 3; ++r) out[r][k] = x[r];
  }
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) X[(size_t)b * 9 + r * 3 + c] = out[r][c];
}

}  // namespace sfm

using namespace sfm;

extern "C" int sfm_kinv3x3(const float* K, int batch, float* Kinv, void* stream) {
  SFM_REQUIRE(K && Kinv, "null pointer argument");
  SFM_REQUIRE(batch >= 1, "batch must be >= 1");
  hipLaunchKernelGGL(k_kinv3, dim3((unsigned)((batch + 63) / 64)), dim3(64), 0, (hipStream_t)stream, K, batch, Kinv,
                     0.0f, 1.0f);
  SFM_LAUNCHED();
  return SFM_OK;
}
