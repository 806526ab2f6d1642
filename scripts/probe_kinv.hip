// Probe (round 3): which float32 operation order reproduces torch.linalg.inv_ex
// (rocsolver getrf + getrs on ROCm) bit for bit on 3x3 matrices.  Every
// variant runs LU with partial pivoting (first maximum |a|), then the two
// triangular solves against the identity, for one batch of matrices.
// mode bits:
//   1   factor A^T (row-major buffer read as column-major) and solve with the
//       transposes (nonunit forward U^T, unit backward L^T, pivots last);
//       else factor A, pivots first, unit forward L, nonunit backward U
//   2   multipliers l = a * (1 / pivot) instead of a / pivot
//   4   fma in the rank-1 updates (a - l * u as one rounding)
//   8   nonunit solve: multiply by 1 / diagonal instead of dividing
//  16   fma in the substitutions
//  32   substitutions column-oriented (axpy, x_j finished first) instead of row-oriented (dot)
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC -o probe_kinv.so probe_kinv.hip
#include <hip/hip_runtime.h>
#include <cmath>

__device__ __forceinline__ float sub_mul(float a, float l, float u, bool f) {
  return f ? __builtin_fmaf(-l, u, a) : a - l * u;
}

__global__ void k_kinv_probe(const float* __restrict__ A, int B, int nmode, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * nmode) return;
  const int b = i / nmode, mode = i % nmode;
  const bool tr = mode & 1, rcpm = mode & 2, fu = mode & 4, rcps = mode & 8, fs = mode & 16, col = mode & 32;
  float M[3][3];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) M[r][c] = tr ? A[b * 9 + c * 3 + r] : A[b * 9 + r * 3 + c];
  int piv[3] = {0, 1, 2};
  for (int j = 0; j < 3; ++j) {
    int p = j;
    float best = fabsf(M[j][j]);
    for (int r = j + 1; r < 3; ++r)
      if (fabsf(M[r][j]) > best) { best = fabsf(M[r][j]); p = r; }
    piv[j] = p;
    if (p != j)
      for (int c = 0; c < 3; ++c) { const float t = M[j][c]; M[j][c] = M[p][c]; M[p][c] = t; }
    const float d = M[j][j];
    const float rd = 1.0f / d;
    for (int r = j + 1; r < 3; ++r) M[r][j] = rcpm ? M[r][j] * rd : M[r][j] / d;
    for (int r = j + 1; r < 3; ++r)
      for (int c = j + 1; c < 3; ++c) M[r][c] = sub_mul(M[r][c], M[r][j], M[j][c], fu);
  }
  float X[3][3];   // X[row][col] of the solution, column k solves for e_k
  for (int k = 0; k < 3; ++k) {
    float x[3] = {k == 0 ? 1.0f : 0.0f, k == 1 ? 1.0f : 0.0f, k == 2 ? 1.0f : 0.0f};
    if (!tr) {
      for (int j = 0; j < 3; ++j)
        if (piv[j] != j) { const float t = x[j]; x[j] = x[piv[j]]; x[piv[j]] = t; }
      // L y = x (unit lower)
      if (col) {
        for (int j = 0; j < 3; ++j)
          for (int r = j + 1; r < 3; ++r) x[r] = sub_mul(x[r], M[r][j], x[j], fs);
      } else {
        for (int r = 1; r < 3; ++r)
          for (int j = 0; j < r; ++j) x[r] = sub_mul(x[r], M[r][j], x[j], fs);
      }
      // U z = y (nonunit upper)
      if (col) {
        for (int j = 2; j >= 0; --j) {
          x[j] = rcps ? x[j] * (1.0f / M[j][j]) : x[j] / M[j][j];
          for (int r = 0; r < j; ++r) x[r] = sub_mul(x[r], M[r][j], x[j], fs);
        }
      } else {
        for (int r = 2; r >= 0; --r) {
          for (int j = r + 1; j < 3; ++j) x[r] = sub_mul(x[r], M[r][j], x[j], fs);
          x[r] = rcps ? x[r] * (1.0f / M[r][r]) : x[r] / M[r][r];
        }
      }
    } else {
      // A = M^T = (P L U)^T: U^T y = x (nonunit lower), L^T z = y (unit upper), then P
      if (col) {
        for (int j = 0; j < 3; ++j) {
          x[j] = rcps ? x[j] * (1.0f / M[j][j]) : x[j] / M[j][j];
          for (int r = j + 1; r < 3; ++r) x[r] = sub_mul(x[r], M[j][r], x[j], fs);
        }
        for (int j = 2; j >= 0; --j)
          for (int r = 0; r < j; ++r) x[r] = sub_mul(x[r], M[j][r], x[j], fs);
      } else {
        for (int r = 0; r < 3; ++r) {
          for (int j = 0; j < r; ++j) x[r] = sub_mul(x[r], M[j][r], x[j], fs);
          x[r] = rcps ? x[r] * (1.0f / M[r][r]) : x[r] / M[r][r];
        }
        for (int r = 1; r >= 0; --r)
          for (int j = r + 1; j < 3; ++j) x[r] = sub_mul(x[r], M[j][r], x[j], fs);
      }
      for (int j = 2; j >= 0; --j)
        if (piv[j] != j) { const float t = x[j]; x[j] = x[piv[j]]; x[piv[j]] = t; }
    }
    for (int r = 0; r < 3; ++r) X[r][k] = x[r];
  }
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) out[((size_t)mode * B + b) * 9 + r * 3 + c] = X[r][c];
}

extern "C" int probe_kinv(const float* A, int B, int nmode, float* out) {
  const int n = B * nmode;
  hipLaunchKernelGGL(k_kinv_probe, dim3((n + 255) / 256), dim3(256), 0, 0, A, B, nmode, out);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
