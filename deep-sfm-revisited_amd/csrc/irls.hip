// Batched robust refinement of E on the GPU: the IRLS
// of EssentialMatrixOptimise -> polish_E_robust_parametric (essential_matrix.cu:
// 76-105, polish_E.cu:1470-1577), which the reference runs on one CPU core.
//
// Per pair and iteration the work is a reduction over all N correspondences
// of the gradient g (5) and J^T W J (15 unique entries), then a 5x5 solve and
// five Givens updates of U, V.  Here:
//   k_irls_init    E -> (U, V) by the Givens decomposition (Edecomp)
//   k_irls_reduce  grid (blocks, pairs): per-block partial sums of the 20
//                  values in a fixed order (deterministic run to run)
//   k_irls_step    one block per pair: sums the partials in block order, the
//                  |g|^2 < 1e-20 stop, E = U diag(1,1,0) V^T, the MaxReps
//                  stop, gauss5 and the rotations — the reference's loop body
// The host launches (reduce, step) max_reps + 1 times; a per-pair done flag
// turns the remaining launches into no-ops.  The sums are reassociated
// relative to the reference's sequential loop, so E agrees to rounding level
// (tests: 1e-4 relative, the north-star bar), not bit for bit.
#include <string>
#include "common.h"

namespace sfm {

constexpr int kIrlsThreads = 256;
constexpr int kIrlsVals = 20;   // g[5], JtJ upper triangle [15]

struct IrlsState {
  double U[9], V[9], E[9];
  int done, rep;
};

__device__ void irls_decompose(double E[3][3], double U[3][3], double V[3][3]) {
  auto unit = [](double c, double s, double& oc, double& os) {
    const double r = sqrt(c * c + s * s);
    oc = c / r;
    os = s / r;
  };
  double zc, zs, yc, ys, xc, xs, uc, us, vc, vs;
  unit(E[0][0], -E[1][0], zc, zs);
  for (int j = 0; j < 3; ++j) {
    const double t = E[0][j] * zc - E[1][j] * zs;
    E[1][j] = E[0][j] * zs + E[1][j] * zc;
    E[0][j] = t;
  }
  unit(E[0][0], -E[2][0], yc, ys);
  for (int j = 0; j < 3; ++j) {
    const double t = E[0][j] * yc - E[2][j] * ys;
    E[2][j] = E[0][j] * ys + E[2][j] * yc;
    E[0][j] = t;
  }
  unit(E[1][1], -E[2][1], xc, xs);
  for (int j = 1; j < 3; ++j) E[1][j] = E[1][j] * xc - E[2][j] * xs;
  unit(E[1][1], -E[1][2], uc, us);
  E[0][2] = us * E[0][1] + uc * E[0][2];
  unit(E[0][0], -E[0][2], vc, vs);
  U[0][0] = yc * zc;  U[0][1] = -zc * xs * ys + xc * zs; U[0][2] = xc * zc * ys + xs * zs;
  U[1][0] = -yc * zs; U[1][1] = xc * zc + xs * ys * zs;  U[1][2] = zc * xs - xc * ys * zs;
  U[2][0] = -ys;      U[2][1] = -yc * xs;                U[2][2] = xc * yc;
  V[0][0] = vc;       V[0][1] = 0;                       V[0][2] = vs;
  V[1][0] = -us * vs; V[1][1] = uc;                      V[1][2] = vc * us;
  V[2][0] = -uc * vs; V[2][1] = -us;                     V[2][2] = uc * vc;
}

__global__ void k_irls_init(const double* __restrict__ E_init, int batch, IrlsState* __restrict__ st) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double E[3][3], U[3][3], V[3][3];
  for (int e = 0; e < 9; ++e) E[e / 3][e % 3] = E_init[b * 9 + e];
  irls_decompose(E, U, V);
  for (int e = 0; e < 9; ++e) {
    st[b].U[e] = U[e / 3][e % 3];
    st[b].V[e] = V[e / 3][e % 3];
    st[b].E[e] = E[e / 3][e % 3];   // the reference leaves E reduced in place
  }
  st[b].done = 0;
  st[b].rep = 0;
}

__global__ __launch_bounds__(kIrlsThreads) void k_irls_reduce(const double* __restrict__ pts, int64_t n_stride,
                                                              const int64_t* __restrict__ n_dev, double delta,
                                                              double alpha, const IrlsState* __restrict__ st,
                                                              double* __restrict__ partial) {
  const int b = blockIdx.y;
  if (st[b].done) return;
  __shared__ double s_red[kIrlsThreads / 64][kIrlsVals];
  double U[9], V[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) { U[e] = st[b].U[e]; V[e] = st[b].V[e]; }
  const int64_t n = n_dev[b];
  const double* P = pts + (size_t)b * n_stride * 4;
  double acc[kIrlsVals];
#pragma unroll
  for (int v = 0; v < kIrlsVals; ++v) acc[v] = 0.0;
  for (int64_t k = (int64_t)blockIdx.x * kIrlsThreads + threadIdx.x; k < n; k += (int64_t)gridDim.x * kIrlsThreads) {
    const double4 w4 = *reinterpret_cast<const double4*>(P + (size_t)k * 4);
    double p[3], q[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      p[j] = w4.x * V[j] + w4.y * V[3 + j] + 1.0 * V[6 + j];
      q[j] = w4.z * U[j] + w4.w * U[3 + j] + 1.0 * U[6 + j];
    }
    const double r = p[0] * q[0] + p[1] * q[1];
    const double W = (fabs(r) < delta) ? 1.0 : alpha * delta / fabs(r);
    const double J[5] = {-p[1] * q[2], -p[0] * q[2], p[1] * q[0] - p[0] * q[1], -p[2] * q[1], -p[2] * q[0]};
#pragma unroll
    for (int i = 0; i < 5; ++i) acc[i] += J[i] * -r * W;
    int t = 5;
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = i; j < 5; ++j) acc[t++] += W * J[i] * J[j];
  }
  // wave reduction (fixed butterfly order), then the block's waves in order
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int v = 0; v < kIrlsVals; ++v) {
    double x = acc[v];
    for (int o = 32; o; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) s_red[wv][v] = x;
  }
  __syncthreads();
  if (threadIdx.x < kIrlsVals) {
    double x = 0.0;
    for (int w = 0; w < kIrlsThreads / 64; ++w) x += s_red[w][threadIdx.x];
    partial[((size_t)b * gridDim.x + blockIdx.x) * kIrlsVals + threadIdx.x] = x;
  }
}

__device__ void irls_rotate_right(double M[3][3], int a, int c, double angle) {
  const double cs = cos(angle), sn = sin(angle);
  for (int i = 0; i < 3; ++i) {
    const double t = M[i][a] * cs - M[i][c] * sn;
    M[i][c] = M[i][a] * sn + M[i][c] * cs;
    M[i][a] = t;
  }
}

__global__ void k_irls_step(int nblk, int max_reps, const double* __restrict__ partial,
                            IrlsState* __restrict__ st) {
  const int b = blockIdx.x;
  if (st[b].done) return;
  __shared__ double s_sum[kIrlsVals];
  if (threadIdx.x < kIrlsVals) {
    double x = 0.0;
    for (int k = 0; k < nblk; ++k) x += partial[((size_t)b * nblk + k) * kIrlsVals + threadIdx.x];
    s_sum[threadIdx.x] = x;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  double g[5], mag = 0.0;
  for (int i = 0; i < 5; ++i) { g[i] = s_sum[i]; mag += g[i] * g[i]; }
  if (mag < 1e-20) { st[b].done = 1; return; }
  double U[3][3], V[3][3];
  for (int e = 0; e < 9; ++e) { U[e / 3][e % 3] = st[b].U[e]; V[e / 3][e % 3] = st[b].V[e]; }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) st[b].E[i * 3 + j] = U[i][0] * V[j][0] + U[i][1] * V[j][1];
  if (st[b].rep == max_reps) { st[b].done = 1; return; }
  double A[5][5];
  int t = 5;
  for (int i = 0; i < 5; ++i)
    for (int j = i; j < 5; ++j) { A[i][j] = s_sum[t]; A[j][i] = s_sum[t]; ++t; }
  // gauss5 (polish_E.cu:340-448): partial pivoting, back substitution
  for (int r = 0; r < 5; ++r) {
    int best = r;
    double mv = fabs(A[r][r]);
    for (int i = r + 1; i < 5; ++i)
      if (fabs(A[i][r]) > mv) { mv = fabs(A[i][r]); best = i; }
    if (best != r) {
      for (int j = r; j < 5; ++j) { const double tmp = A[r][j]; A[r][j] = A[best][j]; A[best][j] = tmp; }
      const double tb = g[r]; g[r] = g[best]; g[best] = tb;
    }
    for (int i = r + 1; i < 5; ++i) {
      const double f = A[i][r] / A[r][r];
      for (int j = r + 1; j < 5; ++j) A[i][j] -= f * A[r][j];
      g[i] -= f * g[r];
    }
  }
  for (int i = 4; i >= 0; --i) {
    for (int j = i + 1; j < 5; ++j) g[i] -= A[i][j] * g[j];
    g[i] /= A[i][i];
  }
  irls_rotate_right(U, 0, 1, g[2]);
  irls_rotate_right(U, 0, 2, g[1]);
  irls_rotate_right(U, 1, 2, g[0]);
  irls_rotate_right(V, 1, 2, g[3]);
  irls_rotate_right(V, 0, 2, g[4]);
  for (int e = 0; e < 9; ++e) { st[b].U[e] = U[e / 3][e % 3]; st[b].V[e] = V[e / 3][e % 3]; }
  st[b].rep += 1;
}

__global__ void k_irls_out(int batch, const IrlsState* __restrict__ st, double* __restrict__ E_out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < batch * 9) E_out[i] = st[i / 9].E[i % 9];
}

static int irls_blocks(int64_t n_max) {
  const int64_t per = (int64_t)kIrlsThreads * 16;                // ~16 points per thread
  return (int)std::max<int64_t>(1, std::min<int64_t>(256, (n_max + per - 1) / per));
}

static size_t irls_ws_bytes(int batch, int64_t n_max) {
  const size_t st = ((size_t)batch * sizeof(IrlsState) + 255) & ~(size_t)255;
  const size_t part = (size_t)batch * irls_blocks(n_max) * kIrlsVals * sizeof(double);
  const size_t nn = (size_t)batch * sizeof(int64_t);
  return st + ((part + 255) & ~(size_t)255) + nn;
}

}  // namespace sfm

using namespace sfm;

extern "C" {

size_t sfm_essential_optimise_workspace_bytes(int batch, int64_t n_max) {
  if (batch < 1 || n_max < 0) return 0;
  return irls_ws_bytes(batch, n_max);
}

int sfm_essential_optimise_batched(const double* pts, int64_t n_stride, const int64_t* n, int batch,
                                   const double* E_init, double delta, double alpha, int max_reps, double* E_out,
                                   void* workspace, size_t workspace_bytes, void* stream) {
  SFM_REQUIRE(pts && n && E_init && E_out, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && batch <= 65535 && n_stride >= 0, "invalid batch");
  SFM_REQUIRE(max_reps >= 0 && max_reps <= (1 << 20), "max_reps out of range");
  int64_t n_max = 0;
  for (int b = 0; b < batch; ++b) {
    SFM_REQUIRE(n[b] >= 0 && n[b] <= n_stride, "point count out of range");
    n_max = std::max(n_max, n[b]);
  }
  const size_t need = irls_ws_bytes(batch, n_stride);
  if (!workspace || workspace_bytes < need) {
    set_error("optimise workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  hipStream_t s = (hipStream_t)stream;
  const int nblk = irls_blocks(n_stride);
  char* base = (char*)workspace;
  IrlsState* st = (IrlsState*)base;
  base += ((size_t)batch * sizeof(IrlsState) + 255) & ~(size_t)255;
  double* partial = (double*)base;
  base += (((size_t)batch * nblk * kIrlsVals * sizeof(double)) + 255) & ~(size_t)255;
  int64_t* n_dev = (int64_t*)base;
  SFM_HIP(hipMemcpyAsync(n_dev, n, (size_t)batch * sizeof(int64_t), hipMemcpyHostToDevice, s));
  ProfScope ps("essential_optimise", s);
  hipLaunchKernelGGL(k_irls_init, dim3((batch + 63) / 64), dim3(64), 0, s, E_init, batch, st);
  for (int it = 0; it <= max_reps; ++it) {
    hipLaunchKernelGGL(k_irls_reduce, dim3(nblk, batch), dim3(kIrlsThreads), 0, s, pts, n_stride, n_dev, delta,
                       alpha, st, partial);
    hipLaunchKernelGGL(k_irls_step, dim3(batch), dim3(64), 0, s, nblk, max_reps, partial, st);
  }
  hipLaunchKernelGGL(k_irls_out, dim3((batch * 9 + 255) / 256), dim3(256), 0, s, batch, st, E_out);
  SFM_LAUNCHED();
  return SFM_OK;
}

}  // extern "C"
