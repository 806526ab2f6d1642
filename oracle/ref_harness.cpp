// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libref_ransac.so).
//
// Compiles the REFERENCE's own five-point solver, Sturm root finder,
// cheirality test and IRLS polish (RANSAC_FiveP/essential_matrix/*.cu, read in
// place from /root/reference via -I, host-compiled with
// -D__host__= -D__device__=, mirroring the single translation unit that the
// reference's kernel_functions.cu / essential_matrix.cu form) and exposes them
// through a small C ABI.  The CUDA kernel loop of EstimateProjectionMatrix<5>
// (kernel_functions.cu:141-226) and ComputeError (232-264) cannot be compiled
// here (cuRAND, __global__, __constant__), so they are restated below around
// the reference solver functions, with the build's specified sampler.
//
// No reference source is copied into this repository; see oracle/Makefile.
// ============================================================================
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>
#include <algorithm>
#include <iostream>

// The reference's translation unit, in the order kernel_functions.cu and
// essential_matrix.cu include it.
#include "common.h"
#include "polish_E.cu"
#include "polydet.cu"
#include "sturm.cu"
#include "polyquotient.cu"
#include "cheirality.cu"
#include "essential_matrix_5pt.cu"

namespace refh {

static inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += W0; k1 += W1; }
    uint64_t p0 = (uint64_t)M0 * c[0];
    uint64_t p1 = (uint64_t)M1 * c[2];
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
  }
}

static inline int64_t sample_index(uint64_t seed, uint32_t h, uint32_t d, int64_t n) {
  uint32_t c[4] = {h, d >> 2, 0u, 0u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  float u = (float)c[d & 3] * 2.3283064e-10f;
  u = u + 2.3283064e-10f / 2.0f;
  float r = u * ((float)(int)(n - 1) + 0.999999f);
  r = r + 0.0f;
  int64_t idx = (int64_t)truncf(r);
  if (idx > n - 1) idx = n - 1;
  if (idx < 0) idx = 0;
  return idx;
}

// ComputeError<double> (kernel_functions.cu:232-264), restated.
static inline bool inlier(const Ematrix& E, const double* q, const double* qp, double thr) {
  double Ex[3], xE[3];
  for (int k = 0; k < 3; k++) { double s = 0.0; for (int l = 0; l < 3; l++) s += E[k][l] * q[l]; Ex[k] = s; }
  for (int k = 0; k < 3; k++) { double s = 0.0; for (int l = 0; l < 3; l++) s += qp[l] * E[l][k]; xE[k] = s; }
  double xEx = 0.0;
  for (int k = 0; k < 3; k++) xEx += qp[k] * Ex[k];
  double d = sqrt(Ex[0] * Ex[0] + Ex[1] * Ex[1] + xE[0] * xE[0] + xE[1] * xE[1]);
  double e = xEx / d;
  if (e < 0.0) e = -e;
  return e <= thr;
}

static int count(const Ematrix& E, const double* qs, const double* qps, int64_t n, double thr) {
  int c = 0;
  for (int64_t k = 0; k < n; ++k) {
    double a[3] = {qs[2 * k], qs[2 * k + 1], 1.0}, b[3] = {qps[2 * k], qps[2 * k + 1], 1.0};
    if (inlier(E, a, b, thr)) ++c;
  }
  return c;
}

}  // namespace refh

extern "C" {

// compute_E_matrices_optimized + compute_P_matrices on explicit 5 matches.
int ref_solve5(const double* q5, const double* qp5, int cheir,
               double* E_roots, int* nroots, double* E_out, double* P_out, int* nP) {
  double q[5][3], qp[5][3];
  for (int i = 0; i < 5; ++i) {
    q[i][0] = q5[2 * i]; q[i][1] = q5[2 * i + 1]; q[i][2] = 1.0;
    qp[i][0] = qp5[2 * i]; qp[i][1] = qp5[2 * i + 1]; qp[i][2] = 1.0;
  }
  Ematrix Es[10];
  Pmatrix Ps[10];
  memset(Es, 0, sizeof(Es));
  memset(Ps, 0, sizeof(Ps));
  int nr = 0;
  compute_E_matrices_optimized(q, qp, Es, nr);
  *nroots = nr;
  if (E_roots) memcpy(E_roots, Es, sizeof(Es));
  int np = nr;
  if (cheir) compute_P_matrices(q, qp, Es, (double*)0, Ps, np, 5);
  if (nP) *nP = cheir ? np : 0;
  if (E_out) memcpy(E_out, Es, sizeof(Es));
  if (P_out) memcpy(P_out, Ps, sizeof(Ps));
  return 0;
}

// EstimateProjectionMatrix<5> / EstimateEssentialMatrix<5> loop restated
// around the reference solver; same canonical slot rules as the oracle.
int ref_ransac5(const double* q, const double* qp, int64_t n, int num_test, int num_ransac_test,
                int nchains, int iters, double thr, uint64_t seed, int cheir,
                double* E_out, double* P_out, int* inliers_out, int* winner_out,
                int* hyp_score, int* hyp_ncand) {
  if (n < 1 || num_test > n || num_ransac_test > n) return 1;
  const int H = nchains * iters;
  std::vector<int> score(H, 0);
  std::vector<double> Ew((size_t)H * 9, 0.0), Pw((size_t)H * 12, 0.0);
  for (int t = 0; t < nchains; ++t) {
    Ematrix Eset[10];
    Pmatrix Pset[10];
    memset(Eset, 0, sizeof(Eset));
    memset(Pset, 0, sizeof(Pset));
    for (int i = 0; i < iters; ++i) {
      const int h = t * iters + i;
      double qs[5][3], qps[5][3];
      for (int d = 0; d < 5; ++d) {
        int64_t idx = refh::sample_index(seed, (uint32_t)h, (uint32_t)d, n);
        qs[d][0] = q[2 * idx]; qs[d][1] = q[2 * idx + 1]; qs[d][2] = 1.0;
        qps[d][0] = qp[2 * idx]; qps[d][1] = qp[2 * idx + 1]; qps[d][2] = 1.0;
      }
      int nE = 0;
      compute_E_matrices_optimized(qs, qps, Eset, nE);
      int nc = nE;
      if (cheir) compute_P_matrices(qs, qps, Eset, (double*)0, Pset, nc, 5);
      if (hyp_ncand) hyp_ncand[h] = nc > 0 ? nc : 0;
      int bc = 0, bi = 0;
      for (int j = 0; j < nc; ++j) {
        int c = refh::count(Eset[j], q, qp, num_test, thr);
        if (c > bc) { bc = c; bi = j; }
      }
      score[h] = refh::count(Eset[bi], q, qp, num_ransac_test, thr);
      memcpy(&Ew[(size_t)h * 9], Eset[bi], sizeof(Ematrix));
      memcpy(&Pw[(size_t)h * 12], Pset[bi], sizeof(Pmatrix));
    }
  }
  int win = -1, wb = 0;
  for (int t = 0; t < nchains; ++t) {
    int tb = 0, th = -1;
    for (int i = 0; i < iters; ++i) { int h = t * iters + i; if (score[h] > tb) { tb = score[h]; th = h; } }
    if (tb > wb) { wb = tb; win = th; }
  }
  if (win >= 0) {
    memcpy(E_out, &Ew[(size_t)win * 9], 9 * sizeof(double));
    memcpy(P_out, &Pw[(size_t)win * 12], 12 * sizeof(double));
  } else {
    memset(E_out, 0, 9 * sizeof(double));
    memset(P_out, 0, 12 * sizeof(double));
  }
  *inliers_out = wb;
  if (winner_out) *winner_out = win;
  if (hyp_score) memcpy(hyp_score, score.data(), sizeof(int) * H);
  return 0;
}

// Edecomp(E, parameters) (polish_E.cu:247-338)
void ref_decompose(const double* E_in, double* params) {
  Ematrix E;
  memcpy(E, E_in, sizeof(E));
  Edecomp(E, params);
}

// Edecomp(E, U, V) (polish_E.cu:147-244)
void ref_decompose_uv(const double* E_in, double* U_out, double* V_out) {
  Ematrix E, U, V;
  memcpy(E, E_in, sizeof(E));
  Edecomp(E, U, V);
  memcpy(U_out, U, sizeof(U));
  memcpy(V_out, V, sizeof(V));
}

// polish_E_robust_parametric (polish_E.cu:1470-1577)
void ref_optimise(const double* pin, const double* qin, int64_t n, const double* E_init,
                  double delta, double alpha, int max_reps, double* E_out) {
  Ematrix E;
  memcpy(E, E_init, sizeof(E));
  polish_E_robust_parametric(E, pin, qin, (int)n, delta, alpha, max_reps);
  memcpy(E_out, E, sizeof(E));
}

}  // extern "C"
