// Host-side essential-matrix utilities of the `essential_matrix` extension:
// the reference runs `optimise`, `decompose` and `decomposeUV` on CPU tensors
// (essential_matrix.cu:29-105 -> polish_E.cu), so they stay host C++ here.
//
//   Edecomp     polish_E.cu:147-338   E = U . diag(1,1,0) . V^T via five Givens
//                                     rotations (angles x, y, z, u, v)
//   IRLS        polish_E.cu:1470-1577 robust (truncated-L2 .. Huber) refinement
//                                     on the 5-parameter manifold
//   solve_5x5   polish_E.cu:340-448   partial-pivot Gaussian elimination
//   update      polish_E.cu:450-472   U <- U Rz Ry Rx, V <- V Ru Rv
//
// Compiled with -ffp-contract=off; results are bit-identical to the
// reference's host code on the same libm.
#include <cmath>
#include <cstring>
#include <vector>
#include <utility>
#include "common.h"

namespace sfm {
namespace {

struct Givens { double c, s; };

struct Decomp {
  Givens x, y, z, u, v;
};

// Left rotations eliminate E[1][0], E[2][0], E[2][1]; right rotations
// E[1][2], E[0][2].  E is modified in place (as the reference does).
Decomp givens_decompose(double E[3][3]) {
  Decomp d;
  auto unit = [](double c, double s) {
    const double r = sqrt(c * c + s * s);
    return Givens{c / r, s / r};
  };
  d.z = unit(E[0][0], -E[1][0]);
  for (int j = 0; j < 3; ++j) {
    const double t = E[0][j] * d.z.c - E[1][j] * d.z.s;
    E[1][j] = E[0][j] * d.z.s + E[1][j] * d.z.c;
    E[0][j] = t;
  }
  d.y = unit(E[0][0], -E[2][0]);
  for (int j = 0; j < 3; ++j) {
    const double t = E[0][j] * d.y.c - E[2][j] * d.y.s;
    E[2][j] = E[0][j] * d.y.s + E[2][j] * d.y.c;
    E[0][j] = t;
  }
  d.x = unit(E[1][1], -E[2][1]);
  for (int j = 1; j < 3; ++j) E[1][j] = E[1][j] * d.x.c - E[2][j] * d.x.s;
  d.u = unit(E[1][1], -E[1][2]);
  E[0][2] = d.u.s * E[0][1] + d.u.c * E[0][2];
  d.v = unit(E[0][0], -E[0][2]);
  return d;
}

void uv_from(const Decomp& d, double U[3][3], double V[3][3]) {
  const double cx = d.x.c, sx = d.x.s, cy = d.y.c, sy = d.y.s, cz = d.z.c, sz = d.z.s;
  const double cu = d.u.c, su = d.u.s, cv = d.v.c, sv = d.v.s;
  U[0][0] = cy * cz;  U[0][1] = -cz * sx * sy + cx * sz; U[0][2] = cx * cz * sy + sx * sz;
  U[1][0] = -cy * sz; U[1][1] = cx * cz + sx * sy * sz;  U[1][2] = cz * sx - cx * sy * sz;
  U[2][0] = -sy;      U[2][1] = -cy * sx;                U[2][2] = cx * cy;
  V[0][0] = cv;       V[0][1] = 0;                       V[0][2] = sv;
  V[1][0] = -su * sv; V[1][1] = cu;                      V[1][2] = cv * su;
  V[2][0] = -cu * sv; V[2][1] = -su;                     V[2][2] = cu * cv;
}

// M <- M . G^T for the Givens rotation of columns (a, b) by angle
void rotate_right(double M[3][3], int a, int b, double angle) {
  const double c = cos(angle), s = sin(angle);
  for (int i = 0; i < 3; ++i) {
    const double t = M[i][a] * c - M[i][b] * s;
    M[i][b] = M[i][a] * s + M[i][b] * c;
    M[i][a] = t;
  }
}

void gauss5(double A[5][5], double b[5]) {
  for (int r = 0; r < 5; ++r) {
    int best = r;
    double mv = fabs(A[r][r]);
    for (int i = r + 1; i < 5; ++i)
      if (fabs(A[i][r]) > mv) { mv = fabs(A[i][r]); best = i; }
    if (best != r) {
      for (int j = r; j < 5; ++j) std::swap(A[r][j], A[best][j]);
      std::swap(b[r], b[best]);
    }
    for (int i = r + 1; i < 5; ++i) {
      const double f = A[i][r] / A[r][r];
      for (int j = r + 1; j < 5; ++j) A[i][j] -= f * A[r][j];
      b[i] -= f * b[r];
    }
  }
  for (int i = 4; i >= 0; --i) {
    for (int j = i + 1; j < 5; ++j) b[i] -= A[i][j] * b[j];
    b[i] /= A[i][i];
  }
}

}  // namespace
}  // namespace sfm

using namespace sfm;

extern "C" {

int sfm_essential_decompose(const double* E_in, double* params) {
  SFM_REQUIRE(E_in && params, "null pointer argument");
  double E[3][3];
  memcpy(E, E_in, sizeof(E));
  const Decomp d = givens_decompose(E);
  params[0] = atan2(d.x.s, d.x.c);
  params[1] = atan2(d.y.s, d.y.c);
  params[2] = atan2(d.z.s, d.z.c);
  params[3] = atan2(d.u.s, d.u.c);
  params[4] = atan2(d.v.s, d.v.c);
  return SFM_OK;
}

int sfm_essential_decompose_uv(const double* E_in, double* U_out, double* V_out) {
  SFM_REQUIRE(E_in && U_out && V_out, "null pointer argument");
  double E[3][3], U[3][3], V[3][3];
  memcpy(E, E_in, sizeof(E));
  uv_from(givens_decompose(E), U, V);
  memcpy(U_out, U, sizeof(U));
  memcpy(V_out, V, sizeof(V));
  return SFM_OK;
}

int sfm_essential_optimise(const double* pin, const double* qin, int64_t n, const double* E_init, double delta,
                           double alpha, int max_reps, double* E_out) {
  SFM_REQUIRE(pin && qin && E_init && E_out, "null pointer argument");
  SFM_REQUIRE(n >= 0, "negative point count");
  double E[3][3], U[3][3], V[3][3];
  memcpy(E, E_init, sizeof(E));
  uv_from(givens_decompose(E), U, V);
  // transformed points p <- p . V, q <- q . U and per-point weights
  std::vector<double> P((size_t)n * 3), Q((size_t)n * 3), W((size_t)n);
  for (int rep = 0;; ++rep) {
    for (int64_t i = 0; i < n; ++i)
      for (int j = 0; j < 3; ++j) {
        P[3 * i + j] = pin[2 * i] * V[0][j] + pin[2 * i + 1] * V[1][j] + 1.0 * V[2][j];
        Q[3 * i + j] = qin[2 * i] * U[0][j] + qin[2 * i + 1] * U[1][j] + 1.0 * U[2][j];
      }
    double g[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    for (int64_t k = 0; k < n; ++k) {
      const double* p = &P[3 * k];
      const double* q = &Q[3 * k];
      const double r = p[0] * q[0] + p[1] * q[1];
      W[k] = (fabs(r) < delta) ? 1.0 : alpha * delta / fabs(r);
      g[0] += -p[1] * q[2] * -r * W[k];
      g[1] += -p[0] * q[2] * -r * W[k];
      g[2] += (p[1] * q[0] - p[0] * q[1]) * -r * W[k];
      g[3] += -p[2] * q[1] * -r * W[k];
      g[4] += -p[2] * q[0] * -r * W[k];
    }
    double mag = 0.0;
    for (int i = 0; i < 5; ++i) mag += g[i] * g[i];
    if (mag < 1e-20) break;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) E[i][j] = U[i][0] * V[j][0] + U[i][1] * V[j][1];
    if (rep == max_reps) break;
    double JtJ[5][5];
    for (int i = 0; i < 5; ++i)
      for (int j = 0; j < 5; ++j) JtJ[i][j] = 0.0;
    for (int64_t k = 0; k < n; ++k) {
      const double* p = &P[3 * k];
      const double* q = &Q[3 * k];
      const double J[5] = {-p[1] * q[2], -p[0] * q[2], p[1] * q[0] - p[0] * q[1], -p[2] * q[1], -p[2] * q[0]};
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 5; ++j) JtJ[i][j] += W[k] * J[i] * J[j];
    }
    gauss5(JtJ, g);
    rotate_right(U, 0, 1, g[2]);
    rotate_right(U, 0, 2, g[1]);
    rotate_right(U, 1, 2, g[0]);
    rotate_right(V, 1, 2, g[3]);
    rotate_right(V, 0, 2, g[4]);
  }
  memcpy(E_out, E, sizeof(E));
  return SFM_OK;
}

}  // extern "C"
