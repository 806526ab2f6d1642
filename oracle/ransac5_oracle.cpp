// ============================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into the product path.
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
// this library (as the checker / the CPU baseline), never as the thing measured.
//
// CPU restatement of the reference's RANSAC five-point essential-matrix path
// (jytime/Deep-SfM-Revisited, RANSAC_FiveP/essential_matrix/).  Written from
// the reference's algorithm description; the floating-point operation ORDER of
// every step follows the reference so results are bit-identical to the
// reference solver compiled on the host (oracle/_ref, see oracle/Makefile).
//
// Parity is pinned by tests/golden/*.npz generated from oracle/_ref (the
// reference's own solver sources compiled with g++) by oracle/gen_golden.py.
//
// Build: g++ -O2 -std=c++17 -fPIC -shared -fopenmp -ffp-contract=off
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace orc {

// ---------------------------------------------------------------------------
// Hypothesis sampler (the build's specified sampler; the reference used
// cuRAND XORWOW, which is not reproducible here — SURVEY.md §8(c)).
// Philox4x32-10 keyed by the 64-bit seed; counter = {h, draw>>2, 0, 0}.
// The uniform follows curand_uniform's (0,1] mapping, the integer follows
// RandomInt (kernel_functions.cu:269-278) in float arithmetic, clamped to N-1.
// ---------------------------------------------------------------------------
static inline void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += W0; k1 += W1; }
    uint64_t p0 = (uint64_t)M0 * c[0];
    uint64_t p1 = (uint64_t)M1 * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k0;
    uint32_t n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
  }
}

static inline uint32_t draw_u32(uint64_t seed, uint32_t h, uint32_t d) {
  uint32_t c[4] = {h, d >> 2, 0u, 0u};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  return c[d & 3];
}

static inline int64_t sample_index(uint64_t seed, uint32_t h, uint32_t d, int64_t n) {
  const float inv32 = 2.3283064e-10f;             // 2^-32 as in curand
  float u = (float)draw_u32(seed, h, d) * inv32;  // exact power-of-two scale
  u = u + inv32 / 2.0f;                           // (0,1]
  int maxi = (int)(n - 1);
  float r = u * ((float)maxi + 0.999999f);         // RandomInt, min_int = 0
  r = r + 0.0f;
  int64_t idx = (int64_t)truncf(r);
  if (idx > n - 1) idx = n - 1;                    // reference quirk: OOB read at u==1
  if (idx < 0) idx = 0;
  return idx;
}

// ---------------------------------------------------------------------------
// Polynomials in (w, x, y, z=1) used by the 5-point solver.
//   P1: linear form, 4 coefficients   (essential_matrix_5pt.h poly4_1)
//   P2: symmetric quadratic, entries (a<=b) of a 4x4 array (poly4_2)
//   P3: symmetric cubic, entries (a<=b<=c) of a 4x4x4 array (poly4_3)
// Products follow essential_matrix_5pt.cu:26-120: each target coefficient is
// the ordered sum of contributions over the (lexicographically ordered)
// lower-degree index sets.
// ---------------------------------------------------------------------------
struct P1 { double c[4]; };
struct P2 { double c[4][4]; };
struct P3 { double c[4][4][4]; };

static inline P2 mul11(const P1& a, const P1& b) {
  P2 r;
  for (int i = 0; i < 4; ++i)
    for (int j = i; j < 4; ++j) {
      if (i == j) r.c[i][j] = a.c[i] * b.c[j];
      else r.c[i][j] = a.c[i] * b.c[j] + a.c[j] * b.c[i];
    }
  return r;
}

static inline void add2(P2& a, const P2& b) {
  for (int i = 0; i < 4; ++i) for (int j = i; j < 4; ++j) a.c[i][j] += b.c[i][j];
}
static inline P2 plus2(const P2& a, const P2& b) {
  P2 r; for (int i = 0; i < 4; ++i) for (int j = i; j < 4; ++j) r.c[i][j] = a.c[i][j] + b.c[i][j];
  return r;
}
static inline P2 minus2(const P2& a, const P2& b) {
  P2 r; for (int i = 0; i < 4; ++i) for (int j = i; j < 4; ++j) r.c[i][j] = a.c[i][j] - b.c[i][j];
  return r;
}

// poly4_2 * poly4_1 (essential_matrix_5pt.cu:64-120): iterate (a<=b) in
// lexicographic order, k = 0..3; the first contribution to a sorted target
// assigns, later ones accumulate.
static inline P3 mul21(const P2& a, const P1& b) {
  P3 r; bool set[4][4][4];
  memset(set, 0, sizeof(set));
  for (int i = 0; i < 4; ++i)
    for (int j = i; j < 4; ++j)
      for (int k = 0; k < 4; ++k) {
        int t0, t1, t2;
        if (k < i) { t0 = k; t1 = i; t2 = j; }
        else if (k <= j) { t0 = i; t1 = k; t2 = j; }
        else { t0 = i; t1 = j; t2 = k; }
        double v = a.c[i][j] * b.c[k];
        if (!set[t0][t1][t2]) { r.c[t0][t1][t2] = v; set[t0][t1][t2] = true; }
        else r.c[t0][t1][t2] += v;
      }
  return r;
}

#define FOR3(i, j, k) for (int i = 0; i < 4; ++i) for (int j = i; j < 4; ++j) for (int k = j; k < 4; ++k)
static inline P3 plus3(const P3& a, const P3& b) { P3 r; FOR3(i, j, k) r.c[i][j][k] = a.c[i][j][k] + b.c[i][j][k]; return r; }
static inline P3 minus3(const P3& a, const P3& b) { P3 r; FOR3(i, j, k) r.c[i][j][k] = a.c[i][j][k] - b.c[i][j][k]; return r; }
static inline P3 scale3(const P3& a, double s) { P3 r; FOR3(i, j, k) r.c[i][j][k] = a.c[i][j][k] * s; return r; }
static inline void add3(P3& a, const P3& b) { FOR3(i, j, k) a.c[i][j][k] += b.c[i][j][k]; }
static inline void zero3(P3& a) { memset(&a, 0, sizeof(a)); }

// Equation set: 5 degrees (w^0..w^4) of a 10x10 coefficient matrix
// (common.h EquationSet).
typedef double Eqs[5][10][10];

// mono_coeff (essential_matrix_5pt.cu:356-426): monomials of a cubic in x,y
// (z=1) grouped by degree in w.  Index: 0 1 x 2 y 3 xx 4 xy 5 yy 6 xxx 7 xxy 8 xyy 9 yyy
static void monomials(const P3& B, Eqs A, int n) {
  const int W = 0, X = 1, Y = 2, Z = 3;
  A[0][n][0] = B.c[Z][Z][Z]; A[0][n][1] = B.c[X][Z][Z]; A[0][n][2] = B.c[Y][Z][Z];
  A[0][n][3] = B.c[X][X][Z]; A[0][n][5] = B.c[Y][Y][Z]; A[0][n][4] = B.c[X][Y][Z];
  A[0][n][6] = B.c[X][X][X]; A[0][n][7] = B.c[X][X][Y]; A[0][n][8] = B.c[X][Y][Y];
  A[0][n][9] = B.c[Y][Y][Y];
  A[1][n][0] = B.c[W][Z][Z]; A[1][n][1] = B.c[W][X][Z]; A[1][n][2] = B.c[W][Y][Z];
  A[1][n][3] = B.c[W][X][X]; A[1][n][5] = B.c[W][Y][Y]; A[1][n][4] = B.c[W][X][Y];
  A[2][n][0] = B.c[W][W][Z]; A[2][n][1] = B.c[W][W][X]; A[2][n][2] = B.c[W][W][Y];
  A[3][n][0] = B.c[W][W][W];
}

// Ematrix_5pt + null_space_solve_5x9 (essential_matrix_5pt.cu:631-711):
// 5 epipolar rows, 4 deterministic filler rows, modified Gram-Schmidt,
// the last 4 orthonormal rows span the null space.
static void nullspace_basis(const double q[5][3], const double qp[5][3], P1 E[3][3]) {
  double M[9][9];
  memset(M, 0, sizeof(M));
  for (int i = 0; i < 5; ++i)
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) M[i][3 * a + b] = qp[i][a] * q[i][b];
  const double PPi = 3.18730379;
  double ran = PPi;
  for (int i = 5; i < 9; ++i)
    for (int j = 0; j < 9; ++j) {
      ran *= PPi;
      ran = 2.0 * (ran - floor(ran)) - 1.0;
      M[i][j] = ran;
    }
  for (int r = 0; r < 9; ++r) {
    double ss = 0.0;
    for (int j = 0; j < 9; ++j) ss += M[r][j] * M[r][j];
    double f = 1.0 / sqrt(ss);
    for (int j = 0; j < 9; ++j) M[r][j] *= f;
    for (int i = r + 1; i < 9; ++i) {
      double dot = 0.0;
      for (int j = 0; j < 9; ++j) dot += M[r][j] * M[i][j];
      for (int j = 0; j < 9; ++j) M[i][j] -= dot * M[r][j];
    }
  }
  for (int e = 0; e < 9; ++e)
    E[e / 3][e % 3] = P1{{M[5][e], M[6][e], M[7][e], M[8][e]}};
}

// EEeqns_5pt (essential_matrix_5pt.cu:428-474): det(E)=0 and
// 2 E E^T E - tr(E E^T) E = 0 as 10 cubic equations.
static void constraint_equations(P1 E[3][3], Eqs A) {
  memset(&A[0][0][0], 0, sizeof(Eqs));
  // trace(E E^T) accumulated in row-major element order (traceEEt)
  P2 tr = mul11(E[0][0], E[0][0]);
  const int ord[8][2] = {{0,1},{0,2},{1,0},{1,1},{1,2},{2,0},{2,1},{2,2}};
  for (int t = 0; t < 8; ++t) tr = plus2(tr, mul11(E[ord[t][0]][ord[t][1]], E[ord[t][0]][ord[t][1]]));
  // determinant by cofactors of column 0 (polydet4)
  P3 d0 = mul21(minus2(mul11(E[1][1], E[2][2]), mul11(E[2][1], E[1][2])), E[0][0]);
  P3 d1 = mul21(minus2(mul11(E[2][1], E[0][2]), mul11(E[0][1], E[2][2])), E[1][0]);
  P3 d2 = mul21(minus2(mul11(E[0][1], E[1][2]), mul11(E[1][1], E[0][2])), E[2][0]);
  monomials(plus3(plus3(d0, d1), d2), A, 0);
  int eqn = 1;
  for (int i = 0; i < 3; ++i) {
    P3 row[3];
    for (int j = 0; j < 3; ++j) zero3(row[j]);
    for (int q = 0; q < 3; ++q) {
      P2 eet; memset(&eet, 0, sizeof(eet));
      for (int p = 0; p < 3; ++p) add2(eet, mul11(E[i][p], E[q][p]));
      for (int j = 0; j < 3; ++j) add3(row[j], mul21(eet, E[q][j]));
    }
    for (int j = 0; j < 3; ++j) monomials(minus3(scale3(row[j], 2.0), mul21(tr, E[i][j])), A, eqn++);
  }
}

// Row operations on the equation set; only the structurally non-zero column
// ranges are touched: deg0 cols [0,lim], deg1 6 cols, deg2 3, deg3 1
// (sweep_up / sweep_down / pivot, essential_matrix_5pt.cu:713-848).
static void row_elim(Eqs A, int prow, int col, int deg, int target) {
  const double fac = A[deg][target][col] / A[deg][prow][col];
  for (int j = 0; j <= col; ++j) A[0][target][j] -= fac * A[0][prow][j];
  for (int j = 0; j < 6; ++j) A[1][target][j] -= fac * A[1][prow][j];
  for (int j = 0; j < 3; ++j) A[2][target][j] -= fac * A[2][prow][j];
  A[3][target][0] -= fac * A[3][prow][0];
}
static void elim_above(Eqs A, int row, int col, int deg) {
  for (int i = 0; i < row; ++i) row_elim(A, row, col, deg, i);
}
static void elim_below(Eqs A, int row, int col, int deg, int last) {
  for (int i = row + 1; i <= last; ++i) row_elim(A, row, col, deg, i);
}
static void partial_pivot(Eqs A, int last) {
  double best = fabs(A[0][last][last]);
  int r = last;
  for (int i = 0; i < last; ++i)
    if (fabs(A[0][i][last]) > best) { r = i; best = fabs(A[0][i][last]); }
  if (r == last) return;
  for (int j = 0; j <= last; ++j) std::swap(A[0][last][j], A[0][r][j]);
  for (int j = 0; j < 6; ++j) std::swap(A[1][last][j], A[1][r][j]);
  for (int j = 0; j < 3; ++j) std::swap(A[2][last][j], A[2][r][j]);
  std::swap(A[3][last][0], A[3][r][0]);
}

// reduce_Ematrix (essential_matrix_5pt.cu:852-900): eliminate to a 3x3
// matrix of polynomials in w (column 0 degree 4, columns 1,2 degree 3).
static void reduce_to_3x3(Eqs A) {
  for (int c = 9; c >= 3; --c) { partial_pivot(A, c); elim_above(A, c, c, 0); }
  elim_below(A, 3, 3, 0, 5);
  elim_below(A, 4, 4, 0, 5);
  elim_above(A, 2, 5, 1);
  elim_above(A, 1, 4, 1);
  elim_below(A, 0, 3, 1, 5);
  elim_below(A, 1, 4, 1, 5);
  elim_below(A, 2, 5, 1, 5);
  for (int i = 0; i < 3; ++i) {
    double f = A[1][i][3 + i] / A[0][3 + i][3 + i];
    A[4][i][0] = -A[3][i + 3][0] * f;
    for (int j = 0; j < 3; ++j) {
      A[3][i][j] -= A[2][i + 3][j] * f;
      A[2][i][j] -= A[1][i + 3][j] * f;
      A[1][i][j] -= A[0][i + 3][j] * f;
    }
  }
}

// compute_determinant / one_cofactor (essential_matrix_5pt.cu:902-948)
static void det_poly(Eqs A, double poly[11]) {
  for (int i = 0; i <= 10; ++i) poly[i] = 0.0;
  const int rr[3][3] = {{0, 1, 2}, {1, 2, 0}, {2, 0, 1}};
  for (int t = 0; t < 3; ++t) {
    const int r0 = rr[t][0], r1 = rr[t][1], r2 = rr[t][2];
    double minor2[7];
    for (int i = 0; i < 7; ++i) minor2[i] = 0.0;
    for (int i = 0; i <= 3; ++i)
      for (int j = 0; j <= 3; ++j)
        minor2[i + j] += A[i][r1][1] * A[j][r2][2] - A[i][r2][1] * A[j][r1][2];
    for (int i = 0; i <= 6; ++i)
      for (int j = 0; j <= 4; ++j) poly[i + j] += A[j][r0][0] * minor2[i];
  }
}

// ---------------------------------------------------------------------------
// Sturm-sequence real root isolation (sturm.cu).  Recursion of sbisect is
// restated with an explicit stack; depth limit MAX_RECURSE_DEPTH = 10.
// ---------------------------------------------------------------------------
static const double kRelErr = 1.0e-12;
static const int kMaxPow = 32;
static const int kMaxIt = 800;
static const int kMaxDepth = 10;
static const double kSmall = 1.0e-12;

struct SPoly { int ord; double c[11]; };

static inline double horner(int ord, const double* c, double x) {
  double f = c[ord];
  for (int i = ord - 1; i >= 0; --i) f = x * f + c[i];
  return f;
}

// modrf_pos (sturm.cu:43-207)
static int regula_falsi(int ord, const double* c, double a, double b, double* val, bool inv) {
  if (inv) { double t = a; a = 1.0 / b; b = 1.0 / t; }
  double fa, fb;
  if (inv) {
    fa = fb = c[0];
    for (int i = 1; i <= ord; ++i) { fa = a * fa + c[i]; fb = b * fb + c[i]; }
  } else {
    fa = fb = c[ord];
    for (int i = ord - 1; i >= 0; --i) { fa = a * fa + c[i]; fb = b * fb + c[i]; }
  }
  if (fa * fb > 0.0) return 0;
  if (fabs(fa) < kRelErr) { *val = inv ? 1.0 / a : a; return 1; }
  if (fabs(fb) < kRelErr) { *val = inv ? 1.0 / b : b; return 1; }
  double lfx = fa;
  for (int it = 0; it < kMaxIt; ++it) {
    double x = (fb * a - fa * b) / (fb - fa);
    double fx;
    if (inv) { fx = c[0]; for (int i = 1; i <= ord; ++i) fx = x * fx + c[i]; }
    else { fx = c[ord]; for (int i = ord - 1; i >= 0; --i) fx = x * fx + c[i]; }
    if (fabs(x) > kRelErr && fabs(fx / x) < kRelErr) { *val = inv ? 1.0 / x : x; return 1; }
    else if (fabs(fx) < kRelErr) { *val = inv ? 1.0 / x : x; return 1; }
    if ((fa * fx) < 0) { b = x; fb = fx; if ((lfx * fx) > 0) fa /= 2; }
    else { a = x; fa = fx; if ((lfx * fx) > 0) fb /= 2; }
    if (fabs(b - a) < fabs(kRelErr * a)) { *val = inv ? 1.0 / a : a; return 1; }
    lfx = fx;
  }
  return 0;
}

// modrf (sturm.cu:218-275), including the reference's omission of the
// leading coefficient when evaluating at +-1 and the end points.
static int regula_falsi_any(int ord, const double* c, double a, double b, double* val) {
  if (a > b) { double t = a; a = b; b = t; }
  if (b <= 1.0 && a >= -1.0) return regula_falsi(ord, c, a, b, val, false);
  if (a >= 1.0 || b <= -1.0) return regula_falsi(ord, c, a, b, val, true);
  double fp1 = 0.0, fm1 = 0.0, fa = 0.0, fb = 0.0;
  for (int i = ord - 1; i >= 0; --i) {
    fp1 = c[i] + fp1;
    fm1 = c[i] - fm1;
    fa = a * fa + c[i];
    fb = b * fb + c[i];
  }
  if (a < -1.0 && b > 1.0) {
    if (fa * fm1 < 0.0) return regula_falsi(ord, c, a, -1.0, val, true);
    else if (fb * fp1 < 0.0) return regula_falsi(ord, c, 1.0, b, val, true);
    else return regula_falsi(ord, c, -1.0, 1.0, val, false);
  } else if (a < -1.0) {
    if (fa * fm1 < 0.0) return regula_falsi(ord, c, a, -1.0, val, true);
    else return regula_falsi(ord, c, -1.0, b, val, false);
  } else {
    if (fb * fp1 < 0.0) return regula_falsi(ord, c, 1.0, b, val, true);
    else return regula_falsi(ord, c, a, 1.0, val, false);
  }
}

// modp (sturm.cu:285-322): remainder of u / v, v monic up to sign.
static int poly_rem(const SPoly& u, const SPoly& v, SPoly& r) {
  for (int i = 0; i <= u.ord; ++i) r.c[i] = u.c[i];
  if (v.c[v.ord] < 0.0) {
    for (int k = u.ord - v.ord - 1; k >= 0; k -= 2) r.c[k] = -r.c[k];
    for (int k = u.ord - v.ord; k >= 0; --k)
      for (int j = v.ord + k - 1; j >= k; --j) r.c[j] = -r.c[j] - r.c[v.ord + k] * v.c[j - k];
  } else {
    for (int k = u.ord - v.ord; k >= 0; --k)
      for (int j = v.ord + k - 1; j >= k; --j) r.c[j] -= r.c[v.ord + k] * v.c[j - k];
  }
  int k = v.ord - 1;
  while (k >= 0 && fabs(r.c[k]) < kSmall) { r.c[k] = 0.0; --k; }
  r.ord = (k < 0) ? 0 : k;
  return r.ord;
}

// buildsturm (sturm.cu:331-360)
static int sturm_chain(int ord, SPoly* s) {
  s[0].ord = ord;
  s[1].ord = ord - 1;
  double f = fabs(s[0].c[ord] * ord);
  for (int i = 1; i <= ord; ++i) s[1].c[i - 1] = s[0].c[i] * i / f;
  int k = 2;
  while (poly_rem(s[k - 2], s[k - 1], s[k])) {
    double g = -fabs(s[k].c[s[k].ord]);
    for (int i = s[k].ord; i >= 0; --i) s[k].c[i] /= g;
    ++k;
  }
  s[k].c[0] = -s[k].c[0];
  return k;
}

// numchanges (sturm.cu:369-385)
static int sign_changes(int np, const SPoly* s, double a) {
  int ch = 0;
  double lf = horner(s[0].ord, s[0].c, a);
  for (int i = 1; i <= np; ++i) {
    double f = horner(s[i].ord, s[i].c, a);
    if (lf == 0.0 || lf * f < 0) ++ch;
    lf = f;
  }
  return ch;
}

// numroots (sturm.cu:393-439), non_neg = false
static int count_real(int np, const SPoly* s, int* atneg, int* atpos) {
  int pos = 0, neg = 0;
  double lf = s[0].c[s[0].ord];
  for (int i = 1; i <= np; ++i) {
    double f = s[i].c[s[i].ord];
    if (lf == 0.0 || lf * f < 0) ++pos;
    lf = f;
  }
  lf = (s[0].ord & 1) ? -s[0].c[s[0].ord] : s[0].c[s[0].ord];
  for (int i = 1; i <= np; ++i) {
    double f = (s[i].ord & 1) ? -s[i].c[s[i].ord] : s[i].c[s[i].ord];
    if (lf == 0.0 || lf * f < 0) ++neg;
    lf = f;
  }
  *atneg = neg; *atpos = pos;
  return neg - pos;
}

struct Interval { double lo, hi; int atlo, athi, off, depth; };

// sbisect<depth> (sturm.cu:450-555) with an explicit work stack.  Root slots
// outside [0,10) (possible only for a numerically non-monotone sequence) are
// not written — the reference would write out of bounds there.
static void isolate_roots(int np, const SPoly* s, double lo, double hi, int atlo, int athi, double* roots) {
  Interval stk[64];
  int sp = 0;
  stk[sp++] = Interval{lo, hi, atlo, athi, 0, 0};
  while (sp > 0) {
    Interval iv = stk[--sp];
    if (iv.depth >= kMaxDepth) continue;
    double mn = iv.lo, mx = iv.hi, mid = 0.0;
    int n = iv.atlo - iv.athi;
    if (n == 1) {
      double v;
      if (regula_falsi_any(s[0].ord, s[0].c, mn, mx, &v)) {
        if (iv.off >= 0 && iv.off < 10) roots[iv.off] = v;
        continue;
      }
      int it;
      bool done = false;
      for (it = 0; it < kMaxIt; ++it) {
        mid = (double)((mn + mx) / 2);
        int atmid = sign_changes(np, s, mid);
        if (fabs(mid) > kRelErr) {
          if (fabs((mx - mn) / mid) < kRelErr) { done = true; break; }
        } else if (fabs(mx - mn) < kRelErr) { done = true; break; }
        if ((iv.atlo - atmid) == 0) mn = mid; else mx = mid;
      }
      (void)done;
      if (iv.off >= 0 && iv.off < 10) roots[iv.off] = mid;
      continue;
    }
    int it, n1 = 0;
    for (it = 0; it < kMaxIt; ++it) {
      mid = (double)((mn + mx) / 2);
      int atmid = sign_changes(np, s, mid);
      n1 = iv.atlo - atmid;
      int n2 = atmid - iv.athi;
      if (n1 != 0 && n2 != 0) {
        if (sp + 2 <= 64) {
          stk[sp++] = Interval{mid, mx, atmid, iv.athi, iv.off + n1, iv.depth + 1};
          stk[sp++] = Interval{mn, mid, iv.atlo, atmid, iv.off, iv.depth + 1};
        }
        break;
      }
      if (n1 == 0) mn = mid; else mx = mid;
    }
    if (it == kMaxIt)
      for (int r = iv.athi; r < iv.atlo; ++r) {
        int slot = iv.off + r - iv.athi;
        if (slot >= 0 && slot < 10) roots[slot] = mid;
      }
  }
}

// find_real_roots_sturm (sturm.cu:557-676), degree 10, non_neg = false.
// Returns nroots (may be <= 0: then no root is valid).
static int real_roots10(const double p[11], double roots[10]) {
  SPoly s[12];
  for (int i = 0; i < 12; ++i) { s[i].ord = 0; for (int j = 0; j < 11; ++j) s[i].c[j] = 0.0; }
  const int deg = 10;
  double norm = 1.0 / p[deg];
  for (int i = 0; i <= deg; ++i) s[0].c[i] = p[i] * norm;
  double v0 = fabs(s[0].c[0]);
  double fac = 1.0;
  if (v0 > 10.0) {
    fac = pow(v0, -1.0 / deg);
    double m = fac;
    for (int i = deg - 1; i >= 0; --i) { s[0].c[i] *= m; m = m * fac; }
  }
  int np = sturm_chain(deg, s);
  int atmin, atmax;
  int nr = count_real(np, s, &atmin, &atmax);
  if (nr == 0) return 0;
  double mn = -1.0;
  int nch = sign_changes(np, s, mn);
  for (int i = 0; nch != atmin && i != kMaxPow; ++i) { mn *= 10.0; nch = sign_changes(np, s, mn); }
  if (nch != atmin) atmin = nch;
  double mx = 1.0;
  nch = sign_changes(np, s, mx);
  for (int i = 0; nch != atmax && i != kMaxPow; ++i) { mx *= 10.0; nch = sign_changes(np, s, mx); }
  if (nch != atmax) atmax = nch;
  nr = atmin - atmax;
  if (nr <= 0) return nr;
  isolate_roots(np, s, mn, mx, atmin, atmax, roots);
  for (int i = 0; i < nr && i < 10; ++i) roots[i] /= fac;
  return nr;
}

// null_space_solve_3x3_half_pivot (essential_matrix_5pt.cu:476-507)
static void nullvec3(double M[3][3], double& x, double& y) {
  int p1;
  double f0 = fabs(M[0][2]), f1 = fabs(M[1][2]), f2 = fabs(M[2][2]);
  if (f0 > f1) p1 = (f0 > f2) ? 0 : 2;
  else p1 = (f1 > f2) ? 1 : 2;
  int r1 = (p1 + 1) % 3, r2 = (p1 + 2) % 3;
  double f = M[r1][2] / M[p1][2];
  M[r1][0] -= f * M[p1][0];
  M[r1][1] -= f * M[p1][1];
  f = M[r2][2] / M[p1][2];
  M[r2][0] -= f * M[p1][0];
  M[r2][1] -= f * M[p1][1];
  int p2 = fabs(M[r1][1]) > fabs(M[r2][1]) ? r1 : r2;
  x = -M[p2][0] / M[p2][1];
  y = -(M[p1][0] + M[p1][1] * x) / M[p1][2];
}

// compute_E_matrix (essential_matrix_5pt.cu:955-1015)
static void essential_from_root(P1 B[3][3], Eqs A, double w, double E[9]) {
  double w2 = w * w, w3 = w2 * w, w4 = w3 * w;
  double M[3][3];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      M[i][j] = A[0][i][j] + w * A[1][i][j] + w2 * A[2][i][j] + w3 * A[3][i][j];
    M[i][0] += w4 * A[4][i][0];
  }
  double x, y;
  nullvec3(M, x, y);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      const P1& p = B[i][j];
      E[3 * i + j] = w * p.c[0] + x * p.c[1] + y * p.c[2] + p.c[3];
    }
}

// compute_E_matrices_optimized (essential_matrix_5pt.cu:1224-1249).
// Returns nroots (<=0 -> no E written).
static int five_point(const double q[5][3], const double qp[5][3], double Es[10][9]) {
  P1 B[3][3];
  nullspace_basis(q, qp, B);
  static thread_local Eqs A;
  constraint_equations(B, A);
  reduce_to_3x3(A);
  double poly[11];
  det_poly(A, poly);
  double roots[10];
  for (int i = 0; i < 10; ++i) roots[i] = 0.0;
  int nr = real_roots10(poly, roots);
  for (int i = 0; i < nr && i < 10; ++i) essential_from_root(B, A, roots[i], Es[i]);
  return nr;
}

// compute_P_matrices (cheirality.cu:4-214), focal = null, npoints = 5.
// Compacts Es in place; returns nP.
static int cheirality(const double q[5][3], const double qp[5][3], double Es[10][9], int nE, double Ps[10][12]) {
  int nP = 0;
  for (int m = 0; m < nE; ++m) {
    double U[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    double V[3][3];
    memcpy(V, Es[m], sizeof(V));
    for (int i = 0; i <= 1; ++i)
      for (int k = i + 1; k < 3; ++k) {
        double a = V[i][i], b = V[k][i];
        double s = sqrt(a * a + b * b);
        if (s == 0.0) continue;
        a /= s; b /= s;
        V[i][i] = s; V[k][i] = 0.0;
        for (int j = i + 1; j < 3; ++j) {
          double c = V[i][j], d = V[k][j];
          V[i][j] = a * c + b * d;
          V[k][j] = a * d - b * c;
        }
        if (k == 1) {
          U[0][0] = U[1][1] = a; U[1][0] = -b; U[0][1] = b; U[2][2] = 1.0;
        } else {
          for (int j = 0; j < 3; ++j) {
            double t = a * U[i][j] + b * U[k][j];
            U[k][j] = -b * U[i][j] + a * U[k][j];
            U[i][j] = t;
          }
        }
      }
    double sc = 1.0 / sqrt(V[0][0] * V[0][0] + V[0][1] * V[0][1] + V[0][2] * V[0][2]);
    for (int i = 0; i < 2; ++i) for (int j = 0; j < 3; ++j) V[i][j] *= sc;
    V[2][0] = V[0][1] * V[1][2] - V[0][2] * V[1][1];
    V[2][1] = V[0][2] * V[1][0] - V[0][0] * V[1][2];
    V[2][2] = V[0][0] * V[1][1] - V[0][1] * V[1][0];
    int c0a = 0, c0b = 0, c1a = 0, c1b = 0;
    for (int pt = 0; pt < 5; ++pt) {
      const double* x1 = q[pt];
      const double* x2 = qp[pt];
      double v0 = 1.0 * x1[0] * V[0][0] + 1.0 * x1[1] * V[0][1] + x1[2] * V[0][2];
      double v2 = 1.0 * x1[0] * V[2][0] + 1.0 * x1[1] * V[2][1] + x1[2] * V[2][2];
      double u1 = 1.0 * x2[0] * U[1][0] + 1.0 * x2[1] * U[1][1] + x2[2] * U[1][2];
      double u2 = 1.0 * x2[0] * U[2][0] + 1.0 * x2[1] * U[2][1] + x2[2] * U[2][2];
      double d1 = v0 * u2 + v2 * u1;
      double d2 = -v0 * u2 + v2 * u1;
      if (-u1 / d1 > 0.0) ++c0a;
      if (v0 / d1 > 0.0) ++c0b;
      if (-u1 / d2 > 0.0) ++c1a;
      if (-v0 / d2 > 0.0) ++c1b;
    }
    int c0 = c0a + c0b, c1 = c1a + c1b;
    int form = -1;  // 0: +R form, 1: -R form
    double tsign = 1.0;
    if (c0 == 10) { form = 0; tsign = 1.0; }
    else if (c0 == 0) { form = 0; tsign = -1.0; }
    else if (c1 == 10) { form = 1; tsign = 1.0; }
    else if (c1 == 0) { form = 1; tsign = -1.0; }
    if (form < 0) continue;
    double* P = Ps[nP];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) {
        if (form == 0) P[4 * i + j] = U[0][i] * V[1][j] - U[1][i] * V[0][j] + U[2][i] * V[2][j];
        else P[4 * i + j] = -U[0][i] * V[1][j] + U[1][i] * V[0][j] + U[2][i] * V[2][j];
      }
    for (int i = 0; i < 3; ++i) P[4 * i + 3] = (tsign > 0) ? U[2][i] : -U[2][i];
    if (m > nP) memcpy(Es[nP], Es[m], sizeof(double) * 9);
    ++nP;
  }
  return nP;
}

// ComputeError<double> (kernel_functions.cu:232-264) -> inlier test
static inline bool is_inlier(const double* E, double x, double y, double xp, double yp, double thr) {
  double q[3] = {x, y, 1.0}, p[3] = {xp, yp, 1.0};
  double Ex[3], xE[3];
  for (int k = 0; k < 3; ++k) { double s = 0.0; for (int l = 0; l < 3; ++l) s += E[3 * k + l] * q[l]; Ex[k] = s; }
  for (int k = 0; k < 3; ++k) { double s = 0.0; for (int l = 0; l < 3; ++l) s += p[l] * E[3 * l + k]; xE[k] = s; }
  double xEx = 0.0;
  for (int k = 0; k < 3; ++k) xEx += p[k] * Ex[k];
  double d = sqrt(Ex[0] * Ex[0] + Ex[1] * Ex[1] + xE[0] * xE[0] + xE[1] * xE[1]);
  double e = xEx / d;
  if (e < 0.0) e = -e;
  return e <= thr;
}

// Round a float to the nearest binary16 value (ties to even; subnormals;
// overflow to inf), returned as a float.  x / q and nearbyintf are exact /
// round-to-nearest-even for the power-of-two quantum q.
static inline float h16(float f) {
  if (!std::isfinite(f)) return f;
  const float a = std::fabs(f);
  if (a >= 65520.0f) return std::copysign(INFINITY, f);     // past max (65504) + half an ulp
  float q;
  if (a < 0x1p-14f) {
    q = 0x1p-24f;                                            // subnormal quantum
  } else {
    int e;
    std::frexp(a, &e);                                       // a in [2^(e-1), 2^e)
    q = std::ldexp(1.0f, e - 1 - 10);
  }
  return std::copysign(std::nearbyint(a / q) * q, f);
}

// ComputeError<T> (kernel_functions.cu:232-264) with E, q, qp held in T
// (T = float for prec 32, binary16 for prec 16), E first scaled by a power of
// two to max |E_ij| in [0.5, 1) (exact; the error is invariant to the scale of
// E, and a small-norm five-point E would underflow in half); every operation rounded to T
// in the reference's source order; sqrt and division correctly rounded (for
// half computed in float and rounded once: 24 >= 2*11+2 bits makes the double
// rounding exact, as for + - *); inputs reach T through float32; the count
// test against the float64 threshold as at kernel_functions.cu:193-194.
// Mirrors ransac5.hip:inlier_lowp.
template <int PREC>
static inline bool is_inlier_lp(const double* E, double xd, double yd, double xpd, double ypd, double thr) {
  auto r = [](float v) { return PREC == 16 ? h16(v) : v; };
  double m = 0.0;
  for (int i = 0; i < 9; ++i) m = std::fmax(m, std::fabs(E[i]));
  int ex = 0;
  if (m > 0.0 && m < 0x1p1000) (void)std::frexp(m, &ex);     // max |E_ij| * 2^-ex in [0.5, 1): exact scaling
  float e[9];
  for (int i = 0; i < 9; ++i) e[i] = r((float)std::ldexp(E[i], -ex));
  const float x = r((float)xd), y = r((float)yd), xp = r((float)xpd), yp = r((float)ypd);
  auto mul = [&](float a, float b) { return r(a * b); };
  auto add = [&](float a, float b) { return r(a + b); };
  const float ex0 = add(add(mul(e[0], x), mul(e[1], y)), e[2]);
  const float ex1 = add(add(mul(e[3], x), mul(e[4], y)), e[5]);
  const float ex2 = add(add(mul(e[6], x), mul(e[7], y)), e[8]);
  const float xe0 = add(add(mul(xp, e[0]), mul(yp, e[3])), e[6]);
  const float xe1 = add(add(mul(xp, e[1]), mul(yp, e[4])), e[7]);
  const float a = add(add(mul(xp, ex0), mul(yp, ex1)), ex2);
  const float D = add(add(add(mul(ex0, ex0), mul(ex1, ex1)), mul(xe0, xe0)), mul(xe1, xe1));
  const float d = r(std::sqrt(D));
  float err = r(a / d);
  if (err < 0.0f) err = -err;
  return (double)err <= thr;
}

// A double rounded once to binary16 (ties to even; subnormals; overflow to
// inf), returned as a double.  The quantum arithmetic is exact in double.
static inline double h16d(double v) {
  if (!(std::fabs(v) < 65520.0)) return (double)h16((float)v);
  const double a = std::fabs(v);
  double q;
  if (a < 0x1p-14) {
    q = 0x1p-24;
  } else {
    int e;
    std::frexp(a, &e);
    q = std::ldexp(1.0, e - 1 - 10);
  }
  return std::copysign(std::nearbyint(a / q) * q, v);
}

// The literal ComputeError<T> (kernel_functions.cu:231-264) with the
// reference's Ematrix = double[3][3] (common.h:26), T = float (prec 33) or
// binary16 (prec 17): q, qp converted to T once; `sum += E[k][l] * q[l]` is a
// double product and a double add, the sum rounded to T; xEx, D, sqrt and the
// division in T (half: computed in float, rounded once -- exact by the
// 24 >= 2*11+2 rule); no scaling of E.  Mirrors ransac5.hip:inlier_lowp_tpl.
template <int PREC>
static inline bool is_inlier_lp_tpl(const double* E, double xd, double yd, double xpd, double ypd, double thr) {
  auto rd = [](double v) { return PREC == 17 ? h16d(v) : (double)(float)v; };     // double -> T
  auto r = [](float v) { return PREC == 17 ? h16(v) : v; };                      // float op result -> T
  const double q[3] = {rd(xd), rd(yd), 1.0}, qp[3] = {rd(xpd), rd(ypd), 1.0};
  float Ex[3], xE[3];
  for (int k = 0; k < 3; ++k) {
    double sum = 0.0;
    for (int l = 0; l < 3; ++l) sum = rd(sum + E[3 * k + l] * q[l]);
    Ex[k] = (float)sum;
  }
  for (int k = 0; k < 3; ++k) {
    double sum = 0.0;
    for (int l = 0; l < 3; ++l) sum = rd(sum + qp[l] * E[3 * l + k]);
    xE[k] = (float)sum;
  }
  float xEx = 0.0f;
  for (int k = 0; k < 3; ++k) xEx = r(xEx + r((float)qp[k] * Ex[k]));
  float D = r(r(Ex[0] * Ex[0]) + r(Ex[1] * Ex[1]));
  D = r(D + r(xE[0] * xE[0]));
  D = r(D + r(xE[1] * xE[1]));
  const float d = r(std::sqrt(D));
  float err = r(xEx / d);
  if (err < 0.0f) err = -err;
  return (double)err <= thr;
}

static inline bool is_inlier_p(const double* E, double x, double y, double xp, double yp, double thr, int prec) {
  if (prec == 32) return is_inlier_lp<32>(E, x, y, xp, yp, thr);
  if (prec == 16) return is_inlier_lp<16>(E, x, y, xp, yp, thr);
  if (prec == 33) return is_inlier_lp_tpl<33>(E, x, y, xp, yp, thr);
  if (prec == 17) return is_inlier_lp_tpl<17>(E, x, y, xp, yp, thr);
  return is_inlier(E, x, y, xp, yp, thr);
}

static int64_t count_inliers(const double* E, const double* q, const double* qp, int64_t n, double thr,
                             int prec = 64) {
  int64_t c = 0;
  for (int64_t k = 0; k < n; ++k) c += is_inlier_p(E, q[2 * k], q[2 * k + 1], qp[2 * k], qp[2 * k + 1], thr, prec);
  return c;
}

}  // namespace orc

using namespace orc;

extern "C" {

int orc_version(void) { return 1; }

uint32_t orc_philox_u32(uint64_t seed, uint32_t h, uint32_t d) { return draw_u32(seed, h, d); }

int64_t orc_sample_index(uint64_t seed, uint32_t h, uint32_t d, int64_t n) { return sample_index(seed, h, d, n); }

// One five-point solve on explicit points (x,y pairs). Outputs the roots' E
// (before cheirality) and, if cheir != 0, the compacted E and P sets.
int orc_solve5(const double* q5, const double* qp5, int cheir,
               double* E_roots /*10x9*/, int* nroots,
               double* E_out /*10x9*/, double* P_out /*10x12*/, int* nP) {
  double q[5][3], qp[5][3];
  for (int i = 0; i < 5; ++i) {
    q[i][0] = q5[2 * i]; q[i][1] = q5[2 * i + 1]; q[i][2] = 1.0;
    qp[i][0] = qp5[2 * i]; qp[i][1] = qp5[2 * i + 1]; qp[i][2] = 1.0;
  }
  double Es[10][9], Ps[10][12];
  memset(Es, 0, sizeof(Es)); memset(Ps, 0, sizeof(Ps));
  int nr = five_point(q, qp, Es);
  *nroots = nr;
  if (E_roots) memcpy(E_roots, Es, sizeof(Es));
  int np = 0;
  if (cheir) np = cheirality(q, qp, Es, nr, Ps);
  if (nP) *nP = np;
  if (E_out) memcpy(E_out, Es, sizeof(Es));
  if (P_out) memcpy(P_out, Ps, sizeof(Ps));
  return 0;
}

int orc_inlier_count(const double* E, const double* q, const double* qp, int64_t n, double thr) {
  return (int)count_inliers(E, q, qp, n, thr);
}

void orc_inlier_mask(const double* E, const double* q, const double* qp, int64_t n, double thr, uint8_t* mask) {
  for (int64_t k = 0; k < n; ++k) mask[k] = is_inlier(E, q[2 * k], q[2 * k + 1], qp[2 * k], qp[2 * k + 1], thr);
}

void orc_inlier_mask_prec(const double* E, const double* q, const double* qp, int64_t n, double thr, int prec,
                          uint8_t* mask) {
  for (int64_t k = 0; k < n; ++k)
    mask[k] = is_inlier_p(E, q[2 * k], q[2 * k + 1], qp[2 * k], qp[2 * k + 1], thr, prec);
}

// Full RANSAC over one pair, restating EstimateProjectionMatrix<5> /
// EstimateEssentialMatrix<5> (kernel_functions.cu:53-226) for `nchains`
// chains x `iters` iterations (reference: 512 threads), plus the host argmax
// (essential_matrix.cu:248-265).  Canonical rules for the reference's
// indeterminate state:
//   * the E slot array persists across a chain's iterations and starts at 0;
//   * the P slot array likewise persists and starts at 0;
//   * if no hypothesis has > 0 inliers, E = P = 0, inliers = 0, winner = -1.
// hyp_score (optional, nchains*iters): rescored inlier count per hypothesis.
// hyp_ncand (optional): nP (cheir) / nroots (no cheir) per hypothesis.
// prec: 64 = ComputeError<double> (the reference), 32 / 16 = is_inlier_lp,
// 33 / 17 = is_inlier_lp_tpl (the literal template form).
int orc_ransac5_prec(const double* q, const double* qp, int64_t n, int num_test, int num_ransac_test,
                     int nchains, int iters, double thr, uint64_t seed, int cheir, int nthreads, int prec,
                     double* E_out, double* P_out, int* inliers_out, int* winner_out,
                     int* hyp_score, int* hyp_ncand, int* hyp_best) {
  if (prec != 64 && prec != 32 && prec != 16 && prec != 33 && prec != 17) return 1;
  if (n < 1 || num_test < 0 || num_ransac_test < 0 || num_test > n || num_ransac_test > n) return 1;
  const int H = nchains * iters;
  std::vector<int> score(H, 0), best(H, 0);
  std::vector<double> Ewin((size_t)H * 9, 0.0), Pwin((size_t)H * 12, 0.0);
  std::vector<int> ncand(H, 0);
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int t = 0; t < nchains; ++t) {
    double Eslots[10][9], Pslots[10][12];
    memset(Eslots, 0, sizeof(Eslots)); memset(Pslots, 0, sizeof(Pslots));
    for (int i = 0; i < iters; ++i) {
      const int h = t * iters + i;
      double qs[5][3], qps[5][3];
      for (int d = 0; d < 5; ++d) {
        int64_t idx = sample_index(seed, (uint32_t)h, (uint32_t)d, n);
        qs[d][0] = q[2 * idx]; qs[d][1] = q[2 * idx + 1]; qs[d][2] = 1.0;
        qps[d][0] = qp[2 * idx]; qps[d][1] = qp[2 * idx + 1]; qps[d][2] = 1.0;
      }
      double Es[10][9];
      memcpy(Es, Eslots, sizeof(Es));
      int nr = five_point(qs, qps, Es);
      int nc = nr > 0 ? nr : 0;
      double Ps[10][12];
      memcpy(Ps, Pslots, sizeof(Ps));
      if (cheir) nc = cheirality(qs, qps, Es, nc, Ps);
      ncand[h] = nc;
      int bi = 0, bc = 0;
      for (int j = 0; j < nc; ++j) {
        int c = (int)count_inliers(Es[j], q, qp, num_test, thr, prec);
        if (c > bc) { bc = c; bi = j; }
      }
      best[h] = bi;
      score[h] = (int)count_inliers(Es[bi], q, qp, num_ransac_test, thr, prec);
      memcpy(&Ewin[(size_t)h * 9], Es[bi], sizeof(double) * 9);
      memcpy(&Pwin[(size_t)h * 12], Ps[bi], sizeof(double) * 12);
      memcpy(Eslots, Es, sizeof(Es));
      memcpy(Pslots, Ps, sizeof(Ps));
    }
  }
  int win = -1, wbest = 0;
  for (int t = 0; t < nchains; ++t) {
    int tb = 0, th = -1;
    for (int i = 0; i < iters; ++i) {
      int h = t * iters + i;
      if (score[h] > tb) { tb = score[h]; th = h; }
    }
    if (tb > wbest) { wbest = tb; win = th; }
  }
  if (win >= 0) {
    memcpy(E_out, &Ewin[(size_t)win * 9], sizeof(double) * 9);
    memcpy(P_out, &Pwin[(size_t)win * 12], sizeof(double) * 12);
  } else {
    memset(E_out, 0, sizeof(double) * 9);
    memset(P_out, 0, sizeof(double) * 12);
  }
  *inliers_out = wbest;
  if (winner_out) *winner_out = win;
  if (hyp_score) memcpy(hyp_score, score.data(), sizeof(int) * H);
  if (hyp_ncand) memcpy(hyp_ncand, ncand.data(), sizeof(int) * H);
  if (hyp_best) memcpy(hyp_best, best.data(), sizeof(int) * H);
  return 0;
}

int orc_ransac5(const double* q, const double* qp, int64_t n, int num_test, int num_ransac_test,
                int nchains, int iters, double thr, uint64_t seed, int cheir, int nthreads,
                double* E_out, double* P_out, int* inliers_out, int* winner_out,
                int* hyp_score, int* hyp_ncand, int* hyp_best) {
  return orc_ransac5_prec(q, qp, n, num_test, num_ransac_test, nchains, iters, thr, seed, cheir, nthreads, 64,
                          E_out, P_out, inliers_out, winner_out, hyp_score, hyp_ncand, hyp_best);
}

// ---------------------------------------------------------------------------
// E decomposition and IRLS refinement (polish_E.cu:147-472, 1470-1577)
// ---------------------------------------------------------------------------
static void givens_params(double E[3][3], double prm[10]) {
  // prm: cx sx cy sy cz sz cu su cv sv
  double cz = E[0][0], sz = -E[1][0], s = sqrt(cz * cz + sz * sz);
  cz /= s; sz /= s;
  for (int j = 0; j < 3; ++j) { double t = E[0][j] * cz - E[1][j] * sz; E[1][j] = E[0][j] * sz + E[1][j] * cz; E[0][j] = t; }
  double cy = E[0][0], sy = -E[2][0];
  s = sqrt(cy * cy + sy * sy); cy /= s; sy /= s;
  for (int j = 0; j < 3; ++j) { double t = E[0][j] * cy - E[2][j] * sy; E[2][j] = E[0][j] * sy + E[2][j] * cy; E[0][j] = t; }
  double cx = E[1][1], sx = -E[2][1];
  s = sqrt(cx * cx + sx * sx); cx /= s; sx /= s;
  for (int j = 1; j < 3; ++j) E[1][j] = E[1][j] * cx - E[2][j] * sx;
  double cu = E[1][1], su = -E[1][2];
  s = sqrt(cu * cu + su * su); cu /= s; su /= s;
  E[0][2] = su * E[0][1] + cu * E[0][2];
  double cv = E[0][0], sv = -E[0][2];
  s = sqrt(cv * cv + sv * sv); cv /= s; sv /= s;
  prm[0] = cx; prm[1] = sx; prm[2] = cy; prm[3] = sy; prm[4] = cz; prm[5] = sz;
  prm[6] = cu; prm[7] = su; prm[8] = cv; prm[9] = sv;
}

static void decompose_uv(double E[3][3], double U[3][3], double V[3][3]) {
  double p[10];
  givens_params(E, p);
  double cx = p[0], sx = p[1], cy = p[2], sy = p[3], cz = p[4], sz = p[5], cu = p[6], su = p[7], cv = p[8], sv = p[9];
  U[0][0] = cy * cz; U[0][1] = -cz * sx * sy + cx * sz; U[0][2] = cx * cz * sy + sx * sz;
  U[1][0] = -cy * sz; U[1][1] = cx * cz + sx * sy * sz; U[1][2] = cz * sx - cx * sy * sz;
  U[2][0] = -sy; U[2][1] = -cy * sx; U[2][2] = cx * cy;
  V[0][0] = cv; V[0][1] = 0; V[0][2] = sv;
  V[1][0] = -su * sv; V[1][1] = cu; V[1][2] = cv * su;
  V[2][0] = -cu * sv; V[2][1] = -su; V[2][2] = cu * cv;
}

static void rotate_cols(double E[3][3], int r1, int r2, double ang) {
  double c = cos(ang), s = sin(ang);
  for (int i = 0; i < 3; ++i) {
    double t = E[i][r1] * c - E[i][r2] * s;
    E[i][r2] = E[i][r1] * s + E[i][r2] * c;
    E[i][r1] = t;
  }
}

static void solve5(double A[5][5], double b[5]) {
  for (int row = 0; row < 5; ++row) {
    int col = row;
    double mv = fabs(A[row][col]);
    int mr = row;
    for (int i = row + 1; i < 5; ++i) { double v = fabs(A[i][col]); if (v > mv) { mv = v; mr = i; } }
    if (row != mr) {
      for (int j = col; j < 5; ++j) std::swap(A[row][j], A[mr][j]);
      std::swap(b[row], b[mr]);
    }
    for (int i = row + 1; i < 5; ++i) {
      double f = A[i][col] / A[row][col];
      for (int j = row + 1; j < 5; ++j) A[i][j] -= f * A[row][j];
      b[i] -= f * b[row];
    }
  }
  for (int i = 4; i >= 0; --i) {
    for (int j = i + 1; j < 5; ++j) b[i] -= A[i][j] * b[j];
    b[i] /= A[i][i];
  }
}

void orc_decompose(const double* E_in, double* params) {
  double E[3][3];
  memcpy(E, E_in, sizeof(E));
  double p[10];
  givens_params(E, p);
  params[0] = atan2(p[1], p[0]);
  params[1] = atan2(p[3], p[2]);
  params[2] = atan2(p[5], p[4]);
  params[3] = atan2(p[7], p[6]);
  params[4] = atan2(p[9], p[8]);
}

void orc_decompose_uv(const double* E_in, double* U_out, double* V_out) {
  double E[3][3], U[3][3], V[3][3];
  memcpy(E, E_in, sizeof(E));
  decompose_uv(E, U, V);
  memcpy(U_out, U, sizeof(U));
  memcpy(V_out, V, sizeof(V));
}

// polish_E_robust_parametric (polish_E.cu:1470-1577)
void orc_optimise(const double* pin, const double* qin, int64_t n, const double* E_init,
                  double delta, double alpha, int max_reps, double* E_out) {
  double E[3][3], U[3][3], V[3][3];
  memcpy(E, E_init, sizeof(E));
  decompose_uv(E, U, V);   // leaves E partially reduced, as the reference does
  std::vector<double> p((size_t)n * 3), qq((size_t)n * 3), w((size_t)n);
  for (int rep = 0;; ++rep) {
    for (int64_t i = 0; i < n; ++i)
      for (int j = 0; j < 3; ++j) {
        p[3 * i + j] = pin[2 * i] * V[0][j] + pin[2 * i + 1] * V[1][j] + 1.0 * V[2][j];
        qq[3 * i + j] = qin[2 * i] * U[0][j] + qin[2 * i + 1] * U[1][j] + 1.0 * U[2][j];
      }
    double g[5] = {0, 0, 0, 0, 0};
    for (int64_t k = 0; k < n; ++k) {
      const double* pk = &p[3 * k];
      const double* qk = &qq[3 * k];
      double e = pk[0] * qk[0] + pk[1] * qk[1];
      w[k] = (fabs(e) < delta) ? 1.0 : alpha * delta / fabs(e);
      g[0] += -pk[1] * qk[2] * -e * w[k];
      g[1] += -pk[0] * qk[2] * -e * w[k];
      g[2] += (pk[1] * qk[0] - pk[0] * qk[1]) * -e * w[k];
      g[3] += -pk[2] * qk[1] * -e * w[k];
      g[4] += -pk[2] * qk[0] * -e * w[k];
    }
    double emag = 0.0;
    for (int i = 0; i < 5; ++i) emag += g[i] * g[i];
    if (emag < 1e-20) break;
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) E[i][j] = U[i][0] * V[j][0] + U[i][1] * V[j][1];
    if (rep == max_reps) break;
    double H[5][5];
    for (int i = 0; i < 5; ++i) for (int j = 0; j < 5; ++j) H[i][j] = 0.0;
    for (int64_t k = 0; k < n; ++k) {
      const double* pk = &p[3 * k];
      const double* qk = &qq[3 * k];
      double J[5];
      J[0] = -pk[1] * qk[2];
      J[1] = -pk[0] * qk[2];
      J[2] = pk[1] * qk[0] - pk[0] * qk[1];
      J[3] = -pk[2] * qk[1];
      J[4] = -pk[2] * qk[0];
      for (int i = 0; i < 5; ++i) for (int j = 0; j < 5; ++j) H[i][j] += w[k] * J[i] * J[j];
    }
    solve5(H, g);
    rotate_cols(U, 0, 1, g[2]);
    rotate_cols(U, 0, 2, g[1]);
    rotate_cols(U, 1, 2, g[0]);
    rotate_cols(V, 1, 2, g[3]);
    rotate_cols(V, 0, 2, g[4]);
  }
  memcpy(E_out, E, sizeof(E));
}

}  // extern "C"
