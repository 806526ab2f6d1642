// Device-side five-point essential-matrix solver for CDNA4 (gfx950).
//
// One lane solves one RANSAC hypothesis.  The floating-point operation order of
// every step follows the reference solver (RANSAC_FiveP/essential_matrix/
// essential_matrix_5pt.cu, sturm.cu, cheirality.cu) so that, compiled with
// -ffp-contract=off, the essential matrices are bit-identical to the
// reference's; the DATA LAYOUT is GPU-first:
//   * symmetric polynomial products are stored packed (10 quadratic / 20 cubic
//     monomials) instead of dense 4x4 / 4x4x4 arrays;
//   * the 5x10x10 equation tensor is split per w-degree into the structurally
//     non-zero blocks only (203 doubles instead of 500);
//   * the Sturm sequence uses 11 polynomials of 11 coefficients (degree 10);
//   * the recursive bisection (sbisect<depth>) is an explicit work stack.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sfm {

// ---------------------------------------------------------------------------
// Packed monomial index tables (compile-time)
// ---------------------------------------------------------------------------
// quadratic monomials (a<=b), lexicographic: 00 01 02 03 11 12 13 22 23 33
__host__ __device__ constexpr int q_idx(int a, int b) {
  return a == 0 ? b : a == 1 ? 3 + b : a == 2 ? 5 + b : 9;
}
// cubic monomials (a<=b<=c), lexicographic
__host__ __device__ constexpr int c_idx(int a, int b, int c) {
  // offsets of the a-blocks: a=0 -> 0 (10 entries), a=1 -> 10 (6), a=2 -> 16 (3), a=3 -> 19
  return a == 0 ? q_idx(b, c) : a == 1 ? 10 + (q_idx(b, c) - 4) : a == 2 ? 16 + (q_idx(b, c) - 7) : 19;
}

struct Lin { double c[4]; };    // a*w + b*x + c*y + d
struct Quad { double c[10]; };
struct Cubic { double c[20]; };

// Lin x Lin (poly4_1::operator*, essential_matrix_5pt.cu:26-62)
__device__ __forceinline__ Quad qmul(const Lin& a, const Lin& b) {
  Quad r;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = i; j < 4; ++j)
      r.c[q_idx(i, j)] = (i == j) ? a.c[i] * b.c[j] : a.c[i] * b.c[j] + a.c[j] * b.c[i];
  return r;
}

// Quad x Lin (poly4_2::operator*, essential_matrix_5pt.cu:64-120): quadratic
// monomials in lexicographic order, w..z inner; the first contribution to a
// cubic monomial assigns it, later ones accumulate.
struct CubicTerm { int8_t target; int8_t first; };
struct CubicTable { CubicTerm t[10][4]; };
__host__ __device__ constexpr CubicTable make_cubic_table() {
  CubicTable tb{};
  bool seen[20] = {};
  for (int i = 0; i < 4; ++i)
    for (int j = i; j < 4; ++j)
      for (int k = 0; k < 4; ++k) {
        int t = (k < i) ? c_idx(k, i, j) : (k <= j) ? c_idx(i, k, j) : c_idx(i, j, k);
        tb.t[q_idx(i, j)][k].target = (int8_t)t;
        tb.t[q_idx(i, j)][k].first = seen[t] ? 0 : 1;
        seen[t] = true;
      }
  return tb;
}

__device__ __forceinline__ Cubic cmul(const Quad& a, const Lin& b) {
  constexpr CubicTable tb = make_cubic_table();
  Cubic r;
#pragma unroll
  for (int p = 0; p < 10; ++p)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double v = a.c[p] * b.c[k];
      if (tb.t[p][k].first) r.c[tb.t[p][k].target] = v;
      else r.c[tb.t[p][k].target] += v;
    }
  return r;
}

// ---------------------------------------------------------------------------
// Equation set, split per degree in w (EquationSet, common.h)
//   e0[10][10] w^0 (all 10 monomials), e1[10][6] w^1, e2[10][3] w^2,
//   e3[10] w^3 (constant monomial), e4[3] w^4 (created by the reduction)
// ---------------------------------------------------------------------------
struct Eqs {
  double e0[10][10];
  double e1[10][6];
  double e2[10][3];
  double e3[10][3];   // only column 0 is a genuine unknown before reduction;
                      // columns 1,2 of rows 0-2 receive fill-in at the end
  double e4[3];
};

// mono_coeff (essential_matrix_5pt.cu:356-426); monomials 0 1 x 2 y 3 xx 4 xy
// 5 yy 6 xxx 7 xxy 8 xyy 9 yyy with (w,x,y,z) = (0,1,2,3)
__device__ __forceinline__ void put_equation(const Cubic& B, Eqs& A, int n) {
  A.e0[n][0] = B.c[c_idx(3, 3, 3)]; A.e0[n][1] = B.c[c_idx(1, 3, 3)]; A.e0[n][2] = B.c[c_idx(2, 3, 3)];
  A.e0[n][3] = B.c[c_idx(1, 1, 3)]; A.e0[n][4] = B.c[c_idx(1, 2, 3)]; A.e0[n][5] = B.c[c_idx(2, 2, 3)];
  A.e0[n][6] = B.c[c_idx(1, 1, 1)]; A.e0[n][7] = B.c[c_idx(1, 1, 2)]; A.e0[n][8] = B.c[c_idx(1, 2, 2)];
  A.e0[n][9] = B.c[c_idx(2, 2, 2)];
  A.e1[n][0] = B.c[c_idx(0, 3, 3)]; A.e1[n][1] = B.c[c_idx(0, 1, 3)]; A.e1[n][2] = B.c[c_idx(0, 2, 3)];
  A.e1[n][3] = B.c[c_idx(0, 1, 1)]; A.e1[n][4] = B.c[c_idx(0, 1, 2)]; A.e1[n][5] = B.c[c_idx(0, 2, 2)];
  A.e2[n][0] = B.c[c_idx(0, 0, 3)]; A.e2[n][1] = B.c[c_idx(0, 0, 1)]; A.e2[n][2] = B.c[c_idx(0, 0, 2)];
  A.e3[n][0] = B.c[c_idx(0, 0, 0)]; A.e3[n][1] = 0.0; A.e3[n][2] = 0.0;
}

// Null-space basis of the 5x9 epipolar system (Ematrix_5pt +
// null_space_solve_5x9, essential_matrix_5pt.cu:631-711): modified
// Gram-Schmidt with 4 deterministic filler rows; rows 5..8 -> basis.
__device__ __forceinline__ void essential_basis(const double q[5][2], const double qp[5][2], Lin Eb[9]) {
  double M[9][9];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const double a[3] = {qp[i][0], qp[i][1], 1.0};
    const double b[3] = {q[i][0], q[i][1], 1.0};
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) M[i][3 * r + s] = a[r] * b[s];
  }
  const double PPi = 3.18730379;
  double ran = PPi;
#pragma unroll
  for (int i = 5; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      ran *= PPi;
      ran = 2.0 * (ran - floor(ran)) - 1.0;
      M[i][j] = ran;
    }
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    double ss = 0.0;
#pragma unroll
    for (int j = 0; j < 9; ++j) ss += M[r][j] * M[r][j];
    const double f = 1.0 / sqrt(ss);
#pragma unroll
    for (int j = 0; j < 9; ++j) M[r][j] *= f;
#pragma unroll
    for (int i = r + 1; i < 9; ++i) {
      double dot = 0.0;
#pragma unroll
      for (int j = 0; j < 9; ++j) dot += M[r][j] * M[i][j];
#pragma unroll
      for (int j = 0; j < 9; ++j) M[i][j] -= dot * M[r][j];
    }
  }
#pragma unroll
  for (int e = 0; e < 9; ++e) { Eb[e].c[0] = M[5][e]; Eb[e].c[1] = M[6][e]; Eb[e].c[2] = M[7][e]; Eb[e].c[3] = M[8][e]; }
}

// Constraint equations (EEeqns_5pt, essential_matrix_5pt.cu:428-474), in
// three parts so that a DPP quad can share them (build_equations_quad):
// trace(E E^T), row-major element order (traceEEt)
__device__ __forceinline__ Quad trace_eet(const Lin Eb[9]) {
  Quad tr = qmul(Eb[0], Eb[0]);
#pragma unroll
  for (int e = 1; e < 9; ++e) {
    Quad s = qmul(Eb[e], Eb[e]);
#pragma unroll
    for (int k = 0; k < 10; ++k) tr.c[k] = tr.c[k] + s.c[k];
  }
  return tr;
}

// equation 0: det(E) by cofactors of column 0 (polydet4)
__device__ __forceinline__ void det_equation(const Lin Eb[9], Eqs& A) {
  Cubic d[3];
  const int rows[3][4] = {{4, 8, 7, 5}, {7, 2, 1, 8}, {1, 5, 4, 2}};  // (a*b - c*d)
  const int col0[3] = {0, 3, 6};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    Quad m1 = qmul(Eb[rows[t][0]], Eb[rows[t][1]]);
    Quad m2 = qmul(Eb[rows[t][2]], Eb[rows[t][3]]);
    Quad df;
#pragma unroll
    for (int k = 0; k < 10; ++k) df.c[k] = m1.c[k] - m2.c[k];
    d[t] = cmul(df, Eb[col0[t]]);
  }
  Cubic det;
#pragma unroll
  for (int k = 0; k < 20; ++k) det.c[k] = (d[0].c[k] + d[1].c[k]) + d[2].c[k];
  put_equation(det, A, 0);
}

// equations 1 + 3i .. 3 + 3i: row i of 2 E E^T E - tr(E E^T) E = 0, with
// Ei[p] = Eb[3i + p] (the row's three entries)
__device__ __forceinline__ void row_equations(const Lin Eb[9], const Lin Ei[3], const Quad& tr, Eqs& A, int i) {
  Cubic acc[3];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int k = 0; k < 20; ++k) acc[j].c[k] = 0.0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    Quad eet;
#pragma unroll
    for (int k = 0; k < 10; ++k) eet.c[k] = 0.0;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      Quad s = qmul(Ei[p], Eb[3 * q + p]);
#pragma unroll
      for (int k = 0; k < 10; ++k) eet.c[k] += s.c[k];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      Cubic s = cmul(eet, Eb[3 * q + j]);
#pragma unroll
      for (int k = 0; k < 20; ++k) acc[j].c[k] += s.c[k];
    }
  }
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    Cubic t = cmul(tr, Ei[j]);
    Cubic r;
#pragma unroll
    for (int k = 0; k < 20; ++k) r.c[k] = acc[j].c[k] * 2.0 - t.c[k];
    put_equation(r, A, 1 + 3 * i + j);
  }
}

__device__ __forceinline__ void build_equations(const Lin Eb[9], Eqs& A) {
  const Quad tr = trace_eet(Eb);
  det_equation(Eb, A);
#pragma unroll
  for (int i = 0; i < 3; ++i) row_equations(Eb, &Eb[3 * i], tr, A, i);
}

// The same ten equations from a DPP quad holding the same Eb on every lane:
// lane 0 writes equation 0, lane s = 1..3 the row i = s - 1 block (its rows
// selected by value, so every index stays static).  Same operations per
// equation as build_equations; the caller synchronises before reading A.
__device__ __forceinline__ void build_equations_quad(const Lin Eb[9], Eqs& A, int s) {
  if (s == 0) {
    det_equation(Eb, A);
  } else {
    const int i = s - 1;
    Lin Ei[3];
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int c = 0; c < 4; ++c) Ei[p].c[c] = i == 0 ? Eb[p].c[c] : i == 1 ? Eb[3 + p].c[c] : Eb[6 + p].c[c];
    row_equations(Eb, Ei, trace_eet(Eb), A, i);
  }
}

// Row operation: row[target] -= fac * row[prow] on the non-zero column blocks
// (sweep_up / sweep_down, essential_matrix_5pt.cu:713-779)
__device__ __forceinline__ void row_axpy(Eqs& A, int prow, int target, int lim0, double fac) {
#pragma unroll
  for (int j = 0; j <= lim0; ++j) A.e0[target][j] -= fac * A.e0[prow][j];
#pragma unroll
  for (int j = 0; j < 6; ++j) A.e1[target][j] -= fac * A.e1[prow][j];
#pragma unroll
  for (int j = 0; j < 3; ++j) A.e2[target][j] -= fac * A.e2[prow][j];
  A.e3[target][0] -= fac * A.e3[prow][0];
}

__device__ __forceinline__ void swap_d(double& a, double& b) { double t = a; a = b; b = t; }

// Partial pivoting on column `last` of the w^0 block (pivot, 801-848)
__device__ __forceinline__ void pivot_rows(Eqs& A, int last) {
  double best = fabs(A.e0[last][last]);
  int r = last;
#pragma unroll
  for (int i = 0; i < last; ++i)
    if (fabs(A.e0[i][last]) > best) { r = i; best = fabs(A.e0[i][last]); }
  if (r == last) return;
#pragma unroll
  for (int j = 0; j <= last; ++j) swap_d(A.e0[last][j], A.e0[r][j]);
#pragma unroll
  for (int j = 0; j < 6; ++j) swap_d(A.e1[last][j], A.e1[r][j]);
#pragma unroll
  for (int j = 0; j < 3; ++j) swap_d(A.e2[last][j], A.e2[r][j]);
  swap_d(A.e3[last][0], A.e3[r][0]);
}

// One elimination column of the sweep-up with every index static (the set
// lives in LDS: dynamic bounds left each row_axpy a loop of dependent LDS
// round trips, 55 % of k_solve_front's cycles).  The pivot row is read once
// into registers; rows i < C never write it, so every element sees the same
// operations in the same order as row_axpy (bit-identical).
template <int C>
__device__ __forceinline__ void eliminate_up(Eqs& A) {
  pivot_rows(A, C);
  const double pv = A.e0[C][C];
  double p0[C + 1], p1[6], p2[3];
#pragma unroll
  for (int j = 0; j <= C; ++j) p0[j] = A.e0[C][j];
#pragma unroll
  for (int j = 0; j < 6; ++j) p1[j] = A.e1[C][j];
#pragma unroll
  for (int j = 0; j < 3; ++j) p2[j] = A.e2[C][j];
  const double p3 = A.e3[C][0];
#pragma unroll
  for (int i = 0; i < C; ++i) {
    const double fac = A.e0[i][C] / pv;
#pragma unroll
    for (int j = 0; j <= C; ++j) A.e0[i][j] -= fac * p0[j];
#pragma unroll
    for (int j = 0; j < 6; ++j) A.e1[i][j] -= fac * p1[j];
#pragma unroll
    for (int j = 0; j < 3; ++j) A.e2[i][j] -= fac * p2[j];
    A.e3[i][0] -= fac * p3;
  }
}

// the last step of reduce_Ematrix: raise the degree to eliminate the x terms
__device__ __forceinline__ void raise_degree(Eqs& A) {
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const double f = A.e1[i][3 + i] / A.e0[3 + i][3 + i];
    A.e4[i] = -A.e3[i + 3][0] * f;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      A.e3[i][j] -= A.e2[i + 3][j] * f;
      A.e2[i][j] -= A.e1[i + 3][j] * f;
      A.e1[i][j] -= A.e0[i + 3][j] * f;
    }
  }
}

// reduce_Ematrix (essential_matrix_5pt.cu:852-900)
__device__ __forceinline__ void reduce_equations(Eqs& A) {
  eliminate_up<9>(A);
  eliminate_up<8>(A);
  eliminate_up<7>(A);
  eliminate_up<6>(A);
  eliminate_up<5>(A);
  eliminate_up<4>(A);
  eliminate_up<3>(A);
  // sweep_down on the w^0 block, rows 3 and 4
#pragma unroll
  for (int r = 3; r <= 4; ++r) {
    const double pv = A.e0[r][r];
#pragma unroll
    for (int i = r + 1; i <= 5; ++i) row_axpy(A, r, i, r, A.e0[i][r] / pv);
  }
  // sweep_up on the w^1 block: (row 2, col 5) then (row 1, col 4)
  {
    const double pv = A.e1[2][5];
    for (int i = 0; i < 2; ++i) row_axpy(A, 2, i, 5, A.e1[i][5] / pv);
  }
  {
    const double pv = A.e1[1][4];
    row_axpy(A, 1, 0, 4, A.e1[0][4] / pv);
  }
  // sweep_down on the w^1 block: (0,3), (1,4), (2,5)
  for (int r = 0; r < 3; ++r) {
    const double pv = A.e1[r][3 + r];
    for (int i = r + 1; i <= 5; ++i) row_axpy(A, r, i, 3 + r, A.e1[i][3 + r] / pv);
  }
  raise_degree(A);
}

// ---------------------------------------------------------------------------
// Cooperative reduction: one DPP quad (4 lanes) per hypothesis
// ---------------------------------------------------------------------------
// With one lane per hypothesis the reduction was 54 % of k_solve_front's
// cycles (git-history scripts/front_stats.py): dependent LDS round trips and divisions on
// waves with 16 of 64 lanes active.  Here the quad holds the ten rows'
// 20-column vector in registers, lane s the columns k = s + 4m (m < 5):
//   k 0..9 -> e0[.][k], 10..15 -> e1[.][k-10], 16..18 -> e2[.][k-16], 19 -> e3[.][0]
// (e3's other columns and e4 first change in raise_degree, which runs on the
// record afterwards).  Column values the pivot search and the factors need are
// broadcast within the quad by DPP; every lane divides (same operands, same
// bits) and updates its own columns.  Each element sees reduce_equations'
// operations in its order, so the record is bit-identical.
template <int O>
__device__ __forceinline__ int quad_bcast_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, O | (O << 2) | (O << 4) | (O << 6), 0xf, 0xf, false);
}

template <int O>
__device__ __forceinline__ double quad_bcast(double v) {
  const unsigned long long u = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)quad_bcast_i<O>((int)(unsigned)u);
  const unsigned hi = (unsigned)quad_bcast_i<O>((int)(unsigned)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// column k's value in row i, from the quad lane that holds it
template <int K>
__device__ __forceinline__ double quad_col(const double (&R)[10][5], int i) {
  return quad_bcast<K & 3>(R[i][K >> 2]);
}

// does this lane's slot m carry a column row_axpy touches at e0 limit LIM?
__device__ __forceinline__ bool quad_in(int s, int m, int lim) {
  const int k = s + 4 * m;
  return k > 9 || k <= lim;
}

// rows [I0, I1) -= (row[i][K] / row[PROW][K]) * row PROW   (row_axpy, e0 limit LIM)
template <int PROW, int K, int I0, int I1, int LIM>
__device__ __forceinline__ void quad_axpy(double (&R)[10][5], int s) {
  const double pv = quad_col<K>(R, PROW);
  double pr[5];
#pragma unroll
  for (int m = 0; m < 5; ++m) pr[m] = R[PROW][m];
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const double fac = quad_col<K>(R, i) / pv;
#pragma unroll
    for (int m = 0; m < 5; ++m)
      if (quad_in(s, m, LIM)) R[i][m] -= fac * pr[m];
  }
}

// pivot_rows + the sweep-up of column C (eliminate_up<C>)
template <int C>
__device__ __forceinline__ void quad_eliminate_up(double (&R)[10][5], int s) {
  constexpr int M = C >> 2;
  double best = fabs(R[C][M]);
  int r = C;
#pragma unroll
  for (int i = 0; i < C; ++i)
    if (fabs(R[i][M]) > best) { r = i; best = fabs(R[i][M]); }
  r = quad_bcast_i<C & 3>(r);                  // the search on the lane holding column C
  if (r != C) {
#pragma unroll
    for (int i = 0; i < C; ++i)
      if (i == r) {
#pragma unroll
        for (int m = 0; m < 5; ++m)
          if (quad_in(s, m, C)) { const double t = R[C][m]; R[C][m] = R[i][m]; R[i][m] = t; }
      }
  }
  quad_axpy<C, C, 0, C, C>(R, s);
}

__device__ __forceinline__ int quad_field(int i, int k) {   // offset in the record, in doubles
  return k < 10 ? i * 10 + k : k < 16 ? 100 + i * 6 + (k - 10) : k < 19 ? 160 + i * 3 + (k - 16) : 190 + i * 3;
}

// reduce_equations up to (not including) raise_degree, on the record `A`
// shared by the quad (LDS); lane s = lane & 3.  Callers synchronise the
// record's writers before and its readers after.
__device__ __forceinline__ void quad_reduce(Eqs& A, int s) {
  static_assert(sizeof(Eqs) == 223 * sizeof(double), "record layout");
  double* f = reinterpret_cast<double*>(&A);
  double R[10][5];
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int m = 0; m < 5; ++m) R[i][m] = f[quad_field(i, s + 4 * m)];
  quad_eliminate_up<9>(R, s);
  quad_eliminate_up<8>(R, s);
  quad_eliminate_up<7>(R, s);
  quad_eliminate_up<6>(R, s);
  quad_eliminate_up<5>(R, s);
  quad_eliminate_up<4>(R, s);
  quad_eliminate_up<3>(R, s);
  // sweep_down on the w^0 block, rows 3 and 4
  quad_axpy<3, 3, 4, 6, 3>(R, s);
  quad_axpy<4, 4, 5, 6, 4>(R, s);
  // sweep_up on the w^1 block: (row 2, col 5) then (row 1, col 4)
  quad_axpy<2, 15, 0, 2, 5>(R, s);
  quad_axpy<1, 14, 0, 1, 4>(R, s);
  // sweep_down on the w^1 block: (0,3), (1,4), (2,5)
  quad_axpy<0, 13, 1, 6, 3>(R, s);
  quad_axpy<1, 14, 2, 6, 4>(R, s);
  quad_axpy<2, 15, 3, 6, 5>(R, s);
#pragma unroll
  for (int i = 0; i < 10; ++i)
#pragma unroll
    for (int m = 0; m < 5; ++m) f[quad_field(i, s + 4 * m)] = R[i][m];
}

// degree-w entry accessor for the reduced 3x3 block
__device__ __forceinline__ double coef(const Eqs& A, int deg, int r, int c) {
  switch (deg) {
    case 0: return A.e0[r][c];
    case 1: return A.e1[r][c];
    case 2: return A.e2[r][c];
    case 3: return A.e3[r][c];
    default: return c == 0 ? A.e4[r] : 0.0;
  }
}

// Degree-10 determinant polynomial (compute_determinant / one_cofactor, 902-948)
__device__ __forceinline__ void determinant_poly(const Eqs& A, double poly[11]) {
#pragma unroll
  for (int i = 0; i <= 10; ++i) poly[i] = 0.0;
  const int rr[3][3] = {{0, 1, 2}, {1, 2, 0}, {2, 0, 1}};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int r0 = rr[t][0], r1 = rr[t][1], r2 = rr[t][2];
    double m[7];
#pragma unroll
    for (int i = 0; i < 7; ++i) m[i] = 0.0;
#pragma unroll
    for (int i = 0; i <= 3; ++i)
#pragma unroll
      for (int j = 0; j <= 3; ++j)
        m[i + j] += coef(A, i, r1, 1) * coef(A, j, r2, 2) - coef(A, i, r2, 1) * coef(A, j, r1, 2);
#pragma unroll
    for (int i = 0; i <= 6; ++i)
#pragma unroll
      for (int j = 0; j <= 4; ++j) poly[i + j] += coef(A, j, r0, 0) * m[i];
  }
}

// ---------------------------------------------------------------------------
// Sturm-sequence real roots (sturm.cu)
// ---------------------------------------------------------------------------
constexpr double kRelErr = 1.0e-12;
constexpr int kMaxPow = 32;
constexpr int kMaxIt = 800;
constexpr int kMaxDepth = 10;
constexpr double kSmall = 1.0e-12;

struct Sturm {
  int ord[11];
  double c[11][11];
};

__device__ __forceinline__ double horner(int ord, const double* c, double x) {
  double f = c[ord];
  for (int i = ord - 1; i >= 0; --i) f = x * f + c[i];
  return f;
}

// modrf_pos (sturm.cu:43-207)
__device__ int falsi(const double* c, double a, double b, double* val, bool inv) {
  const int ord = 10;
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
    const double x = (fb * a - fa * b) / (fb - fa);
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

// modrf (sturm.cu:218-275), leading coefficient omitted at +-1 as in the reference
__device__ int falsi_any(const double* c, double a, double b, double* val) {
  if (a > b) { double t = a; a = b; b = t; }
  if (b <= 1.0 && a >= -1.0) return falsi(c, a, b, val, false);
  if (a >= 1.0 || b <= -1.0) return falsi(c, a, b, val, true);
  double fp1 = 0.0, fm1 = 0.0, fa = 0.0, fb = 0.0;
  for (int i = 9; i >= 0; --i) {
    fp1 = c[i] + fp1;
    fm1 = c[i] - fm1;
    fa = a * fa + c[i];
    fb = b * fb + c[i];
  }
  if (a < -1.0 && b > 1.0) {
    if (fa * fm1 < 0.0) return falsi(c, a, -1.0, val, true);
    if (fb * fp1 < 0.0) return falsi(c, 1.0, b, val, true);
    return falsi(c, -1.0, 1.0, val, false);
  }
  if (a < -1.0) {
    if (fa * fm1 < 0.0) return falsi(c, a, -1.0, val, true);
    return falsi(c, -1.0, b, val, false);
  }
  if (fb * fp1 < 0.0) return falsi(c, 1.0, b, val, true);
  return falsi(c, a, 1.0, val, false);
}

// modp (sturm.cu:285-322): remainder of s[u] / s[v] into s[r]
__device__ int remainder_into(Sturm& S, int u, int v, int r) {
  const int uo = S.ord[u], vo = S.ord[v];
  for (int i = 0; i <= uo; ++i) S.c[r][i] = S.c[u][i];
  if (S.c[v][vo] < 0.0) {
    for (int k = uo - vo - 1; k >= 0; k -= 2) S.c[r][k] = -S.c[r][k];
    for (int k = uo - vo; k >= 0; --k)
      for (int j = vo + k - 1; j >= k; --j) S.c[r][j] = -S.c[r][j] - S.c[r][vo + k] * S.c[v][j - k];
  } else {
    for (int k = uo - vo; k >= 0; --k)
      for (int j = vo + k - 1; j >= k; --j) S.c[r][j] -= S.c[r][vo + k] * S.c[v][j - k];
  }
  int k = vo - 1;
  while (k >= 0 && fabs(S.c[r][k]) < kSmall) { S.c[r][k] = 0.0; --k; }
  S.ord[r] = (k < 0) ? 0 : k;
  return S.ord[r];
}

// buildsturm (sturm.cu:331-360)
__device__ int build_sturm(Sturm& S) {
  const int ord = 10;
  S.ord[0] = ord;
  S.ord[1] = ord - 1;
  const double f = fabs(S.c[0][ord] * ord);
  for (int i = 1; i <= ord; ++i) S.c[1][i - 1] = S.c[0][i] * i / f;
  int k = 2;
  while (k <= 10 && remainder_into(S, k - 2, k - 1, k)) {
    const double g = -fabs(S.c[k][S.ord[k]]);
    for (int i = S.ord[k]; i >= 0; --i) S.c[k][i] /= g;
    ++k;
  }
  S.c[k][0] = -S.c[k][0];
  return k;
}

// numchanges (sturm.cu:369-385)
__device__ int sign_changes(const Sturm& S, int np, double a) {
  int ch = 0;
  double lf = horner(S.ord[0], S.c[0], a);
  for (int i = 1; i <= np; ++i) {
    const double f = horner(S.ord[i], S.c[i], a);
    if (lf == 0.0 || lf * f < 0) ++ch;
    lf = f;
  }
  return ch;
}

// numroots (sturm.cu:393-439), non_neg = false
__device__ int count_real_roots(const Sturm& S, int np, int* atneg, int* atpos) {
  int pos = 0, neg = 0;
  double lf = S.c[0][S.ord[0]];
  for (int i = 1; i <= np; ++i) {
    const double f = S.c[i][S.ord[i]];
    if (lf == 0.0 || lf * f < 0) ++pos;
    lf = f;
  }
  lf = (S.ord[0] & 1) ? -S.c[0][S.ord[0]] : S.c[0][S.ord[0]];
  for (int i = 1; i <= np; ++i) {
    const double f = (S.ord[i] & 1) ? -S.c[i][S.ord[i]] : S.c[i][S.ord[i]];
    if (lf == 0.0 || lf * f < 0) ++neg;
    lf = f;
  }
  *atneg = neg;
  *atpos = pos;
  return neg - pos;
}

// sbisect<depth> (sturm.cu:450-555) as an explicit depth-first work stack
__device__ void isolate(const Sturm& S, int np, double lo, double hi, int atlo, int athi, double roots[10]) {
  struct Iv { double lo, hi; int atlo, athi, off, depth; };
  Iv stk[24];
  int sp = 0;
  stk[sp++] = Iv{lo, hi, atlo, athi, 0, 0};
  while (sp > 0) {
    const Iv iv = stk[--sp];
    if (iv.depth >= kMaxDepth) continue;
    double mn = iv.lo, mx = iv.hi, mid = 0.0;
    if (iv.atlo - iv.athi == 1) {
      double v;
      if (falsi_any(S.c[0], mn, mx, &v)) {
        if (iv.off >= 0 && iv.off < 10) roots[iv.off] = v;
        continue;
      }
      for (int it = 0; it < kMaxIt; ++it) {
        mid = (double)((mn + mx) / 2);
        const int atmid = sign_changes(S, np, mid);
        if (fabs(mid) > kRelErr) {
          if (fabs((mx - mn) / mid) < kRelErr) break;
        } else if (fabs(mx - mn) < kRelErr) break;
        if ((iv.atlo - atmid) == 0) mn = mid; else mx = mid;
      }
      if (iv.off >= 0 && iv.off < 10) roots[iv.off] = mid;
      continue;
    }
    int it;
    for (it = 0; it < kMaxIt; ++it) {
      mid = (double)((mn + mx) / 2);
      const int atmid = sign_changes(S, np, mid);
      const int n1 = iv.atlo - atmid, n2 = atmid - iv.athi;
      if (n1 != 0 && n2 != 0) {
        if (sp + 2 <= 24) {
          stk[sp++] = Iv{mid, mx, atmid, iv.athi, iv.off + n1, iv.depth + 1};
          stk[sp++] = Iv{mn, mid, iv.atlo, atmid, iv.off, iv.depth + 1};
        }
        break;
      }
      if (n1 == 0) mn = mid; else mx = mid;
    }
    if (it == kMaxIt)
      for (int r = iv.athi; r < iv.atlo; ++r) {
        const int slot = iv.off + r - iv.athi;
        if (slot >= 0 && slot < 10) roots[slot] = mid;
      }
  }
}

// x^y for the root-scaling step of find_real_roots_sturm (sturm.cu:580),
// correctly rounded via double-double log/exp (host libm pow is <=0.52 ulp,
// so this agrees with it except in rare hard cases).
struct dd { double hi, lo; };
__device__ __forceinline__ dd dd_two_sum(double a, double b) {
  double s = a + b, bb = s - a;
  return dd{s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd dd_add(dd a, dd b) {
  dd s = dd_two_sum(a.hi, b.hi);
  dd t = dd_two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = dd_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return dd_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ dd dd_mul(dd a, dd b) {
  double p = a.hi * b.hi;
  double e = fma(a.hi, b.hi, -p);
  e += a.hi * b.lo + a.lo * b.hi;
  return dd_two_sum(p, e);
}
__device__ __forceinline__ dd dd_mul_d(dd a, double b) {
  double p = a.hi * b;
  double e = fma(a.hi, b, -p);
  e += a.lo * b;
  return dd_two_sum(p, e);
}
__device__ __forceinline__ dd dd_div(dd a, dd b) {
  double q1 = a.hi / b.hi;
  dd r = dd_add(a, dd_mul_d(b, -q1));
  double q2 = r.hi / b.hi;
  r = dd_add(r, dd_mul_d(b, -q2));
  double q3 = r.hi / b.hi;
  return dd_add(dd_two_sum(q1, q2), dd{q3, 0.0});
}
__device__ dd dd_log(double x) {
  int e;
  double m = frexp(x, &e);          // x = m 2^e, m in [0.5, 1)
  if (m < 0.70710678118654752) { m *= 2.0; e -= 1; }
  // log(m) = 2 atanh(s), s = (m-1)/(m+1)
  dd s = dd_div(dd{m - 1.0, 0.0}, dd_two_sum(m, 1.0));   // m-1 exact (Sterbenz)
  dd s2 = dd_mul(s, s);
  dd term = s, sum = s;
  for (int k = 3; k <= 61; k += 2) {
    term = dd_mul(term, s2);
    sum = dd_add(sum, dd_div(term, dd{(double)k, 0.0}));
  }
  const dd ln2 = {0.6931471805599452862, 2.3190468138462996e-17};
  return dd_add(dd_mul_d(sum, 2.0), dd_mul_d(ln2, (double)e));
}
__device__ double dd_exp_round(dd z) {
  const dd ln2 = {0.6931471805599452862, 2.3190468138462996e-17};
  const double k = rint(z.hi / ln2.hi);
  dd r = dd_add(z, dd_mul_d(ln2, -k));
  r = dd_mul_d(r, 1.0 / 1024.0);                 // exact scaling
  dd sum = {1.0, 0.0}, term = {1.0, 0.0};
  for (int n = 1; n <= 14; ++n) {
    term = dd_div(dd_mul(term, r), dd{(double)n, 0.0});
    sum = dd_add(sum, term);
  }
  for (int i = 0; i < 10; ++i) sum = dd_mul(sum, sum);
  return ldexp(sum.hi + sum.lo, (int)k);
}
__device__ double cr_pow(double x, double y) {
  return dd_exp_round(dd_mul_d(dd_log(x), y));
}

// find_real_roots_sturm (sturm.cu:557-676), degree 10, non_neg = false.
// Returns nroots; <= 0 means no valid root.
__device__ int real_roots(const double poly[11], double roots[10]) {
  Sturm S;
  for (int i = 0; i < 11; ++i) { S.ord[i] = 0; for (int j = 0; j < 11; ++j) S.c[i][j] = 0.0; }
  const double norm = 1.0 / poly[10];
  for (int i = 0; i <= 10; ++i) S.c[0][i] = poly[i] * norm;
  const double v0 = fabs(S.c[0][0]);
  double fac = 1.0;
  if (v0 > 10.0) {
    fac = cr_pow(v0, -1.0 / 10);
    double m = fac;
    for (int i = 9; i >= 0; --i) { S.c[0][i] *= m; m = m * fac; }
  }
  const int np = build_sturm(S);
  int atmin, atmax;
  int nr = count_real_roots(S, np, &atmin, &atmax);
  if (nr == 0) return 0;
  double mn = -1.0;
  int nch = sign_changes(S, np, mn);
  for (int i = 0; nch != atmin && i != kMaxPow; ++i) { mn *= 10.0; nch = sign_changes(S, np, mn); }
  if (nch != atmin) atmin = nch;
  double mx = 1.0;
  nch = sign_changes(S, np, mx);
  for (int i = 0; nch != atmax && i != kMaxPow; ++i) { mx *= 10.0; nch = sign_changes(S, np, mx); }
  if (nch != atmax) atmax = nch;
  nr = atmin - atmax;
  if (nr <= 0) return nr;
  isolate(S, np, mn, mx, atmin, atmax, roots);
  for (int i = 0; i < nr && i < 10; ++i) roots[i] /= fac;
  return nr;
}

// ---------------------------------------------------------------------------
// Register-resident Sturm root isolation (used by k_roots).  After
// build_sturm, polynomial i of the sequence has degree ord[i] <= 10 - i, so
// the whole sequence fits a static, zero-padded layout of 66 doubles
// (polynomial i at offset i*(23-i)/2, 11-i slots).  Horner over the padded
// coefficients gives bit-identical values to Horner from ord[i]: the padded
// steps produce x*0 + 0 = +-0 and the first real step (+-0)*x + c = c
// exactly.  Every loop below is fully unrolled over static indices, so the
// coefficients stay in registers instead of scratch (the reference-order
// mul-then-add evaluation is unchanged).
// ---------------------------------------------------------------------------
constexpr int sturm_off(int i) { return i * (23 - i) / 2; }
constexpr int kSturmRegs = sturm_off(11);   // 66

struct SturmR {
  double c[kSturmRegs];
  int ord[11];
  int np;
};

template <int I>
__device__ __forceinline__ double horner_r(const SturmR& S, double x) {
  constexpr int o = sturm_off(I), d = 10 - I;
  double f = S.c[o + d];
#pragma unroll
  for (int j = d - 1; j >= 0; --j) f = x * f + S.c[o + j];
  return f;
}

template <int I>
__device__ __forceinline__ void sign_step(const SturmR& S, double a, double& lf, int& ch) {
  if (I <= S.np) {
    const double f = horner_r<I>(S, a);
    if (lf == 0.0 || lf * f < 0) ++ch;
    lf = f;
  }
}

#ifdef SFM_ROOTS_STATS
// experiment builds only (git-history scripts/roots_stats.py): Sturm-sequence evaluations
// and falsi steps per k_roots thread, indexed by (block, thread)
__device__ unsigned int g_roots_evals[1 << 17];
__device__ unsigned int g_roots_falsi[1 << 17];
#define ROOTS_COUNT(arr) \
  (++arr[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x])
__device__ unsigned long long g_roots_phase[4][1 << 17];   // cycles: scale, build, bracket, isolate
#define ROOTS_PHASE(i, t0)                                                                         \
  do {                                                                                             \
    const unsigned long long t1_ = __builtin_amdgcn_s_memtime();                                   \
    g_roots_phase[i][((size_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x] +=   \
        t1_ - t0;                                                                                  \
    t0 = t1_;                                                                                      \
  } while (0)
#else
#define ROOTS_PHASE(i, t0) ((void)0)
#define ROOTS_COUNT(arr) ((void)0)
#endif

// numchanges (sturm.cu:369-385)
__device__ __forceinline__ int sign_changes_r(const SturmR& S, double a) {
  ROOTS_COUNT(g_roots_evals);
  int ch = 0;
  double lf = horner_r<0>(S, a);
  sign_step<1>(S, a, lf, ch); sign_step<2>(S, a, lf, ch); sign_step<3>(S, a, lf, ch);
  sign_step<4>(S, a, lf, ch); sign_step<5>(S, a, lf, ch); sign_step<6>(S, a, lf, ch);
  sign_step<7>(S, a, lf, ch); sign_step<8>(S, a, lf, ch); sign_step<9>(S, a, lf, ch);
  sign_step<10>(S, a, lf, ch);
  return ch;
}

// The isolation below is force-inlined into its caller: a SturmR passed by
// reference to an outlined call has to live in memory (scratch), and every
// Horner step then waited on it (95 % of k_roots' time).

// Work stack of isolate_r in LDS, one column per lane (stride kStkLanes), so
// that pushes and pops cost an LDS round trip instead of a scratch one.
// Depth-first, a node at depth d is processed with at most one pending sibling
// per level 1..d on the stack, and only nodes at depth < kMaxDepth split, so
// the stack never holds more than kMaxDepth + 1 entries and the capacity test
// below (the reference's 24-entry array) never fails at 12 either.
constexpr int kStkDepth = kMaxDepth + 2;
constexpr int kStkLanes = 32;
struct IsoStack {
  double* lohi;   // [kStkDepth][2][kStkLanes] + lane
  int* ints;      // [kStkDepth][4][kStkLanes] + lane
  __device__ __forceinline__ void put(int i, double lo, double hi, int atlo, int athi, int off, int depth) const {
    lohi[(2 * i) * kStkLanes] = lo;
    lohi[(2 * i + 1) * kStkLanes] = hi;
    ints[(4 * i) * kStkLanes] = atlo;
    ints[(4 * i + 1) * kStkLanes] = athi;
    ints[(4 * i + 2) * kStkLanes] = off;
    ints[(4 * i + 3) * kStkLanes] = depth;
  }
};

// roots[off] = v with static indices (a dynamic index would put roots in scratch)
__device__ __forceinline__ void put_root(double roots[10], int off, double v) {
#pragma unroll
  for (int i = 0; i < 10; ++i)
    if (i == off) roots[i] = v;
}

// sbisect<depth> (sturm.cu:450-555) with modrf (218-275) as a per-lane state
// machine over an explicit depth-first work stack.  Each pass of the loop
// advances every lane by one unit of work: popping an interval (with modrf's
// case analysis and end-point evaluations), one regula-falsi step, or one
// bisection step (one Sturm-sequence evaluation, shared by the single-root and
// multi-root bisections).  A wave's time then follows its longest lane's step
// count; nested loops (falsi and bisection inside the stack loop) made every
// lane wait for the slowest lane's inner loop at each level.  Each lane runs
// exactly the operations of sbisect/modrf in their order: results are
// unchanged (the single-root bisection skips the Sturm evaluation of the step
// that stops it, whose count the reference discards).
__device__ __forceinline__ void isolate_r(const SturmR& S, double lo, double hi, int atlo, int athi, double roots[10],
                                          const IsoStack& stk) {
  constexpr int kPop = 0, kFalsi = 1, kBis1 = 2, kBisN = 3;
  const double* c = S.c;   // s[0] occupies c[0..10]
  int sp = 0;
  stk.put(sp++, lo, hi, atlo, athi, 0, 0);
  int mode = kPop, it = 0;
  int iatlo = 0, iathi = 0, ioff = 0, idepth = 0;
  double mn = 0.0, mx = 0.0, mid = 0.0;
  double fa = 0.0, fb = 0.0, a = 0.0, b = 0.0, lfx = 0.0;
  bool inv = false;
  for (;;) {
    if (mode == kPop) {
      if (sp == 0) break;
      --sp;
      mn = stk.lohi[(2 * sp) * kStkLanes];
      mx = stk.lohi[(2 * sp + 1) * kStkLanes];
      iatlo = stk.ints[(4 * sp) * kStkLanes];
      iathi = stk.ints[(4 * sp + 1) * kStkLanes];
      ioff = stk.ints[(4 * sp + 2) * kStkLanes];
      idepth = stk.ints[(4 * sp + 3) * kStkLanes];
      if (idepth >= kMaxDepth) continue;
      it = 0;
      if (iatlo - iathi != 1) {
        mode = kBisN;
      } else {
        // modrf (sturm.cu:218-275): pick (a, b, inverted), then modrf_pos's
        // end-point evaluations (sturm.cu:43-80)
        a = mn;
        b = mx;
        if (a > b) { const double t = a; a = b; b = t; }
        if (b <= 1.0 && a >= -1.0) {
          inv = false;
        } else if (a >= 1.0 || b <= -1.0) {
          inv = true;
        } else {
          double fp1 = 0.0, fm1 = 0.0, ga = 0.0, gb = 0.0;
#pragma unroll
          for (int i = 9; i >= 0; --i) {
            fp1 = c[i] + fp1;
            fm1 = c[i] - fm1;
            ga = a * ga + c[i];
            gb = b * gb + c[i];
          }
          if (a < -1.0 && b > 1.0) {
            if (ga * fm1 < 0.0) { b = -1.0; inv = true; }
            else if (gb * fp1 < 0.0) { a = 1.0; inv = true; }
            else { a = -1.0; b = 1.0; inv = false; }
          } else if (a < -1.0) {
            if (ga * fm1 < 0.0) { b = -1.0; inv = true; }
            else { a = -1.0; inv = false; }
          } else {
            if (gb * fp1 < 0.0) { a = 1.0; inv = true; }
            else { b = 1.0; inv = false; }
          }
        }
        if (inv) { const double t = a; a = 1.0 / b; b = 1.0 / t; }
        if (inv) {
          fa = fb = c[0];
#pragma unroll
          for (int i = 1; i <= 10; ++i) { fa = a * fa + c[i]; fb = b * fb + c[i]; }
        } else {
          fa = fb = c[10];
#pragma unroll
          for (int i = 9; i >= 0; --i) { fa = a * fa + c[i]; fb = b * fb + c[i]; }
        }
        if (fa * fb > 0.0) {
          mode = kBis1;                              // modrf failed: bisection on [mn, mx]
        } else if (fabs(fa) < kRelErr) {
          put_root(roots, ioff, inv ? 1.0 / a : a);  // stays kPop
        } else if (fabs(fb) < kRelErr) {
          put_root(roots, ioff, inv ? 1.0 / b : b);
        } else {
          lfx = fa;
          mode = kFalsi;
        }
      }
    }
    if (mode == kFalsi) {
      // one iteration of modrf_pos's loop (sturm.cu:82-205)
      ROOTS_COUNT(g_roots_falsi);
      const double x = (fb * a - fa * b) / (fb - fa);
      double fx;
      if (inv) {
        fx = c[0];
#pragma unroll
        for (int i = 1; i <= 10; ++i) fx = x * fx + c[i];
      } else {
        fx = c[10];
#pragma unroll
        for (int i = 9; i >= 0; --i) fx = x * fx + c[i];
      }
      bool found = false;
      double v = x;
      if (fabs(x) > kRelErr && fabs(fx / x) < kRelErr) found = true;
      else if (fabs(fx) < kRelErr) found = true;
      if (!found) {
        if ((fa * fx) < 0) { b = x; fb = fx; if ((lfx * fx) > 0) fa /= 2; }
        else { a = x; fa = fx; if ((lfx * fx) > 0) fb /= 2; }
        if (fabs(b - a) < fabs(kRelErr * a)) {
          found = true;
          v = a;
        } else {
          lfx = fx;
          if (++it == kMaxIt) { mode = kBis1; it = 0; }   // modrf_pos gave up
        }
      }
      if (found) { put_root(roots, ioff, inv ? 1.0 / v : v); mode = kPop; }
    } else if (mode >= kBis1) {
      mid = (double)((mn + mx) / 2);
      bool stop = false;
      if (mode == kBis1) {
        if (fabs(mid) > kRelErr) stop = fabs((mx - mn) / mid) < kRelErr;
        else stop = fabs(mx - mn) < kRelErr;
      }
      if (!stop) {
        const int atmid = sign_changes_r(S, mid);
        if (mode == kBis1) {
          if ((iatlo - atmid) == 0) mn = mid; else mx = mid;
          stop = ++it == kMaxIt;
        } else {
          const int n1 = iatlo - atmid, n2 = atmid - iathi;
          if (n1 != 0 && n2 != 0) {
            if (sp + 2 <= kStkDepth) {
              stk.put(sp++, mid, mx, atmid, iathi, ioff + n1, idepth + 1);
              stk.put(sp++, mn, mid, iatlo, atmid, ioff, idepth + 1);
            }
            mode = kPop;
          } else {
            // An interval that no longer changes (it has shrunk to adjacent
            // doubles around a multiple root) repeats this step until the
            // iteration limit, with the same mid: jump to the limit.
            const bool fixed = (n1 == 0) ? mid == mn : mid == mx;
            if (n1 == 0) mn = mid; else mx = mid;
            if (fixed) it = kMaxIt - 1;
            if (++it == kMaxIt) {
              for (int r = iathi; r < iatlo; ++r) put_root(roots, ioff + r - iathi, mid);
              mode = kPop;
            }
          }
        }
      }
      if (stop) { put_root(roots, ioff, mid); mode = kPop; }
    }
  }
}

// ---------------------------------------------------------------------------
// Split isolation (k_roots_split, tuning key roots_split = 1, default).
//
// isolate_r above advances each lane through pops (with modrf's case analysis
// and end-point evaluations), bisections and regula-falsi steps in one loop,
// so every pass pays for all of them whenever any lane of the wave is in each
// mode, and a wave lasts as long as its busiest hypothesis (p50 11 Sturm
// evaluations + 38 falsi steps, p99 89 + 70: git-history scripts/roots_stats.py).  What
// happens to an isolated single-root interval depends on nothing but the
// interval, its sign-change count and the sequence, and its root lands at a
// fixed slot (ioff), so the work is split in phases:
//   1. each hypothesis lane runs the isolation (the multi-root bisections),
//      and where isolate_r would call modrf on a single-root node it appends
//      the node (interval, count, slot) to the wave's task list in LDS;
//   2. all 64 lanes of the wave then run modrf over the task list -- the case
//      analysis and end-point evaluations when a lane claims a task, then one
//      regula-falsi step per pass -- each lane claiming the next task when its
//      own ends (a ballot and a prefix count, no atomics): the ~77 tasks of a
//      32-hypothesis wave spread over 64 lanes;
//   3. a node where modrf fails (end points of equal sign: 20 % of the
//      hypotheses have one, git-history scripts/roots_split_stats.py) or gives up (its
//      iteration limit) goes back to its hypothesis lane, which holds the
//      Sturm sequence in registers, for sbisect's bisection.
// Every node sees exactly the reference's operations in their order, and
// roots are written to their slot, so the roots are bit-identical to
// isolate_r's (tests/test_gpu_roots_split.py: the whole workspace).
// ---------------------------------------------------------------------------
// NL hypothesis lanes share one task pool: kStkLanes (one wave per block,
// roots_split = 1) or kStkLanes x the block's waves (roots_split = 2, the
// cross-wave pool: phases 2 and 3 are claimed by all the block's waves; it
// measured 2-6 % slower than per-wave pools, profiles/r04_roots_pool_ab.txt;
// the cause is not isolated -- the LDS counters are shared by four waves, and
// a CU holds one such block instead of four independent ones)
template <int NL>
struct RootsSharedT {
  static constexpr int kTasks = NL * 10;    // a hypothesis has at most 10 isolated roots
  double seq[kSturmRegs][NL];               // each hypothesis' Sturm sequence (s[0] = c[0..10])
  int np[NL];
  double tmn[kTasks], tmx[kTasks];          // single-root nodes: interval
  int tatlo[kTasks];                        // sign changes at its low end
  int tmeta[kTasks];                        // owner | ioff << 8 (owner: block hypothesis lane < 256)
  int dlist[kTasks];                        // nodes for sbisect's bisection (phase 3)
  double roots[10][NL];                     // root slots (scaled), 0 where none is found
  int ntask, ndl;
  int next2, next3;                         // pooled claims of phases 2 / 3 (LDS atomics)
};
using RootsShared = RootsSharedT<kStkLanes>;
static_assert(4 * kStkLanes <= 256, "owner lanes fit tmeta's 8 bits");

// isolate_p1's work stack: IsoStack with the four small integers packed in one
// word (sign-change counts and slots <= 10, depth <= kMaxDepth + 1)
struct IsoStackP {
  double* lohi;   // [kStkDepth][2][kStkLanes] + lane
  int* meta;      // [kStkDepth][kStkLanes] + lane
  __device__ __forceinline__ void put(int i, double lo, double hi, int atlo, int athi, int off, int depth) const {
    lohi[(2 * i) * kStkLanes] = lo;
    lohi[(2 * i + 1) * kStkLanes] = hi;
    meta[i * kStkLanes] = atlo | (athi << 8) | (off << 16) | (depth << 24);
  }
};

// phase 1: isolate_r's multi-root bisections; single-root nodes become tasks
// (`lane`: the hypothesis' owner index in the pool, its stack pre-offset)
template <class SH>
__device__ __forceinline__ void isolate_p1(const SturmR& S, double lo, double hi, int atlo, int athi,
                                           const IsoStackP& stk, SH& sh, int lane) {
  int sp = 0;
  stk.put(sp++, lo, hi, atlo, athi, 0, 0);
  bool bis = false;
  int it = 0, iatlo = 0, iathi = 0, ioff = 0, idepth = 0;
  double mn = 0.0, mx = 0.0;
  for (;;) {
    if (!bis) {
      if (sp == 0) break;
      --sp;
      mn = stk.lohi[(2 * sp) * kStkLanes];
      mx = stk.lohi[(2 * sp + 1) * kStkLanes];
      const int m = stk.meta[sp * kStkLanes];
      iatlo = m & 0xff;
      iathi = (m >> 8) & 0xff;
      ioff = (m >> 16) & 0xff;
      idepth = m >> 24;
      if (idepth >= kMaxDepth) continue;
      it = 0;
      if (iatlo - iathi != 1) {
        bis = true;
      } else {
        const int t = atomicAdd(&sh.ntask, 1);                 // modrf: phase 2
        sh.tmn[t] = mn;
        sh.tmx[t] = mx;
        sh.tatlo[t] = iatlo;
        sh.tmeta[t] = lane | (ioff << 8);
      }
    }
    if (bis) {
      const double mid = (double)((mn + mx) / 2);
      const int atmid = sign_changes_r(S, mid);
      const int n1 = iatlo - atmid, n2 = atmid - iathi;
      if (n1 != 0 && n2 != 0) {
        if (sp + 2 <= kStkDepth) {
          stk.put(sp++, mid, mx, atmid, iathi, ioff + n1, idepth + 1);
          stk.put(sp++, mn, mid, iatlo, atmid, ioff, idepth + 1);
        }
        bis = false;
      } else {
        // An interval that no longer changes (it has shrunk to adjacent
        // doubles around a multiple root) repeats this step until the
        // iteration limit, with the same mid: jump to the limit.
        const bool fixed = (n1 == 0) ? mid == mn : mid == mx;
        if (n1 == 0) mn = mid; else mx = mid;
        if (fixed) it = kMaxIt - 1;
        if (++it == kMaxIt) {
          for (int r = iathi; r < iatlo; ++r) sh.roots[ioff + r - iathi][lane] = mid;
          bis = false;
        }
      }
    }
  }
}

// phase 2: modrf (sturm.cu:208-275) and modrf_pos's loop (43-205) over the
// task list, on every lane.  POOL: the list is the block's (every wave of the
// block claims from it through an LDS counter); else the wave's own.  A node
// writes its root to a fixed slot, so who claims it changes no result.
template <bool POOL, class SH>
__device__ __forceinline__ void falsi_tasks(SH& sh, int lane) {
  const int ntask = sh.ntask;
  int next = 0, cur = -1, it = 0, owner = 0, ioff = 0;
  bool inv = false;
  double a = 0.0, b = 0.0, fa = 0.0, fb = 0.0, lfx = 0.0;
  double c[11];
#pragma unroll
  for (int i = 0; i <= 10; ++i) c[i] = 0.0;
  for (;;) {
    const unsigned long long idle = __ballot(cur < 0);
    const int rank = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(idle >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)idle, 0u));
    if (POOL) {
      int b0 = 0;
      if (lane == 0 && idle) b0 = atomicAdd(&sh.next2, __popcll(idle));
      next = __builtin_amdgcn_readfirstlane(b0);          // every lane is active here: lane 0 is the first
    }
    bool fresh = false;
    if (cur < 0 && next + rank < ntask) {
      cur = next + rank;
      fresh = true;
    }
    if (!POOL) next += __popcll(idle);
    if (__ballot(cur >= 0) == 0ull) break;
    if (fresh) {
      const int m = sh.tmeta[cur];
      owner = m & 0xff;
      ioff = m >> 8;
#pragma unroll
      for (int i = 0; i <= 10; ++i) c[i] = sh.seq[i][owner];
      // modrf: pick (a, b, inverted), then modrf_pos's end-point evaluations
      a = sh.tmn[cur];
      b = sh.tmx[cur];
      if (a > b) { const double t = a; a = b; b = t; }
      if (b <= 1.0 && a >= -1.0) {
        inv = false;
      } else if (a >= 1.0 || b <= -1.0) {
        inv = true;
      } else {
        double fp1 = 0.0, fm1 = 0.0, ga = 0.0, gb = 0.0;
#pragma unroll
        for (int i = 9; i >= 0; --i) {
          fp1 = c[i] + fp1;
          fm1 = c[i] - fm1;
          ga = a * ga + c[i];
          gb = b * gb + c[i];
        }
        if (a < -1.0 && b > 1.0) {
          if (ga * fm1 < 0.0) { b = -1.0; inv = true; }
          else if (gb * fp1 < 0.0) { a = 1.0; inv = true; }
          else { a = -1.0; b = 1.0; inv = false; }
        } else if (a < -1.0) {
          if (ga * fm1 < 0.0) { b = -1.0; inv = true; }
          else { a = -1.0; inv = false; }
        } else {
          if (gb * fp1 < 0.0) { a = 1.0; inv = true; }
          else { b = 1.0; inv = false; }
        }
      }
      if (inv) { const double t = a; a = 1.0 / b; b = 1.0 / t; }
      if (inv) {
        fa = fb = c[0];
#pragma unroll
        for (int i = 1; i <= 10; ++i) { fa = a * fa + c[i]; fb = b * fb + c[i]; }
      } else {
        fa = fb = c[10];
#pragma unroll
        for (int i = 9; i >= 0; --i) { fa = a * fa + c[i]; fb = b * fb + c[i]; }
      }
      lfx = fa;
      it = 0;
      if (fa * fb > 0.0) {                                      // modrf failed: phase 3
        sh.dlist[atomicAdd(&sh.ndl, 1)] = cur;
        cur = -1;
      } else if (fabs(fa) < kRelErr) {
        sh.roots[ioff][owner] = inv ? 1.0 / a : a;
        cur = -1;
      } else if (fabs(fb) < kRelErr) {
        sh.roots[ioff][owner] = inv ? 1.0 / b : b;
        cur = -1;
      }
    }
    if (cur >= 0) {
      const double x = (fb * a - fa * b) / (fb - fa);
      double fx;
      if (inv) {
        fx = c[0];
#pragma unroll
        for (int i = 1; i <= 10; ++i) fx = x * fx + c[i];
      } else {
        fx = c[10];
#pragma unroll
        for (int i = 9; i >= 0; --i) fx = x * fx + c[i];
      }
      bool found = false;
      double v = x;
      if (fabs(x) > kRelErr && fabs(fx / x) < kRelErr) found = true;
      else if (fabs(fx) < kRelErr) found = true;
      if (!found) {
        if ((fa * fx) < 0) { b = x; fb = fx; if ((lfx * fx) > 0) fa /= 2; }
        else { a = x; fa = fx; if ((lfx * fx) > 0) fb /= 2; }
        if (fabs(b - a) < fabs(kRelErr * a)) {
          found = true;
          v = a;
        } else {
          lfx = fx;
          if (++it == kMaxIt) {                                 // modrf_pos gave up: phase 3
            sh.dlist[atomicAdd(&sh.ndl, 1)] = cur;
            cur = -1;
          }
        }
      }
      if (found) {
        sh.roots[ioff][owner] = inv ? 1.0 / v : v;
        cur = -1;
      }
    }
  }
}

// phase 3: sbisect's bisection after modrf (sturm.cu:465-497), speculated
// three levels deep.  Lanes form groups of 8; a group takes one node of the
// list and, each pass, its lanes 0..6 evaluate the Sturm sequence at the
// 7 midpoints of the next three bisection levels (heap order: lane 0 the
// current midpoint, lanes 1 / 2 its left / right halves' midpoints, ...).  A
// midpoint is computed from its interval exactly as the sequential loop
// would reach it, so the walk down the tree (the stop tests, the sign-change
// decision, the iteration limit) reproduces the sequential bisection's
// steps and its final midpoint bit for bit, three steps per pass.
template <bool POOL, class SH>
__device__ __forceinline__ void bisect_deferred(SH& sh, int lane) {
  const int ndl = sh.ndl;
  if (ndl == 0) return;
  const int j = lane & 7, gbase = lane & ~7;
  int next = 0, cur = -1, it = 0, iatlo = 0, owner = 0, ioff = 0;
  double mn = 0.0, mx = 0.0;
  SturmR T;
  for (;;) {
    // the leader (j == 0) of each idle group claims the next node, in group order
    const unsigned long long idle = __ballot(cur < 0 && j == 0);
    if (POOL) {
      int b0 = 0;
      if (lane == 0 && idle) b0 = atomicAdd(&sh.next3, __popcll(idle));
      next = __builtin_amdgcn_readfirstlane(b0);
    }
    const unsigned long long below = gbase == 0 ? 0ull : (idle & ((1ull << gbase) - 1ull));
    const int t = next + __popcll(below);
    if (cur < 0 && t < ndl) {
      cur = sh.dlist[t];
      mn = sh.tmn[cur];
      mx = sh.tmx[cur];
      iatlo = sh.tatlo[cur];
      owner = sh.tmeta[cur] & 0xff;
      ioff = sh.tmeta[cur] >> 8;
      it = 0;
#pragma unroll
      for (int i = 0; i < kSturmRegs; ++i) T.c[i] = sh.seq[i][owner];
      T.np = sh.np[owner];
    }
    if (!POOL) next += __popcll(idle);
    if (__ballot(cur >= 0) == 0ull) break;
    // this lane's node: its interval down the heap path from [mn, mx]
    double lo = mn, hi = mx;
    const int k = j < 7 ? j : 0;
    const int depth = k == 0 ? 0 : (k < 3 ? 1 : 2);
    for (int d = depth - 1; d >= 0; --d) {
      // bit d of (k + 1) below its leading one: 0 = left half, 1 = right half
      const double m = (double)((lo + hi) / 2);
      if (((k + 1) >> d) & 1) lo = m; else hi = m;
    }
    const double mid = (double)((lo + hi) / 2);
    bool stop;
    if (fabs(mid) > kRelErr) stop = fabs((hi - lo) / mid) < kRelErr;
    else stop = fabs(hi - lo) < kRelErr;
    int atmid = 0;
    if (cur >= 0 && j < 7 && !stop) {
      ROOTS_COUNT(g_roots_falsi);                            // split stats: Sturm evaluations of phase 3
      atmid = sign_changes_r(T, mid);
    }
    // the walk, the same in every lane of the group
    int node = 0;
    bool done = false;
    double root = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int src = gbase + node;
      const double m = __shfl(mid, src);
      const bool st = __shfl((int)stop, src) != 0;
      const int am = __shfl(atmid, src);
      if (cur >= 0 && !done) {
        if (st) {
          done = true;
          root = m;
        } else {
          if ((iatlo - am) == 0) { mn = m; node = 2 * node + 2; } else { mx = m; node = 2 * node + 1; }
          if (++it == kMaxIt) {
            done = true;
            root = m;
          }
        }
      }
    }
    if (cur >= 0 && done) {
      if (j == 0) sh.roots[ioff][owner] = root;
      cur = -1;
    }
  }
}

// buildsturm + modp (sturm.cu:285-360) on registers, for the generic case in
// which every remainder keeps its full degree (ord[k] = 10 - k: no leading
// coefficient falls under kSmall before the last step).  The operations are
// remainder_into's, in its order, with every index static, so the sequence
// never touches scratch (the general form lives in a 1 KB local array whose
// every access waited on scratch memory: ~95 % of k_roots' time).  Returns
// false, with R unspecified, when a remainder would be truncated; the caller
// then takes the general path.
template <int K>
__device__ __forceinline__ bool sturm_step_r(SturmR& R) {
  constexpr int uo = 12 - K, vo = 11 - K;
  constexpr int ou = sturm_off(K - 2), ov = sturm_off(K - 1), orr = sturm_off(K);
  double t[uo + 1];
#pragma unroll
  for (int i = 0; i <= uo; ++i) t[i] = R.c[ou + i];
  if (R.c[ov + vo] < 0.0) {
    t[0] = -t[0];                                 // k = uo - vo - 1 = 0
#pragma unroll
    for (int k = 1; k >= 0; --k)
#pragma unroll
      for (int j = vo + k - 1; j >= k; --j) t[j] = -t[j] - t[vo + k] * R.c[ov + j - k];
  } else {
#pragma unroll
    for (int k = 1; k >= 0; --k)
#pragma unroll
      for (int j = vo + k - 1; j >= k; --j) t[j] -= t[vo + k] * R.c[ov + j - k];
  }
  if constexpr (K < 10) {
    if (fabs(t[vo - 1]) < kSmall) return false;   // would truncate: general path
    const double g = -fabs(t[vo - 1]);
#pragma unroll
    for (int i = vo - 1; i >= 0; --i) R.c[orr + i] = t[i] / g;
    return sturm_step_r<K + 1>(R);
  } else {
    // K = 10: the remainder has order 0 and ends the sequence (np = 10); its
    // constant is truncated to 0 when small and then negated, as buildsturm does
    const double c0 = fabs(t[0]) < kSmall ? 0.0 : t[0];
    R.c[orr] = -c0;
    return true;
  }
}

// Leading coefficients' sign changes at -inf / +inf (numroots, sturm.cu:393-439)
// for the generic orders ord[i] = 10 - i.
__device__ __forceinline__ int count_real_roots_r(const SturmR& R, int* atneg, int* atpos) {
  int pos = 0, neg = 0;
  double lf = R.c[sturm_off(0) + 10];
#pragma unroll
  for (int i = 1; i <= 10; ++i) {
    const double f = R.c[sturm_off(i) + 10 - i];
    if (lf == 0.0 || lf * f < 0) ++pos;
    lf = f;
  }
  lf = R.c[sturm_off(0) + 10];                    // ord 0 = 10, even
#pragma unroll
  for (int i = 1; i <= 10; ++i) {
    const double l = R.c[sturm_off(i) + 10 - i];
    const double f = ((10 - i) & 1) ? -l : l;
    if (lf == 0.0 || lf * f < 0) ++neg;
    lf = f;
  }
  *atneg = neg;
  *atpos = pos;
  return neg - pos;
}

// find_real_roots_sturm (sturm.cu:557-676) with the iterative part on the
// register-resident sequence; identical results to real_roots.  SPLIT: phase 1
// of the split isolation (isolate_p1; the roots are completed by phases 2-3
// in sh and scaled by the caller with *fac_out); R is left holding the
// sequence for phase 3.
template <bool SPLIT, class SH = RootsShared>
__device__ __forceinline__ int real_roots_t(const double poly[11], double roots[10], const IsoStack& stk, SturmR& R,
                                            SH* sh, const IsoStackP* stk_p, int lane, double* fac_out) {
#ifdef SFM_ROOTS_STATS
  unsigned long long ts = __builtin_amdgcn_s_memtime();
#endif
  // normalisation and root scaling (sturm.cu:570-590) on registers
  double c0[11];
  {
    const double norm = 1.0 / poly[10];
#pragma unroll
    for (int i = 0; i <= 10; ++i) c0[i] = poly[i] * norm;
  }
  double fac = 1.0;
  {
    const double v0 = fabs(c0[0]);
    if (v0 > 10.0) {
      fac = cr_pow(v0, -1.0 / 10);
      double m = fac;
#pragma unroll
      for (int i = 9; i >= 0; --i) { c0[i] *= m; m = m * fac; }
    }
  }
  ROOTS_PHASE(0, ts);
  bool generic;
  {
#pragma unroll
    for (int i = 0; i <= 10; ++i) R.c[sturm_off(0) + i] = c0[i];
    const double f = fabs(c0[10] * 10);
#pragma unroll
    for (int i = 1; i <= 10; ++i) R.c[sturm_off(1) + i - 1] = c0[i] * i / f;
    generic = sturm_step_r<2>(R);
  }
  if (generic) {
#pragma unroll
    for (int i = 0; i <= 10; ++i) R.ord[i] = 10 - i;
    R.np = 10;
    int atmin, atmax;
    int nr = count_real_roots_r(R, &atmin, &atmax);
    ROOTS_PHASE(1, ts);
    if (nr == 0) return 0;
    double mn = -1.0;
    int nch = sign_changes_r(R, mn);
    for (int i = 0; nch != atmin && i != kMaxPow; ++i) { mn *= 10.0; nch = sign_changes_r(R, mn); }
    if (nch != atmin) atmin = nch;
    double mx = 1.0;
    nch = sign_changes_r(R, mx);
    for (int i = 0; nch != atmax && i != kMaxPow; ++i) { mx *= 10.0; nch = sign_changes_r(R, mx); }
    if (nch != atmax) atmax = nch;
    nr = atmin - atmax;
    ROOTS_PHASE(2, ts);
    if (nr <= 0) return nr;
    if constexpr (SPLIT) {
      *fac_out = fac;
#pragma unroll
      for (int i = 0; i < kSturmRegs; ++i) sh->seq[i][lane] = R.c[i];
      sh->np[lane] = R.np;
      isolate_p1(R, mn, mx, atmin, atmax, *stk_p, *sh, lane);
    } else {
      isolate_r(R, mn, mx, atmin, atmax, roots, stk);
      for (int i = 0; i < nr && i < 10; ++i) roots[i] /= fac;
    }
    ROOTS_PHASE(3, ts);
    return nr;
  }
  {
    Sturm S;
    for (int i = 0; i < 11; ++i) { S.ord[i] = 0; for (int j = 0; j < 11; ++j) S.c[i][j] = 0.0; }
    const double norm = 1.0 / poly[10];
    for (int i = 0; i <= 10; ++i) S.c[0][i] = poly[i] * norm;
    const double v0 = fabs(S.c[0][0]);
    double fac = 1.0;
    if (v0 > 10.0) {
      fac = cr_pow(v0, -1.0 / 10);
      double m = fac;
      for (int i = 9; i >= 0; --i) { S.c[0][i] *= m; m = m * fac; }
    }
    const int np = build_sturm(S);
    int atmin, atmax;
    int nr = count_real_roots(S, np, &atmin, &atmax);
    if (nr == 0) return 0;
    // register copy, zero above each polynomial's degree
#pragma unroll
    for (int i = 0; i <= 10; ++i) {
      R.ord[i] = S.ord[i];
#pragma unroll
      for (int j = 0; j <= 10 - i; ++j) R.c[sturm_off(i) + j] = (i <= np && j <= S.ord[i]) ? S.c[i][j] : 0.0;
    }
    R.np = np;
    double mn = -1.0;
    int nch = sign_changes_r(R, mn);
    for (int i = 0; nch != atmin && i != kMaxPow; ++i) { mn *= 10.0; nch = sign_changes_r(R, mn); }
    if (nch != atmin) atmin = nch;
    double mx = 1.0;
    nch = sign_changes_r(R, mx);
    for (int i = 0; nch != atmax && i != kMaxPow; ++i) { mx *= 10.0; nch = sign_changes_r(R, mx); }
    if (nch != atmax) atmax = nch;
    nr = atmin - atmax;
    if (nr <= 0) return nr;
    if constexpr (SPLIT) {
      *fac_out = fac;
#pragma unroll
      for (int i = 0; i < kSturmRegs; ++i) sh->seq[i][lane] = R.c[i];
      sh->np[lane] = R.np;
      isolate_p1(R, mn, mx, atmin, atmax, *stk_p, *sh, lane);
    } else {
      isolate_r(R, mn, mx, atmin, atmax, roots, stk);
      for (int i = 0; i < nr && i < 10; ++i) roots[i] /= fac;
    }
    return nr;
  }
}

__device__ __forceinline__ int real_roots_r(const double poly[11], double roots[10], const IsoStack& stk) {
  SturmR R;
  return real_roots_t<false, RootsShared>(poly, roots, stk, R, nullptr, nullptr, 0, nullptr);
}

// null_space_solve_3x3_half_pivot (essential_matrix_5pt.cu:476-507)
__device__ __forceinline__ void null3(double M[3][3], double& x, double& y) {
  int p1;
  const double f0 = fabs(M[0][2]), f1 = fabs(M[1][2]), f2 = fabs(M[2][2]);
  if (f0 > f1) p1 = (f0 > f2) ? 0 : 2;
  else p1 = (f1 > f2) ? 1 : 2;
  const int r1 = (p1 + 1) % 3, r2 = (p1 + 2) % 3;
  double f = M[r1][2] / M[p1][2];
  M[r1][0] -= f * M[p1][0];
  M[r1][1] -= f * M[p1][1];
  f = M[r2][2] / M[p1][2];
  M[r2][0] -= f * M[p1][0];
  M[r2][1] -= f * M[p1][1];
  const int p2 = fabs(M[r1][1]) > fabs(M[r2][1]) ? r1 : r2;
  x = -M[p2][0] / M[p2][1];
  y = -(M[p1][0] + M[p1][1] * x) / M[p1][2];
}

// compute_E_matrix (essential_matrix_5pt.cu:955-1015)
__device__ void essential_at_root(const Lin Eb[9], const Eqs& A, double w, double E[9]) {
  const double w2 = w * w, w3 = w2 * w, w4 = w3 * w;
  double M[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      M[i][j] = A.e0[i][j] + w * A.e1[i][j] + w2 * A.e2[i][j] + w3 * A.e3[i][j];
    M[i][0] += w4 * A.e4[i];
  }
  double x, y;
  null3(M, x, y);
#pragma unroll
  for (int e = 0; e < 9; ++e) E[e] = w * Eb[e].c[0] + x * Eb[e].c[1] + y * Eb[e].c[2] + Eb[e].c[3];
}

// Cheirality test of one E against the 5 sample points (compute_P_matrices,
// cheirality.cu:4-214 with focal = null).  Returns -1 if rejected, else
// writes P (row-major 3x4).
__device__ bool cheirality_P(const double Ein[9], const double q[5][2], const double qp[5][2], double P[12]) {
  double U[3][3] = {{1.0, 0.0, 0.0}, {0.0, 1.0, 0.0}, {0.0, 0.0, 1.0}};
  double V[3][3];
#pragma unroll
  for (int e = 0; e < 9; ++e) V[e / 3][e % 3] = Ein[e];
#pragma unroll
  for (int i = 0; i <= 1; ++i)
#pragma unroll
    for (int k = i + 1; k < 3; ++k) {
      double a = V[i][i], b = V[k][i];
      const double s = sqrt(a * a + b * b);
      if (s == 0.0) continue;
      a /= s; b /= s;
      V[i][i] = s; V[k][i] = 0.0;
#pragma unroll
      for (int j = i + 1; j < 3; ++j) {
        const double c = V[i][j], d = V[k][j];
        V[i][j] = a * c + b * d;
        V[k][j] = a * d - b * c;
      }
      if (k == 1) {
        U[0][0] = U[1][1] = a; U[1][0] = -b; U[0][1] = b; U[2][2] = 1.0;
      } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const double t = a * U[i][j] + b * U[k][j];
          U[k][j] = -b * U[i][j] + a * U[k][j];
          U[i][j] = t;
        }
      }
    }
  const double sc = 1.0 / sqrt(V[0][0] * V[0][0] + V[0][1] * V[0][1] + V[0][2] * V[0][2]);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) V[i][j] *= sc;
  V[2][0] = V[0][1] * V[1][2] - V[0][2] * V[1][1];
  V[2][1] = V[0][2] * V[1][0] - V[0][0] * V[1][2];
  V[2][2] = V[0][0] * V[1][1] - V[0][1] * V[1][0];
  int c0 = 0, c1 = 0;
#pragma unroll
  for (int pt = 0; pt < 5; ++pt) {
    const double x0 = q[pt][0], x1 = q[pt][1], y0 = qp[pt][0], y1 = qp[pt][1];
    const double v0 = x0 * V[0][0] + x1 * V[0][1] + V[0][2];
    const double v2 = x0 * V[2][0] + x1 * V[2][1] + V[2][2];
    const double u1 = y0 * U[1][0] + y1 * U[1][1] + U[1][2];
    const double u2 = y0 * U[2][0] + y1 * U[2][1] + U[2][2];
    const double d1 = v0 * u2 + v2 * u1;
    const double d2 = -v0 * u2 + v2 * u1;
    c0 += (-u1 / d1 > 0.0) + (v0 / d1 > 0.0);
    c1 += (-u1 / d2 > 0.0) + (-v0 / d2 > 0.0);
  }
  int form;
  double ts;
  if (c0 == 10) { form = 0; ts = 1.0; }
  else if (c0 == 0) { form = 0; ts = -1.0; }
  else if (c1 == 10) { form = 1; ts = 1.0; }
  else if (c1 == 0) { form = 1; ts = -1.0; }
  else return false;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int j = 0; j < 3; ++j)
      P[4 * i + j] = form == 0 ? U[0][i] * V[1][j] - U[1][i] * V[0][j] + U[2][i] * V[2][j]
                               : -U[0][i] * V[1][j] + U[1][i] * V[0][j] + U[2][i] * V[2][j];
    P[4 * i + 3] = ts > 0.0 ? U[2][i] : -U[2][i];
  }
  return true;
}

// ---------------------------------------------------------------------------
// Hypothesis sampler: Philox4x32-10, counter {h, draw>>2, 0, 0}, key = seed;
// curand_uniform-style (0,1] float; RandomInt float arithmetic
// (kernel_functions.cu:269-278) with the index clamped to n-1.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    const uint32_t lo0 = 0xD2511F53u * c[0], hi0 = __umulhi(0xD2511F53u, c[0]);
    const uint32_t lo1 = 0xCD9E8D57u * c[2], hi1 = __umulhi(0xCD9E8D57u, c[2]);
    const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
  }
}

__device__ __forceinline__ void sample5(uint64_t seed, uint32_t h, int64_t n, int64_t idx[5]) {
  uint32_t a[4] = {h, 0u, 0u, 0u}, b[4] = {h, 1u, 0u, 0u};
  philox(a, (uint32_t)seed, (uint32_t)(seed >> 32));
  philox(b, (uint32_t)seed, (uint32_t)(seed >> 32));
  const uint32_t r[5] = {a[0], a[1], a[2], a[3], b[0]};
  const float scale = (float)(int)(n - 1) + 0.999999f;
#pragma unroll
  for (int d = 0; d < 5; ++d) {
    float u = (float)r[d] * 2.3283064e-10f;
    u = u + 2.3283064e-10f / 2.0f;
    float v = u * scale;
    v = v + 0.0f;
    int64_t k = (int64_t)truncf(v);
    idx[d] = k > n - 1 ? n - 1 : (k < 0 ? 0 : k);
  }
}

}  // namespace sfm
