// Sanitizer driver (test infrastructure only; SURVEY.md §5 "Race detection /
// sanitizers").  Built by `make -C oracle sanitize` with
// -fsanitize=address,undefined -fno-sanitize-recover=all around the two
// host-side C++ sources of the path:
//   oracle/ransac5_oracle.cpp              the CPU restatement (checker)
//   deep-sfm-revisited_amd/csrc/host_polish.cpp  the product's host IRLS /
//                                          decompose (essential_matrix.optimise,
//                                          decompose, decomposeUV)
// and run by tests/test_sanitizers.py.  Every entry point is driven over
// ordinary, degenerate and edge inputs (duplicate and collinear samples,
// zero and non-finite E, n = 0 / 1, thresholds outside the fast paths,
// reduced precisions).  Any out-of-bounds access, use after free, leak,
// signed overflow, misaligned access or other undefined behaviour aborts the
// run with a report; a clean run prints "sanitize ok".
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

extern "C" {
int orc_solve5(const double*, const double*, int, double*, int*, double*, double*, int*);
int orc_inlier_count(const double*, const double*, const double*, int64_t, double);
void orc_inlier_mask(const double*, const double*, const double*, int64_t, double, uint8_t*);
void orc_inlier_mask_prec(const double*, const double*, const double*, int64_t, double, int, uint8_t*);
int orc_ransac5_prec(const double*, const double*, int64_t, int, int, int, int, double, uint64_t, int, int, int,
                     double*, double*, int*, int*, int*, int*, int*);
void orc_decompose(const double*, double*);
void orc_decompose_uv(const double*, double*, double*);
void orc_optimise(const double*, const double*, int64_t, const double*, double, double, int, double*);
int sfm_essential_decompose(const double*, double*);
int sfm_essential_decompose_uv(const double*, double*, double*);
int sfm_essential_optimise(const double*, const double*, int64_t, const double*, double, double, int, double*);
}

// host_polish.cpp's error sink lives in capi.hip (not built here)
namespace sfm {
void set_error(const std::string&) {}
}

static std::mt19937_64 rng(20260417);
static double uni(double a, double b) { return std::uniform_real_distribution<double>(a, b)(rng); }

// a rigid two-view scene in normalised coordinates with outliers
static void scene(int n, std::vector<double>& q, std::vector<double>& qp, double out_frac) {
  q.resize(2 * n);
  qp.resize(2 * n);
  const double ax = uni(-0.05, 0.05), ay = uni(-0.05, 0.05);
  const double t[3] = {uni(-0.3, 0.3), uni(-0.1, 0.1), 1.0};
  for (int i = 0; i < n; ++i) {
    const double X = uni(-4, 4), Y = uni(-2, 2), Z = uni(5, 40);
    const double X2 = X + ay * Z + t[0], Y2 = Y - ax * Z + t[1], Z2 = Z - ay * X + ax * Y + t[2];
    q[2 * i] = X / Z;
    q[2 * i + 1] = Y / Z;
    qp[2 * i] = X2 / Z2 + uni(-2e-4, 2e-4);
    qp[2 * i + 1] = Y2 / Z2 + uni(-2e-4, 2e-4);
    if (uni(0, 1) < out_frac) {
      qp[2 * i] = uni(-0.5, 0.5);
      qp[2 * i + 1] = uni(-0.5, 0.5);
    }
  }
}

static int checks = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    ++checks;                                                          \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "check failed at line %d: %s\n", __LINE__, #c); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  // 1. five-point solves: random, duplicate-point, collinear and all-zero samples
  for (int k = 0; k < 400; ++k) {
    double q5[10], qp5[10], Er[90], Eo[90], Po[120];
    for (int i = 0; i < 10; ++i) { q5[i] = uni(-1, 1); qp5[i] = uni(-1, 1); }
    if (k % 4 == 1) { q5[2] = q5[0]; q5[3] = q5[1]; qp5[2] = qp5[0]; qp5[3] = qp5[1]; }   // duplicate
    if (k % 4 == 2) for (int i = 0; i < 5; ++i) { q5[2 * i + 1] = 0.3 * q5[2 * i]; }        // collinear
    if (k % 50 == 3) { std::memset(q5, 0, sizeof(q5)); std::memset(qp5, 0, sizeof(qp5)); }
    int nr = -1, np = -1;
    orc_solve5(q5, qp5, k & 1, Er, &nr, Eo, Po, &np);
    EXPECT(nr >= 0 && nr <= 10);
    EXPECT(!(k & 1) || (np >= 0 && np <= nr));
  }
  // 2. full RANSAC: dense and tiny pairs, prefixes, thresholds, precisions, cheirality on/off
  std::vector<double> q, qp;
  const int ns[] = {1, 5, 37, 900};
  const double thrs[] = {1e-4, 1e-3, 0.3, 2.0};
  const int precs[] = {64, 32, 16};
  for (int n : ns) {
    scene(n, q, qp, 0.2);
    for (double thr : thrs)
      for (int prec : precs)
        for (int cheir = 0; cheir < 2; ++cheir) {
          const int nchains = 8, iters = 2;
          double E[9], P[12];
          int inl = -1, win = -2;
          std::vector<int> score(nchains * iters), ncand(nchains * iters), best(nchains * iters);
          const int nt = n > 3 ? n / 2 : n;
          const int rc = orc_ransac5_prec(q.data(), qp.data(), n, nt, n, nchains, iters, thr, 1234, cheir, 1, prec,
                                          E, P, &inl, &win, score.data(), ncand.data(), best.data());
          EXPECT(rc == 0);
          EXPECT(inl >= 0 && inl <= n && win >= -1 && win < nchains * iters);
        }
    if (n >= 5) {
      double E[9] = {0, -1, 0.1, 1, 0, -0.2, -0.1, 0.2, 0};
      std::vector<uint8_t> m(n);
      orc_inlier_mask(E, q.data(), qp.data(), n, 1e-3, m.data());
      orc_inlier_mask_prec(E, q.data(), qp.data(), n, 1e-3, 16, m.data());
      const double Z[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      EXPECT(orc_inlier_count(Z, q.data(), qp.data(), n, 1e-3) == 0);        // 0/0: never an inlier
      const double N[9] = {NAN, 0, 0, 0, 0, 0, 0, 0, 0};
      EXPECT(orc_inlier_count(N, q.data(), qp.data(), n, 1e-3) == 0);
    }
  }
  // argument errors are refused, not read past
  {
    double E[9], P[12];
    int inl, win;
    EXPECT(orc_ransac5_prec(q.data(), qp.data(), 10, 11, 10, 8, 1, 1e-3, 1, 1, 1, 64, E, P, &inl, &win, nullptr,
                            nullptr, nullptr) != 0);
    EXPECT(orc_ransac5_prec(q.data(), qp.data(), 10, 10, 10, 8, 1, 1e-3, 1, 1, 1, 8, E, P, &inl, &win, nullptr,
                            nullptr, nullptr) != 0);
  }
  // 3. host IRLS and decompositions (product host code and its restatement)
  scene(500, q, qp, 0.3);
  const double E0[9] = {0.01, -0.99, 0.1, 1.0, 0.02, -0.3, -0.1, 0.3, 0.0};
  const double Ez[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  const double Ei[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
  const double* Es[] = {E0, Ez, Ei};
  for (const double* E : Es) {
    double a[9], b[9], pa[5], pb[5], U[9], V[9], U2[9], V2[9];
    const int64_t counts[] = {0, 1, 500};
    for (int64_t n : counts)
      for (int reps : {0, 3, 200}) {
        EXPECT(sfm_essential_optimise(q.data(), qp.data(), n, E, 1e-3, 0.0, reps, a) == 0);
        orc_optimise(q.data(), qp.data(), n, E, 1e-3, 0.0, reps, b);
        EXPECT(std::memcmp(a, b, sizeof(a)) == 0 || (std::isnan(a[0]) && std::isnan(b[0])));
        EXPECT(sfm_essential_optimise(q.data(), qp.data(), n, E, 2e-3, 1.0, reps, a) == 0);
      }
    EXPECT(sfm_essential_decompose(E, pa) == 0);
    orc_decompose(E, pb);
    EXPECT(sfm_essential_decompose_uv(E, U, V) == 0);
    orc_decompose_uv(E, U2, V2);
  }
  EXPECT(sfm_essential_optimise(nullptr, qp.data(), 1, E0, 1e-3, 0, 1, nullptr) != 0);
  std::printf("sanitize ok: %d checks\n", checks);
  return 0;
}
