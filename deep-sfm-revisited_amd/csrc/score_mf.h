// Phase 3d of the RANSAC (included by ransac5.hip): inlier scoring on the
// matrix cores with split-f16 operands (k_score_mf, the default scorer).
//
// The Sampson test of ComputeError (kernel_functions.cu:232-264) is, per
// (candidate E, point), a comparison of two polynomials in the point:
//   a = x'^T E x          bilinear: 9 monomials (x'x, x'y, x', y'x, y'y, y', x, y, 1)
//   D = |Ex|_01^2 + |x'^T E|_01^2   quadratic: 11 monomials (x^2, y^2, 1, xy, x, y,
//                                   x'^2, y'^2, x'y', x', y')
// inlier iff a^2 <= thr^2 D.  For a tile of 32 candidates x 32 points both are
// 32x32 GEMMs over the monomials, K <= 16: v_mfma_f32_32x32x16_f16 tiles.
//
//   a  needs ~22 significant bits (it cancels from terms ~1 down to ~1e-4):
//      coefficients c and monomials m are split c = c_hi + c_lo (f16 each) and
//      a = sum c_hi m_hi + c_hi m_lo + c_lo m_hi: 27 products, two MFMAs
//      (hi x hi first, from a zero accumulator).
//   D  has no such cancellation away from the epipole: one f16 MFMA each for
//      Ylo ~ t_lo D - eps_in and Yhi ~ t_hi D + eps_out, the two sides of the
//      decision band; eps and every error bound enter through two extra
//      monomials M^2, M^4 (M = max(1, |x|, |y|, |x'|, |y'|)).
// Decision per output element (3 VALU): aa = a*a; inlier iff aa < Ylo,
// outlier iff aa > Yhi; otherwise undecided -> the wave's LDS queue -> the
// float64 test of k_score32 (inlier_f64v + reference order).
//
// Error bounds (u = 2^-24; everything scaled: a' = 2^k a with 2^k <= 1/thr,
// E pre-scaled by a power of two to max |E_ij| in [0.5, 1); S = sum |c_j m_j|
// <= |c|_1 M^2):
//   * split representation: |c - c_hi - c_lo| <= 2^-22 |c| (+2^-25 absolute
//     when c_lo is subnormal), same for m; the dropped c_lo m_lo <= 2^-22 |c m|
//     -> 3 * 2^-22 S + 18 * 2^-25 (max|c| + M^2); the monomials are formed in
//     float32 from float32 coordinates, +0.75 * 2^-22 S (3.75 * 2^-22 in all).
//   * MFMA accumulation (derived, whatever the rounding): each f16 x f16
//     product is exact in f32 (11 x 11 significand bits, exponents in range),
//     so a v_mfma_f32_32x32x16_f16 output is the sum of n = 17 exact operands
//     (16 products and C).  If every one of its n - 1 additions rounds
//     faithfully in f32 (to nearest, toward zero or any direction: error < 1
//     ulp = 2u of the partial sum, whose magnitude is <= sum|operands|), in any
//     order or tree, the error is <= (n - 1) 2u sum|ops| = 32u (|C| + sum|ab|).
//     If instead the adder aligns all n operands to the largest exponent and
//     truncates each at 24 bits before one final rounding, the error is <=
//     n 2u max|op| + 2u |result| <= 36u (|C| + sum|ab|).  The bound used is
//     K_acc = SFM_MF_ACC_U u with SFM_MF_ACC_U = 36 (the larger; the
//     round-2 build used 16, above the 7.95u measured by
//     git-history scripts/probe_mfma_f16.hip but not derived): K_acc S (1 + 2^-9) for the
//     hi x hi MFMA, K_acc (|a| + 2^-8 S) for the second.
//   * the reference's own float64 rounding: 2^-46 S absolute, 2^-40 relative.
//   => |a'_computed - a'| <= alpha = aS * |c|_1 M^2 + ... + K_acc |a'|; the
//      K_acc |a'| part (<= 36u < 2^-18) is a relative factor folded into t
//      (1 -/+ 2^-18).
//   * certain inlier: (|a| + alpha)^2 <= (1 + 2^-6) a^2 + 65 alpha^2 (AM-GM)
//     <= t D  <=  aa < t_lo D - eps1,  t_lo = t / (1 + 2^-6) (and the
//     aa rounding 2^-22, ...), eps1 = 65 alpha^2 / (1 + 2^-6).
//     certain outlier: aa > t_hi D + eps2, t_hi = t / (1 - 2^-6), eps2 = 64
//     alpha^2 / (1 - 2^-6) (if |a| < alpha the test cannot fire).
//   * Ylo / Yhi themselves: f16 coefficients and monomials (2^-11 relative
//     each) and the accumulation: eta <= 1.048e-3 (>= 2^-10 + K_acc + margin,
//     K_acc = 36u = 2^-18.8) sum|g_j| M^2 (+ subnormal
//     terms), subtracted from / added to the coefficients of M^2; eps via M^4.
//     Directed rounding keeps every eps / eta coefficient >= its bound.
// Validity: 2^-15 <= thr < 1 (k in [0, 15]), finite non-zero E (zero E scores
// 0 exactly: a = D = 0 gives NaN in the reference; non-finite E: every
// evaluation goes to float64), M <= 15.9 per point (else float64).
// Numerically emulated before the kernel was written: 0 wrong decisions and
// 0.65 % undecided over 28M evaluations of 1398 KITTI candidates.

#ifndef SFM_MF_ACC_U
#define SFM_MF_ACC_U 36
#endif
static_assert(SFM_MF_ACC_U <= 64, "the relative part K_acc |a'| must stay below the 2^-18 folded into t");

// The AM-GM slack delta = 2^-SFM_MF_AMGM of the certain-inlier / outlier
// tests above (2^-6 written out there, the round-2 value).  In general
//   (|a| + alpha)^2 <= (1 + delta) a^2 + (1 + 1/delta) alpha^2,
//   (|a| - alpha)^2 >= (1 - delta) a^2 - (1/delta - 1) alpha^2   (|a| >= alpha),
// so t_lo = t / (1 + delta), eps1 = (1 + 1/delta) alpha^2 / (1 + delta),
// t_hi = t / (1 - delta), eps2 = (1/delta) alpha^2 / (1 - delta) (>= the
// (1/delta - 1) needed; with |a| < alpha the outlier test cannot fire since
// eps2 > alpha^2 for delta <= 1/2).  delta trades the relative band (t_lo,
// t_hi) against the alpha^2 terms; at the bench threshold 1e-4 the alpha^2
// terms dominate and delta = 2^-5 minimises the undecided band
// (git-history scripts/band_width_model.py: 0.193 % at 2^-6, 0.145 % at 2^-5, 0.146 % at 2^-4).
#ifndef SFM_MF_AMGM
#define SFM_MF_AMGM 5
#endif
static_assert(SFM_MF_AMGM >= 1 && SFM_MF_AMGM <= 10, "delta in [2^-10, 1/2]");

// a^2 folded into the band MFMAs (k_score_mf2, score_mf2.h): there the
// decisions are the signs of z1 = MFMA(C = aa, -Ylo rows) ~ aa - Ylo and
// z2 = MFMA(C = aa, -Yhi rows) ~ aa - Yhi, aa = fl(a * a), instead of
// fma(a, a, -Ylo) and fma(-a, a, Yhi).  The accumulator C = aa is one of the
// n = 17 MFMA operands, so the accumulation adds <= K_acc aa (K_acc = 36u) to
// the error already in eta, and aa itself rounds once (u):
//   inlier  (z1 < 0; C = +0 and exact products never give -0):
//     aa (1 - K_acc) < Ylo  =>  a^2 <= aa (1 + u) < Ylo (1 + 2^-18)   (Ylo > 0;
//     else the test cannot fire), covered by t_lo * (1 - 2^-18) (the
//     subtracted eps / eta terms only grow when scaled up);
//   outlier (sign bit of z2 clear, z2 >= +0 -- ties included):
//     aa (1 + K_acc) >= Yhi  =>  a^2 >= aa (1 - u) >= Yhi (1 - 2^-18), so with
//     t_hi, eps2 and eta_hi all scaled by (1 + 2^-17) a^2 is still strictly
//     above the unscaled Yhi, the strict outlier bound of the proof above.
// k_score_mf and the VALU decisions stay valid under the slightly wider band.
constexpr double kMfFoldLo = 1.0 - 0x1p-18;
constexpr double kMfFoldHi = 1.0 + 0x1p-17;
constexpr double kMfDelta = 1.0 / (double)(1 << SFM_MF_AMGM);
constexpr double kMfPin = 1.0 + (double)(1 << SFM_MF_AMGM);    // 1 + 1/delta
constexpr double kMfPout = (double)(1 << SFM_MF_AMGM);         // 1/delta

typedef _Float16 mf_half8 __attribute__((ext_vector_type(8)));
typedef float mf_float16 __attribute__((ext_vector_type(16)));

#ifndef SFM_MF_SUB
#define SFM_MF_SUB 3
#endif
constexpr int kMfSub = SFM_MF_SUB;            // candidate groups per item (one staged span serves them all)
#ifndef SFM_MF_WAVES
#define SFM_MF_WAVES 12
#endif
#ifndef SFM_MF_SPAN
#define SFM_MF_SPAN 768
#endif
#ifndef SFM_MF_WPE
#define SFM_MF_WPE (SFM_MF_WAVES / 4)
#endif
constexpr int kMfWaves = SFM_MF_WAVES;      // waves per block (3 per SIMD): one 32-candidate tile each
constexpr int kMfSpan = SFM_MF_SPAN;        // points per item (B fragments staged in LDS)
constexpr int kMfTiles = kMfSpan / 32;
constexpr int kMfQueue = 256;               // undecided entries per wave (drained in windows of this size)
constexpr int kMfRec = 64;                  // f16 per candidate: 4 A rows of K = 16
constexpr float kMfMaxM = 15.9f;            // M^4 stays below the f16 maximum

// per-candidate A rows (k_mf_cands): a1 [c_hi 0..8, c_hi 0..6] | a2 [c_hi 7..8,
// c_lo 0..8, 0 x5] | Ylo [g_lo 0..10 (g_2 - eps1c), -eta_lo, -eps1 s1, -eps1 s2, 0 x2] | Yhi [g_hi, +eta_hi, ...]
// and per-point B columns (staged in k_score_mf) with the same K order:
// b1 [m_hi 0..8, m_lo 0..6] | b2 [m_lo 7..8, m_hi 0..8, 0 x5] | bD [md 0..10, M^2, (s1/4)^2, (s2/4)^2, 0 x2]

struct MfParams {
  int k;                 // a' = 2^k a
  double t_lo, t_hi;     // scaled thresholds thr^2 4^k with the slack factors above
};

__host__ inline bool mf_params(double thr, MfParams* p) {
  if (!(thr >= 0x1p-15 && thr < 1.0)) return false;
  int k = 0;
  while (k < 15 && std::ldexp(thr, k + 1) <= 1.0) ++k;          // 2^k <= 1/thr < 2^(k+1)
  const double t = std::ldexp(thr * thr, 2 * k);                 // in (0.25, 1]
  p->k = k;
  p->t_lo = t * (1.0 - 0x1p-40) * (1.0 - 0x1p-22) * (1.0 - 0x1p-18) * kMfFoldLo / (1.0 + kMfDelta);
  p->t_hi = t * (1.0 + 0x1p-40) * (1.0 + 0x1p-22) * (1.0 + 0x1p-18) * kMfFoldHi / (1.0 - kMfDelta);
  return true;
}

// an f16 no smaller than v (v >= 0): inflate past one rounding, plus one
// subnormal quantum; v past the f16 range -> +inf (the caller checks)
__device__ __forceinline__ _Float16 f16_up(double v) {
  return (_Float16)(float)(v * (1.0 + 0x1p-10) + 0x1p-24);
}

// float32 form of f16_up for v >= 0 below the f16 range: v (1 + 2^-10)
// rounds down by at most 2^-24 relative and the conversion by 2^-11, so the
// result is >= v; the 2^-24 quantum covers values under the f16 normal range.
__device__ __forceinline__ _Float16 f16_upf(float v) {
  return (_Float16)(v * (1.0f + 0x1p-10f) + 0x1p-24f);
}

// One thread per candidate: the four A rows of its record.
__global__ void k_mf_cands(int cmax, const int32_t* __restrict__ cand_total, const double* __restrict__ candE,
                           _Float16* __restrict__ candF, MfParams mp, unsigned long long* __restrict__ claim,
                           int32_t* __restrict__ lead) {
  const int b = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  // k_score_mf2's range-claim counters (one per XCD) and its finished-block
  // count start every launch at 0, and so do k_mf2_lead's rest counts and
  // k_mf2_keep's kept counts (lead[128 .. 256))
  if (claim && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 9) claim[threadIdx.x] = 0ull;
  if (lead && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 2 * SFM_MAX_BATCH)
    lead[2 * SFM_MAX_BATCH + threadIdx.x] = 0;
  if (c >= cand_total[b]) return;
  const double* E = candE + ((size_t)b * cmax + c) * kCandStride;
  _Float16 row[kMfRec];
#pragma unroll
  for (int i = 0; i < kMfRec; ++i) row[i] = (_Float16)0.0f;
  double m = 0.0;
  bool finite = true;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    finite = finite && isfinite(E[i]);
    m = fmax(m, fabs(E[i]));
  }
  // zero E: a = D = 0, the reference's 0/0 is NaN -> never an inlier: Ylo = Yhi = -1
  // (every evaluation a decided outlier); non-finite E: Ylo = -1, Yhi = +1 (all undecided)
  bool special = !finite || m == 0.0;
  if (!special) {
    int e;
    (void)frexp(m, &e);
    double cc[9], hi[9], lo[9], En[9];
    double cm = 0.0;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      En[i] = ldexp(E[i], -e);                    // exact: max |En| in [0.5, 1)
      cc[i] = ldexp(En[i], mp.k);                 // a' coefficients, <= 2^15
      hi[i] = (double)(_Float16)(float)cc[i];
      lo[i] = (double)(_Float16)(float)(cc[i] - hi[i]);
      cm = fmax(cm, fabs(cc[i]));
    }
    // monomial order of a: E_ij x'_i x_j -> (x'x, x'y, x', y'x, y'y, y', x, y, 1) = E row-major
#pragma unroll
    for (int j = 0; j < 9; ++j) row[j] = (_Float16)hi[j];
#pragma unroll
    for (int j = 0; j < 7; ++j) row[9 + j] = (_Float16)hi[j];
    row[16] = (_Float16)hi[7];
    row[17] = (_Float16)hi[8];
#pragma unroll
    for (int j = 0; j < 9; ++j) row[18 + j] = (_Float16)lo[j];
    // D = sum_{r<2} (E_r . x)^2 + sum_{c<2} (x' . E_c)^2 on (x^2, y^2, 1, xy, x, y, x'^2, y'^2, x'y', x', y')
    const double e00 = En[0], e01 = En[1], e02 = En[2], e10 = En[3], e11 = En[4], e12 = En[5], e20 = En[6];
    const double e21 = En[7];
    double g[11];
    g[0] = e00 * e00 + e10 * e10;
    g[1] = e01 * e01 + e11 * e11;
    g[2] = (e02 * e02 + e12 * e12) + (e20 * e20 + e21 * e21);
    g[3] = 2.0 * (e00 * e01 + e10 * e11);
    g[4] = 2.0 * (e00 * e02 + e10 * e12);
    g[5] = 2.0 * (e01 * e02 + e11 * e12);
    g[6] = e00 * e00 + e01 * e01;
    g[7] = e10 * e10 + e11 * e11;
    g[8] = 2.0 * (e00 * e10 + e01 * e11);
    g[9] = 2.0 * (e00 * e20 + e01 * e21);
    g[10] = 2.0 * (e10 * e20 + e11 * e21);
    double sl = 0.0, sh = 0.0, ml = 0.0, mh = 0.0;
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const _Float16 gl = (_Float16)(float)(mp.t_lo * g[j]);
      const _Float16 gh = (_Float16)(float)(mp.t_hi * g[j]);
      row[32 + j] = gl;
      row[48 + j] = gh;
      sl += fabs((double)gl); ml = fmax(ml, fabs((double)gl));
      sh += fabs((double)gh); mh = fmax(mh, fabs((double)gh));
    }
    // alpha <= aS S + 2^-24 (s1 + s2 + 1) + 9 * 2^-24 max|c| with S = sum |c_j m_j| and the
    // point's group sums s1 = |x'x| + |x'y| + |y'x| + |y'y|, s2 = |x'| + |y'| + |x| + |y|
    // (subnormal lo parts: 2^-25 absolute per product on either side, doubled):
    //   alpha <= K1 s1 + K2 s2 + K3,  K1 = aS C1 + 2^-24, K2 = aS C2 + 2^-24,
    //   K3 = aS |c_8| + 2^-24 + 9 * 2^-24 max|c|,  C1 / C2 = max |c| over each group;
    //   alpha^2 <= 3 (K1^2 s1^2 + K2^2 s2^2 + K3^2)   (Cauchy-Schwarz)
    // eps terms ride on the monomials (s1/4)^2, (s2/4)^2 and '1'.
    constexpr double kAcc = SFM_MF_ACC_U * 0x1p-24;          // MFMA accumulation bound per operand sum
    const double aS = kAcc * (1.0 + 0x1p-9) + 3.75 * 0x1p-22 + kAcc * 0x1p-8 + 0x1p-46;
    const double C1 = fmax(fmax(fabs(cc[0]), fabs(cc[1])), fmax(fabs(cc[3]), fabs(cc[4])));
    const double C2 = fmax(fmax(fabs(cc[2]), fabs(cc[5])), fmax(fabs(cc[6]), fabs(cc[7])));
    const double K1 = aS * C1 + 0x1p-24, K2 = aS * C2 + 0x1p-24;
    const double K3 = aS * fabs(cc[8]) + 0x1p-24 + 9.0 * 0x1p-24 * cm;
    const double infl = 3.0 * (1.0 + 0x1p-9);
    const double e1s1 = 16.0 * infl * kMfPin * K1 * K1 / (1.0 + kMfDelta);     // x (s1/4)^2
    const double e1s2 = 16.0 * infl * kMfPin * K2 * K2 / (1.0 + kMfDelta);
    const double e1c = infl * kMfPin * K3 * K3 / (1.0 + kMfDelta);
    const double e2s1 = 16.0 * infl * kMfPout * K1 * K1 / (1.0 - kMfDelta) * kMfFoldHi;
    const double e2s2 = 16.0 * infl * kMfPout * K2 * K2 / (1.0 - kMfDelta) * kMfFoldHi;
    const double e2c = infl * kMfPout * K3 * K3 / (1.0 - kMfDelta) * kMfFoldHi;
    // the constant monomial carries g_2 -/+ eps (its f16 rounding is covered by eta)
    row[32 + 2] = (_Float16)(float)(mp.t_lo * g[2] - e1c);
    row[48 + 2] = (_Float16)(float)(mp.t_hi * g[2] + e2c);
    sl = 0.0; sh = 0.0; ml = 0.0; mh = 0.0;
#pragma unroll
    for (int j = 0; j < 11; ++j) {
      const double gl = (double)row[32 + j], gh = (double)row[48 + j];
      sl += fabs(gl); ml = fmax(ml, fabs(gl));
      sh += fabs(gh); mh = fmax(mh, fabs(gh));
    }
    // eta: f16 coefficients and monomials (2^-11 relative each; 2^-25 absolute
    // when subnormal, on either side) and the accumulation, per M^2 (M >= 1)
    const double eta_lo = (1.048e-3 * sl + 11.0 * 0x1p-25 * (ml + 1.0)) * (1.0 + 0x1p-9);
    const double eta_hi = (1.048e-3 * sh + 11.0 * 0x1p-25 * (mh + 1.0)) * (1.0 + 0x1p-9) * kMfFoldHi;
    const _Float16 Blo = f16_up(eta_lo), Bhi = f16_up(eta_hi);
    const _Float16 S1lo = f16_up(e1s1), S2lo = f16_up(e1s2), S1hi = f16_up(e2s1), S2hi = f16_up(e2s2);
    if (isfinite((float)Blo) && isfinite((float)Bhi) && isfinite((float)S1lo) && isfinite((float)S2lo) &&
        isfinite((float)S1hi) && isfinite((float)S2hi) && isfinite((float)row[32 + 2]) &&
        isfinite((float)row[48 + 2])) {
      row[32 + 11] = -Blo;
      row[32 + 12] = -S1lo;
      row[32 + 13] = -S2lo;
      row[48 + 11] = Bhi;
      row[48 + 12] = S1hi;
      row[48 + 13] = S2hi;
    } else {
      special = true;
      finite = false;
    }
  }
  if (special) {
#pragma unroll
    for (int i = 0; i < kMfRec; ++i) row[i] = (_Float16)0.0f;
    row[32 + 2] = (_Float16)(-1.0f);                             // Ylo = -1 (monomial '1')
    row[48 + 2] = (_Float16)(finite ? -1.0f : 1.0f);             // Yhi = -1 (outlier) / +1 (undecided)
  }
  // sentinel monomials (zero for every live in-range point): a dead slot
  // carries kMfSentinel in K = 14 (Ylo = Yhi = -S: a decided outlier), a point
  // outside the f16 range in K = 15 (Ylo = -S, Yhi = +S: undecided -> float64)
  row[32 + 14] = (_Float16)(-1.0f);
  row[32 + 15] = (_Float16)(-1.0f);
  row[48 + 14] = (_Float16)(-1.0f);
  row[48 + 15] = (_Float16)(1.0f);
  uint4* out = reinterpret_cast<uint4*>(candF + ((size_t)b * cmax + c) * kMfRec);
  const uint4* in = reinterpret_cast<const uint4*>(row);
#pragma unroll
  for (int i = 0; i < kMfRec / 8; ++i) out[i] = in[i];
}

// Stage one point's three B columns into the LDS fragment image of its tile:
// frag[t][f][lane][8], lane = 32 h + r holds K = 8h .. 8h+7 of column r.
// Monomials in float32 from float32 coordinates (relative error <= 3 * 2^-24
// against the float64 point, 0.75 * 2^-22 of the 3.75 * 2^-22 representation
// term of aS), split into f16 hi + lo: m - hi is exact in float32, lo rounds
// once (2^-22 |m|).  A dead slot (past the span) is zero but for the sentinel
// K = 14, a point past the f16 range (M > 15.9, or NaN) zero but for K = 15
// (see k_mf_cands: decided outlier / undecided for every candidate row).
constexpr float kMfSentinel = 60000.0f;     // exact in f16; +-S dominates every live Ylo / Yhi term

__device__ __forceinline__ void mf_stage_point(const double4 v, bool live, _Float16* frag_tile, int r) {
  const float x = (float)v.x, y = (float)v.y, xp = (float)v.z, yp = (float)v.w;
  float M = fmaxf(fmaxf(fabsf(x), fabsf(y)), fmaxf(fabsf(xp), fabsf(yp)));
  M = fmaxf(M, 1.0f);
  const bool bad = live && !(M <= kMfMaxM);
  _Float16 col[48];
#pragma unroll
  for (int i = 0; i < 48; ++i) col[i] = (_Float16)0.0f;
  if (!live) {
    col[32 + 14] = (_Float16)kMfSentinel;
  } else if (bad) {
    col[32 + 15] = (_Float16)kMfSentinel;
  } else {
    const float ma[9] = {xp * x, xp * y, xp, yp * x, yp * y, yp, x, y, 1.0f};
    _Float16 hi[9], lo[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      hi[j] = (_Float16)ma[j];
      lo[j] = (_Float16)(ma[j] - (float)hi[j]);
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) col[j] = hi[j];
#pragma unroll
    for (int j = 0; j < 7; ++j) col[9 + j] = lo[j];
    col[16] = lo[7];
    col[17] = lo[8];
#pragma unroll
    for (int j = 0; j < 9; ++j) col[18 + j] = hi[j];
    const float md[11] = {x * x, y * y, 1.0f, x * y, x, y, xp * xp, yp * yp, xp * yp, xp, yp};
#pragma unroll
    for (int j = 0; j < 11; ++j) col[32 + j] = (_Float16)md[j];
    // bound monomials, rounded up (>= their float64-point values): M^2 for the
    // Ylo / Yhi rounding terms, (s1/4)^2 and (s2/4)^2 for the a-error terms.
    // In float32: M is within 2^-24 of the float64 point's, each product ma
    // within 3 * 2^-24, each sum of non-negative terms adds <= 2^-24 per add;
    // the factors (1 + 2^-19) and (1 + 2^-18) cover that and their own
    // rounding, f16_upf the squaring and the f16 conversion.
    const float Mu = M * (1.0f + 0x1p-19f);
    const float s1 = ((fabsf(ma[0]) + fabsf(ma[1])) + (fabsf(ma[3]) + fabsf(ma[4]))) * (0.25f + 0x1p-20f);
    const float s2 = ((fabsf(xp) + fabsf(yp)) + (fabsf(x) + fabsf(y))) * (0.25f + 0x1p-20f);
    col[32 + 11] = f16_upf(Mu * Mu);
    col[32 + 12] = f16_upf(s1 * s1);
    col[32 + 13] = f16_upf(s2 * s2);
  }
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      *reinterpret_cast<uint4*>(frag_tile + ((size_t)f * 64 + 32 * h + r) * 8) =
          *reinterpret_cast<const uint4*>(col + 16 * f + 8 * h);
}

// row of accumulator register g in half h of a 32x32 MFMA output
__host__ __device__ constexpr int mf_row(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

// The float64 test of queued (candidate row, point) evaluations, with the
// span's points and the tile's E rows read from LDS (no global latency).
__device__ __forceinline__ void mf_drain(const double* __restrict__ sE, const double4* __restrict__ spts, int p0,
                                         int T, int R, const ScoreConsts& kc, int lane, int32_t (*cnt)[2],
                                         const uint32_t* q, int qn) {
#pragma unroll 1
  for (int i = lane; i < qn; i += 64) {
    const uint32_t e = q[i];
    const int c = (int)(e >> 24), r = (int)(e & 0xffffffu), p = p0 + r;   // r: index in the span
    if (inlier_f64v(sE + c * 10, spts[r], kc)) {
      if (p < T) atomicAdd(&cnt[c][0], 1);
      if (p < R) atomicAdd(&cnt[c][1], 1);
    }
  }
}

#ifdef SFM_MF_STAMPS
// experiment builds only (git-history scripts/mf_stamps.py): per-phase wave cycles of
// k_score_mf: [0] item setup + staging, [1] tile loop, [2] queue build,
// [3] float64 drain, [4] count reduction + atomics, [5] block barrier,
// [6] next-item prefetch issue; [7] items (vector atomics only)
constexpr int kMfStamps = 8;
__device__ unsigned long long g_mf_stamps[kMfStamps];
extern "C" int sfm_experiment_mf_stamps(unsigned long long* out, int reset) {
  if (reset) {
    unsigned long long z[kMfStamps] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_mf_stamps), z, sizeof(z)) == hipSuccess ? 0 : 2;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mf_stamps), kMfStamps * 8) == hipSuccess ? 0 : 2;
}
#define MF_STAMP(i)                                                                       \
  do {                                                                                    \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                         \
    mf_acc_[i] += now_ - mf_t0_;                                                          \
    mf_t0_ = now_;                                                                        \
  } while (0)
#else
#define MF_STAMP(i) do { } while (0)
#endif

struct MfAcc {
  mf_float16 a, lo, hi;
};
struct MfB {                                                  // one tile's B fragments (ds_read_b128 x 3)
  mf_half8 b1, b2, bd;
};

__device__ __forceinline__ MfB mf_load_b(const _Float16* frag_tile, int lane) {
  MfB b;
  b.b1 = *reinterpret_cast<const mf_half8*>(frag_tile + (size_t)(0 * 64 + lane) * 8);
  b.b2 = *reinterpret_cast<const mf_half8*>(frag_tile + (size_t)(1 * 64 + lane) * 8);
  b.bd = *reinterpret_cast<const mf_half8*>(frag_tile + (size_t)(2 * 64 + lane) * 8);
  return b;
}

__device__ __forceinline__ MfAcc mf_tile_mfma(const MfB& B, mf_half8 A1, mf_half8 A2, mf_half8 AL, mf_half8 AH) {
  mf_float16 z;
#pragma unroll
  for (int g = 0; g < 16; ++g) z[g] = 0.0f;
  MfAcc r;
  r.a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B.b1, z, 0, 0, 0);          // hi x hi (+7 hi x lo) first
  r.lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(AL, B.bd, z, 0, 0, 0);
  r.hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(AH, B.bd, z, 0, 0, 0);
  r.a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, B.b2, r.a, 0, 0, 0);        // the small products
  return r;
}

// Decisions of one tile: 4 VALU per evaluation, no scalar masks.
//   z1 = fl(a^2 - Ylo) (one FMA): inlier  iff a^2 < Ylo  iff sign(z1)
//   z2 = fl(Yhi - a^2):           outlier iff a^2 > Yhi  iff sign(z2)
// The FMA rounds once, so the sign of z is the sign of the exact difference
// (an exact zero is +0 in round-to-nearest: a^2 = Ylo is not an inlier, a^2 =
// Yhi not an outlier, as the strict compares say); with finite operands (the
// sentinels replace the old +inf / NaN offsets) no NaN arises.  Each sign bit
// is shifted into a per-register bit string (v_alignbit: s = s << 1 | z >> 31),
// so after n tiles bit n-1-t of s1[g] / s2[g] holds tile t's inlier / outlier
// flag; undecided = neither.
__device__ __forceinline__ void mf_tile_decide(const MfAcc& r, uint32_t (&s1)[16], uint32_t (&s2)[16]) {
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float z1 = __builtin_fmaf(r.a[g], r.a[g], -r.lo[g]);
    const float z2 = __builtin_fmaf(-r.a[g], r.a[g], r.hi[g]);
    s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(z1), 31);
    s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(z2), 31);
  }
}

// Sum each of 16 per-lane values over the 32 lanes of each wave half by
// recursive halving (16 lane exchanges instead of 16 x 5).  Afterwards lane
// L (of its half) holds the sum for g = (L >> 1) & 15, on lanes L and L ^ 1.
__device__ __forceinline__ int mf_half_reduce(int (&v)[16], int lane) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool b = (lane & 16) != 0;
    const int recv = __shfl_xor(b ? v[k] : v[k + 8], 16, 64);
    v[k] = (b ? v[k + 8] : v[k]) + recv;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool b = (lane & 8) != 0;
    const int recv = __shfl_xor(b ? v[k] : v[k + 4], 8, 64);
    v[k] = (b ? v[k + 4] : v[k]) + recv;
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const bool b = (lane & 4) != 0;
    const int recv = __shfl_xor(b ? v[k] : v[k + 2], 4, 64);
    v[k] = (b ? v[k + 2] : v[k]) + recv;
  }
  {
    const bool b = (lane & 2) != 0;
    const int recv = __shfl_xor(b ? v[0] : v[1], 2, 64);
    v[0] = (b ? v[1] : v[0]) + recv;
  }
  return v[0] + __shfl_xor(v[0], 1, 64);
}

// inclusive prefix sum over the 64 lanes: Hillis-Steele inside each 16-lane
// row with DPP row shifts (zero-filled at the row start, VALU speed), then the
// totals of the preceding rows from three lane reads
__device__ __forceinline__ int mf_wave_scan(int x, int lane) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);   // row_shr:8
  const int r0 = __builtin_amdgcn_readlane(x, 15), r1 = __builtin_amdgcn_readlane(x, 31);
  const int r2 = __builtin_amdgcn_readlane(x, 47);
  const int row = lane >> 4;
  return x + (row >= 1 ? r0 : 0) + (row >= 2 ? r1 : 0) + (row >= 3 ? r2 : 0);
}

static_assert(kMfTiles <= 32, "one bit per tile in 32-bit strings");

// Block barrier for LDS reuse only.  __syncthreads() also waits for every
// outstanding global access of the wave (s_waitcnt vmcnt(0)): here that is
// the next item's prefetch and the previous item's count atomics, whose
// latency under load (thousands of cycles) would then be paid at every
// barrier.  LDS accesses are complete at lgkmcnt(0); register results of the
// global loads are still waited for where they are used.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


template <class Src, bool SAME>
__global__ __launch_bounds__(kMfWaves * 64) __attribute__((amdgpu_waves_per_eu(SFM_MF_WPE, SFM_MF_WPE))) void k_score_mf(const Src src, PairParams pp, int batch, int cmax,
                                                           const int32_t* __restrict__ cand_total,
                                                           const double* __restrict__ candE,
                                                           const _Float16* __restrict__ candF,
                                                           int32_t* __restrict__ cntT, int32_t* __restrict__ cntR,
                                                           ScoreConsts kc) {
  __shared__ __attribute__((aligned(16))) _Float16 s_frag[kMfTiles][3][64][8];
  __shared__ double4 s_pts[kMfSpan];
  __shared__ double s_E[kMfWaves][kKC * 10];                 // E (9) + guard Kg of the wave's tile
  __shared__ uint32_t s_queue[kMfWaves][kMfQueue];
  __shared__ int32_t s_cnt[kMfWaves][kKC][2];               // float64 drain counts
  __shared__ int32_t s_first[SFM_MAX_BATCH + 1];
  __shared__ int32_t s_ctot[SFM_MAX_BATCH];                  // cand_total, read once
  __shared__ int32_t s_spans[SFM_MAX_BATCH];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int hl = lane >> 5, rl = lane & 31;
  if (tid == 0) {
    int acc = 0;
    for (int b = 0; b < batch; ++b) {
      const int tiles = (cand_total[b] + kKC - 1) / kKC;
      const int groups = (tiles + kMfWaves * kMfSub - 1) / (kMfWaves * kMfSub);
      const int spans = (max(pp.test[b], pp.rtest[b]) + kMfSpan - 1) / kMfSpan;
      s_spans[b] = spans;
      s_first[b] = acc;
      s_ctot[b] = cand_total[b];
      acc += groups * spans;
    }
    s_first[batch] = acc;
  }
  for (int i = tid; i < kMfWaves * kKC * 2; i += kMfWaves * 64) (&s_cnt[0][0][0])[i] = 0;
  __syncthreads();
  const int total = s_first[batch];
  int32_t(*cnt)[2] = s_cnt[wv];
  uint32_t* queue = s_queue[wv];
  const double* sE = s_E[wv];
  // item -> (pair, candidate group, span) and its prefetch: the next item's
  // points, A rows and E rows are loaded into registers while the current
  // item computes, so staging costs no global latency
  struct Item { int b, p0, p1, c0, nc, T, R; };   // c0, nc: the item's first candidate group
  auto item_of = [&](int item, int b) {                       // b: a pair at or before the item's
    Item it;
    while (item >= s_first[b + 1]) ++b;
    const int local = item - s_first[b];
    const int spans = s_spans[b];
    const int group = local / spans, span = local - group * spans;
    it.b = b;
    it.T = pp.test[b];
    it.R = pp.rtest[b];
    it.p0 = span * kMfSpan;
    it.p1 = min(max(it.T, it.R), it.p0 + kMfSpan);
    it.c0 = (group * kMfSub * kMfWaves + wv) * kKC;
    it.nc = max(0, min(kKC, s_ctot[b] - it.c0));
    // wave-uniform by construction; say so, so that addresses stay scalar
    it.b = __builtin_amdgcn_readfirstlane(it.b);
    it.p0 = __builtin_amdgcn_readfirstlane(it.p0);
    it.p1 = __builtin_amdgcn_readfirstlane(it.p1);
    it.c0 = __builtin_amdgcn_readfirstlane(it.c0);
    it.nc = __builtin_amdgcn_readfirstlane(it.nc);
    it.T = __builtin_amdgcn_readfirstlane(it.T);
    it.R = __builtin_amdgcn_readfirstlane(it.R);
    return it;
  };
  constexpr int kPtsPerThread = (kMfSpan + kMfWaves * 64 - 1) / (kMfWaves * 64);
  constexpr int kEPerLane = (kKC * 10 + 63) / 64;
  double4 pv[kPtsPerThread];
  double ev[kEPerLane];
  mf_half8 nA1, nA2, nAL, nAH;
  // one candidate group's E rows (-> s_E at its start) and split-f16 A rows
  auto prefetch_cands = [&](int b, int c0, int nc) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int lh = ln >> 5, lr = ln & 31;   // lane half and row of the A fragment
    if (nc > 0) {                                            // uniform; record c0 exists
      const char* rec0 = reinterpret_cast<const char*>(candE + ((size_t)b * cmax + c0) * kCandStride);
      const int lim = nc * 10;
#pragma unroll
      for (int j = 0; j < kEPerLane; ++j) {                  // E (9) + Kg of record i / 10
        const int i = ln + 64 * j;
        const unsigned o = i < lim ? (unsigned)((i / 10) * kCandStride + i % 10) * 8u : 0u;
        ev[j] = *reinterpret_cast<const double*>(rec0 + o);
      }
    }
    if (lr < nc) {
      const mf_half8* rec = reinterpret_cast<const mf_half8*>(candF + ((size_t)b * cmax + c0 + lr) * kMfRec);
      nA1 = rec[0 + lh];
      nA2 = rec[2 + lh];
      nAL = rec[4 + lh];
      nAH = rec[6 + lh];
    } else {                                                 // absent row: every evaluation a decided outlier
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        nA1[j] = (_Float16)0.0f; nA2[j] = (_Float16)0.0f; nAL[j] = (_Float16)0.0f; nAH[j] = (_Float16)0.0f;
      }
      if (lh == 0) {                                         // K = 2: the monomial '1' -> Ylo = Yhi = -1
        nAL[2] = (_Float16)(-1.0f); nAH[2] = (_Float16)(-1.0f);
      } else {                                               // K = 14, 15: sentinels -> -S (outlier)
        nAL[6] = (_Float16)(-1.0f); nAL[7] = (_Float16)(-1.0f);
        nAH[6] = (_Float16)(-1.0f); nAH[7] = (_Float16)(-1.0f);
      }
    }
  };
  auto prefetch = [&](const Item& it) {
    // an opaque copy of the lane index: the per-lane offsets below are then
    // recomputed per call instead of being hoisted out of the item loop,
    // where they would occupy (and spill) registers through the tile loop
    int ln = lane;
    asm volatile("" : "+v"(ln));
#pragma unroll
    for (int j = 0; j < kPtsPerThread; ++j) {
      const int i = wv * 64 + ln + j * kMfWaves * 64;
      const int p = it.p0 + i;
      pv[j] = src.load(it.b, (i < kMfSpan && p < it.p1) ? p : it.p0);
    }
    prefetch_cands(it.b, it.c0, it.nc);
  };
  Item cur;
  if (blockIdx.x < total) {
    cur = item_of(blockIdx.x, 0);
    prefetch(cur);
  }
#ifdef SFM_MF_STAMPS
  unsigned long long mf_t0_ = __builtin_amdgcn_s_memtime();
  unsigned long long mf_acc_[kMfStamps] = {};
#endif
  for (int item = blockIdx.x; item < total; item += gridDim.x) {
#ifdef SFM_MF_STAMPS
    mf_acc_[7] += 1;
#endif
    const int b = cur.b, p0 = cur.p0, p1 = cur.p1, T = cur.T, R = cur.R;
    const int cg0 = cur.c0;
    // 1. stage the prefetched span (points + B columns) and E rows into LDS
#pragma unroll
    for (int j = 0; j < kPtsPerThread; ++j) {
      const int i = tid + j * kMfWaves * 64;
      if (i < kMfSpan) {
        s_pts[i] = pv[j];
        mf_stage_point(pv[j], p0 + i < p1, &s_frag[i >> 5][0][0][0], i & 31);
      }
    }
#pragma unroll
    for (int j = 0; j < kEPerLane; ++j) {
      const int i = lane + 64 * j;
      if (i < kKC * 10) s_E[wv][i] = ev[j];
    }
    lds_barrier();
    // 2. the next item's loads fly while this one drains and reduces (issued
    // after the tile loop: its registers are not live during the MFMAs)
    auto prefetch_next = [&]() {
      if (item + (int)gridDim.x < total) {
        const Item nxt = item_of(item + gridDim.x, cur.b);   // items rise monotonically
        prefetch(nxt);
        cur = nxt;
      }
    };
    MF_STAMP(0);
    // kMfSub candidate groups run over the staged span in turn; each group's
    // rows were loaded while the previous group drained (unrolled: the last
    // group's next-item prefetch must not be live through the others)
#pragma unroll
    for (int sub = 0; sub < kMfSub; ++sub) {
    const int c0 = __builtin_amdgcn_readfirstlane(cg0 + sub * kMfWaves * kKC);
    const int nc = max(0, min(kKC, s_ctot[b] - c0));
    if (sub > 0) {
#pragma unroll
      for (int j = 0; j < kEPerLane; ++j) {
        const int i = lane + 64 * j;
        if (i < kKC * 10) s_E[wv][i] = ev[j];
      }
      wave_sync();
    }
    const mf_half8 A1 = nA1, A2 = nA2, AL = nAL, AH = nAH;
    auto prefetch_after = [&]() {
      if (sub + 1 < kMfSub) prefetch_cands(b, c0 + kMfWaves * kKC, max(0, min(kKC, s_ctot[b] - c0 - kMfWaves * kKC)));
      else prefetch_next();
    };
    if (nc <= 0) prefetch_after();
    if (nc > 0) {
      const int ntiles = (p1 - p0 + 31) >> 5;
      uint32_t s1[16], s2[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) { s1[g] = 0u; s2[g] = 0u; }
      // 168 VGPRs, three waves per SIMD: the MFMA and LDS latencies of one
      // wave's tile are covered by the other two (measured 5 % faster than two
      // waves per SIMD with a ping-pong of two accumulator sets, 256 VGPRs)
      const _Float16* fr = &s_frag[0][0][0][0];
      constexpr int kTileHalves = 3 * 64 * 8;
      // three waves per SIMD: one accumulator set, the B fragments one tile ahead
      MfB bn = mf_load_b(fr, lane);
      for (int t = 0; t < ntiles; ++t) {
        const MfB bc = bn;
        if (t + 1 < ntiles) bn = mf_load_b(fr + (size_t)(t + 1) * kTileHalves, lane);
        const MfAcc r = mf_tile_mfma(bc, A1, A2, AL, AH);
        mf_tile_decide(r, s1, s2);
      }
      MF_STAMP(1);
      prefetch_after();
      MF_STAMP(6);
      // bit n-1-t <-> tile t; dead slots are decided outliers
      const uint32_t vm = ntiles >= 32 ? ~0u : ((1u << ntiles) - 1u);
      // 3. the undecided evaluations -> the queue -> float64.  Each lane
      // writes its own entries at its exclusive prefix; a span with more than
      // kMfQueue undecided evaluations is drained in several windows.
      int nl = 0;
#pragma unroll
      for (int g = 0; g < 16; ++g) nl += __popc(~(s1[g] | s2[g]) & vm);
      const int incl = mf_wave_scan(nl, lane);
      const int qtotal = __builtin_amdgcn_readlane(incl, 63);
      for (int base = 0; base < qtotal; base += kMfQueue) {
        int pos = incl - nl - base;
        if (qtotal <= kMfQueue) {
          // the usual case, one window: every entry fits, no bounds test.
          // Entry = row << 24 | span-relative point (< kMfSpan, so any N fits);
          // bit j of a string is tile ntiles-1-j, point 32 (ntiles-1-j) + rl
          // of the span = top - 32 j.
          uint32_t* q = queue + pos;
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            uint32_t u = ~(s1[g] | s2[g]) & vm;
            const uint32_t top = ((uint32_t)mf_row(g, hl) << 24) | (uint32_t)(32 * (ntiles - 1) + rl);
            while (u) {
              *q++ = top - 32u * (uint32_t)__builtin_ctz(u);
              u &= u - 1u;
            }
          }
        } else {
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            uint32_t u = ~(s1[g] | s2[g]) & vm;
            const uint32_t top = ((uint32_t)mf_row(g, hl) << 24) | (uint32_t)(32 * (ntiles - 1) + rl);
            while (u) {
              if (pos >= 0 && pos < kMfQueue) queue[pos] = top - 32u * (uint32_t)__builtin_ctz(u);
              u &= u - 1u;
              ++pos;
            }
          }
        }
        wave_sync();
        MF_STAMP(2);
        mf_drain(sE, s_pts, p0, T, R, kc, lane, cnt, queue, min(kMfQueue, qtotal - base));
        wave_sync();
        MF_STAMP(3);
      }
      MF_STAMP(2);
      // 4. counts: popcounts of the inlier strings (masked to each prefix),
      // summed over the 32 points of each half, plus the float64 counts
      int cT[16], cR[16];
      if (SAME) {
#pragma unroll
        for (int g = 0; g < 16; ++g) cT[g] = __popc(s1[g]);
      } else {
        // tile t holds a point below prefix X iff t < ceil((X - p0 - rl) / 32)
        auto prefix_mask = [&](int X) {
          const int tX = min(ntiles, max(0, X - p0 - rl + 31) >> 5);
          return tX >= 32 ? ~0u : (vm & ~((1u << (ntiles - tX)) - 1u));
        };
        const uint32_t mT = prefix_mask(T), mR = prefix_mask(R);
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          cT[g] = __popc(s1[g] & mT);
          cR[g] = __popc(s1[g] & mR);
        }
      }
      const int sumT = mf_half_reduce(cT, lane);
      const int sumR = SAME ? sumT : mf_half_reduce(cR, lane);
      if ((lane & 1) == 0) {
        const int c = mf_row((rl >> 1) & 15, hl);
        const int dT = sumT + cnt[c][0], dR = sumR + cnt[c][1];
        cnt[c][0] = 0;
        cnt[c][1] = 0;
        if (c < nc) {
          if (dT) atomicAdd(cntT + (size_t)b * cmax + c0 + c, dT);
          if (dR) atomicAdd(cntR + (size_t)b * cmax + c0 + c, dR);
        }
      }
      wave_sync();
      MF_STAMP(4);
    }
    }
    lds_barrier();                                            // the span is re-staged next item
    MF_STAMP(5);
  }
#ifdef SFM_MF_STAMPS
  if (lane == 0)
    for (int i = 0; i < kMfStamps; ++i) atomicAdd(&g_mf_stamps[i], mf_acc_[i]);
#endif
}
