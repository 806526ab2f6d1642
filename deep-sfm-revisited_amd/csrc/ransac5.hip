// RANSAC five-point essential matrix on CDNA4 (gfx950).
//
// Replaces the reference's essential_matrix extension hot path
// (RANSAC_FiveP/essential_matrix/essential_matrix.cu:110-280 host drivers,
// kernel_functions.cu:53-226 kernels).  The reference runs 512 threads, each
// looping over `ransac_iter` hypotheses and scoring every candidate E against
// all N correspondences serially.  Here the same semantics are split into
// data-parallel phases:
//
//   k_solve   one lane per hypothesis: Philox sample, five-point solve,
//             cheirality, compaction.                      (latency-bound)
//   k_chain   one lane per reference thread ("chain"): resolves the stale
//             slot-0 E/P state a chain carries across its iterations and
//             emits a dense candidate list (prefix sum per pair).
//   k_score   persistent, tiles of 32 candidates x 8192 points: the
//             Sampson-style inlier test, wave-ballot popcounts, int atomics.
//                                                           (fp64-VALU-bound)
//   k_select  per pair: preselect/rescore per hypothesis, first-max argmax.
//
// Inlier decisions are bit-identical to the reference's IEEE evaluation
// e = |x'^T E x| / sqrt(Ex0^2+Ex1^2+xE0^2+xE1^2) <= thr (ComputeError,
// kernel_functions.cu:232-264).  The score kernel decides most (candidate,
// point) pairs on an FMA evaluation with a proven error bound (see
// inlier_fast below) and re-evaluates the rare undecided ones in the
// reference's exact operation order.
#include <algorithm>
#include <mutex>
#include <vector>
#include "common.h"
#include "five_point.h"

namespace sfm {

constexpr int kChains = SFM_RANSAC_CHAINS;
constexpr int kMaxSlots = 10;
constexpr size_t kMf2ClaimBytes = 9 * sizeof(unsigned long long);   // k_score_mf2's per-XCD claim counters + done
constexpr int kCandStride = 18;   // per candidate: E f64[9], Kg, then float[14] (E f32[9], A1, B1, A2, B2, ok32)
// solve state fields: E basis (36), the 3x3 blocks of the reduced equations
// that compute_E_matrix reads (39), the five samples (20), det poly (11), roots (10)
constexpr int kStEb = 0, kStA = 36, kStQ = 75, kStPoly = 95, kStRoots = 106, kStateFields = 116;
constexpr int kKC = 32;           // candidates per score tile
constexpr int kPPL = 8;           // points per lane per chunk
constexpr int kScoreThreads = 256;
constexpr int kChunk = kScoreThreads * kPPL;
constexpr int kPPL32 = 8;          // points per lane per chunk in k_score32 (6, 10, 12 measured slower)
constexpr int kPtsPerItem = 8192;  // points per k_score item (a whole number of chunks)
static_assert(kPtsPerItem % kChunk == 0, "item = whole chunks");

struct PairParams {
  int64_t n[SFM_MAX_BATCH];
  int32_t test[SFM_MAX_BATCH];     // num_test_points
  int32_t rtest[SFM_MAX_BATCH];    // num_ransac_test_points
  int32_t splits[SFM_MAX_BATCH];   // point splits of max(test, rtest)
};

struct Workspace {
  int32_t* nroots;     // [B][H]
  int32_t* ncand;      // [B][H]
  double* hypE;        // [B][H][10][9]
  double* hypP;        // [B][H][10][12]
  double* hypP0;       // [B][H][12]
  double* sstate;      // [kStateFields][B][H]: solve state between k_solve_front, k_roots, k_solve_back
  int32_t* cand_off;   // [B][H]
  int32_t* chain_ref;  // [B][H] (latest k <= i with a root) + 1 | (latest k < i with a candidate) + 1 << 16
  int32_t* cand_total; // [64]
  double* candE;       // [B][Cmax][12]
  int32_t* cntT;       // [B][Cmax]
  int32_t* cntR;       // [B][Cmax]
  int32_t* score;      // [B][H]
  _Float16* candF;     // [B][Cmax][64] split-f16 A rows of k_score_mf (k_mf_cands)
  unsigned long long* cov;      // [B][Cmax] pruning bound state: count | points covered << 32
  int32_t* best_lb;             // [64] largest partial count seen (a lower bound on the winning score)
  unsigned long long* skipped;  // [1] evaluations skipped by pruning (whole call)
  unsigned long long* claim;    // [9] k_score_mf2's range-claim counters and finished-block count (zero between launches)
  int32_t* cmap;       // [B][Cmax] k_mf2_keep: the kept candidates of each pair
  int32_t* cmap2;      // [B][Cmax] k_mf2_keep_map: those kept again at the end (one-sided pruning)
  int32_t* lead;       // [5][64] k_mf2_lead / _keep: leader count, index, rest count, kept candidates,
                       // kept candidates left to the matrix-core pass (one-sided pruning)
  int32_t* bnd;        // [4][64] k_mf2_split: span boundaries of the pruned launches per pair
  double* pack;        // [n_max][4] (last: its size is the only n_max-dependent one)
};

__host__ __device__ inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

// Lay out the workspace; returns the byte count (ptrs filled when base != nullptr).
static size_t layout(char* base, int bc, int64_t n_max, int iters, Workspace* w) {
  const size_t H = (size_t)kChains * iters, C = H * kMaxSlots;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* p = base ? base + off : nullptr; off += align_up(bytes); return p; };
  Workspace t;
  t.nroots = (int32_t*)take(bc * H * 4);
  t.ncand = (int32_t*)take(bc * H * 4);
  t.hypE = (double*)take(bc * H * kMaxSlots * 9 * 8);
  t.hypP = (double*)take(bc * H * kMaxSlots * 12 * 8);
  t.hypP0 = (double*)take(bc * H * 12 * 8);
  t.sstate = (double*)take((size_t)kStateFields * bc * H * 8);
  t.cand_off = (int32_t*)take(bc * H * 4);
  t.chain_ref = (int32_t*)take(bc * H * 4);
  t.cand_total = (int32_t*)take(SFM_MAX_BATCH * 4);
  t.candE = (double*)take(bc * C * kCandStride * 8);
  t.cntT = (int32_t*)take(bc * C * 4);
  t.cntR = (int32_t*)take(bc * C * 4);
  t.cov = (unsigned long long*)take(bc * C * 8);     // must follow cntR (prune_state)
  t.best_lb = (int32_t*)take(SFM_MAX_BATCH * 64 * 4);    // kBestStride
  t.skipped = (unsigned long long*)take(8);
  t.score = (int32_t*)take(bc * H * 4);
  t.candF = (_Float16*)take(bc * C * 64 * 2);
  // before pack: run_packed re-lays the workspace out with n_max = 0, so every
  // field it uses must sit at an offset independent of n_max
  t.claim = (unsigned long long*)take(kMf2ClaimBytes);
  t.cmap = (int32_t*)take(bc * C * 4);
  t.cmap2 = (int32_t*)take(bc * C * 4);
  t.lead = (int32_t*)take(SFM_MAX_BATCH * 5 * 4);
  t.bnd = (int32_t*)take(SFM_MAX_BATCH * 4 * 4);
  t.pack = (double*)take((size_t)std::max<int64_t>(n_max, 0) * 4 * 8);
  if (w) *w = t;
  return off;
}

// ---------------------------------------------------------------------------
// Correspondence sources.  The kernels read point k of pair b through one of
//   PackedSrc  packed (x, y, x', y') float64 rows (sfm_ransac5_packed)
//   FlowSrc    the dense flow itself: pixel (u, v) of the margin crop, q =
//              K^-1 (u, v, 1), qp = K^-1 (u + fu, v + fv, 1) in float32 rows
//              (k0*x + k1*y) + k2, widened (SFMnet.py:179-263, flow2coord
//              298-318) -- the fused path of SURVEY §8(f) row 2: no staging
//              buffer, 8 bytes of flow per point instead of 32.
// Both yield bit-identical values (k_flow_points uses FlowSrc).
// ---------------------------------------------------------------------------
struct PackedSrc {
  const double* pts;
  int64_t n_stride;
  __device__ __forceinline__ double4 load(int b, int64_t k) const {
    return *reinterpret_cast<const double4*>(pts + ((size_t)b * n_stride + k) * 4);
  }
  PackedSrc shifted(int b0) const { return PackedSrc{pts + (size_t)b0 * n_stride * 4, n_stride}; }
};

struct FlowSrc {
  const float* flow;   // [B][2][H][W]
  const float* Kinv;   // [B][3][3]
  int H, W, wn, margin;
  double inv_wn;       // 1 / wn: k / wn by one multiply and one exact correction (k < 2^31)
  __device__ __forceinline__ double4 load(int b, int64_t k64) const {
    const int k = (int)k64;
    int row = (int)((double)k * inv_wn);
    int col = k - row * wn;
    if (col < 0) { --row; col += wn; } else if (col >= wn) { ++row; col -= wn; }
    const int v = row + margin, u = col + margin;
    const float* Ki = Kinv + b * 9;
    const float* F = flow + (size_t)b * 2 * H * W;
    const float fu = F[(size_t)v * W + u], fv = F[(size_t)H * W + (size_t)v * W + u];
    const float u1 = (float)u, v1 = (float)v;
    const float u2 = u1 + fu, v2 = v1 + fv;
    const float x1 = (Ki[0] * u1 + Ki[1] * v1) + Ki[2];
    const float y1 = (Ki[3] * u1 + Ki[4] * v1) + Ki[5];
    const float x2 = (Ki[0] * u2 + Ki[1] * v2) + Ki[2];
    const float y2 = (Ki[3] * u2 + Ki[4] * v2) + Ki[5];
    return make_double4(x1, y1, x2, y2);
  }
  FlowSrc shifted(int b0) const {
    return FlowSrc{flow + (size_t)b0 * 2 * H * W, Kinv + (size_t)b0 * 9, H, W, wn, margin, inv_wn};
  }
};

// ---------------------------------------------------------------------------
// Phase 1: one lane per hypothesis
// ---------------------------------------------------------------------------
// The solve is latency-bound (scratch-resident polynomial state, data-dependent
// Sturm iterations): only `lanes` lanes of each wave carry a hypothesis, so a
// pair's 4096 hypotheses occupy 4096 / lanes waves and every CU has several
// independent instruction streams to hide the scratch latency.
// The solve runs as three kernels so that each keeps a small live state:
//   k_solve_front  sample, E basis, constraint equations, reduction, det poly
//   k_roots        Sturm root isolation on a register-resident sequence
//                  (88 % of the former single kernel's time was spent here,
//                  waiting on scratch-resident coefficients)
//   k_solve_back   E per root, cheirality, compaction
// The state in between (116 doubles per hypothesis) is stored field-major.
__device__ __forceinline__ double& st_at(double* st, size_t stride, int f, size_t hb) { return st[f * stride + hb]; }

constexpr int kFrontLanes = 16;   // upper bound of the solve_lanes key

#ifdef SFM_FRONT_STATS
// experiment builds only: per wave (lane 0 of each block), the s_memtime
// stamps at the end of each phase of k_solve_front relative to its start:
// sample+load, basis, equations, reduction, determinant, state stores
__device__ unsigned long long g_front_cycles[6][1 << 15];
#define FRONT_STAMP(i)                                                                          \
  do {                                                                                          \
    __builtin_amdgcn_s_waitcnt(0);                                                              \
    if (threadIdx.x == 0)                                                                       \
      g_front_cycles[i][(size_t)blockIdx.y * gridDim.x + blockIdx.x] = __builtin_amdgcn_s_memtime() - t_front; \
  } while (0)
extern "C" int sfm_experiment_front_stats(unsigned long long* cycles, int n) {
  return hipMemcpyFromSymbol(cycles, HIP_SYMBOL(g_front_cycles), (size_t)6 * n * 8) == hipSuccess ? 0 : 2;
}
#else
#define FRONT_STAMP(i) do { } while (0)
#endif

// COOP (tuning key solve_coop, default): the reduction runs on DPP quads,
// four lanes per hypothesis (quad_reduce in five_point.h), so all 64 lanes of
// the wave work on the 16 hypotheses' reductions instead of 16 of them.
template <class Src, bool COOP>
__global__ __launch_bounds__(64) void k_solve_front(const Src src, PairParams pp, int H, uint64_t seed, int lanes,
                                                    double* __restrict__ st, size_t stride) {
#ifdef SFM_FRONT_STATS
  const unsigned long long t_front = __builtin_amdgcn_s_memtime();
#endif
  const int b = blockIdx.y;
  // COOP: quad g = lane / 4 carries hypothesis g; its four lanes draw the same
  // sample and build the same basis (the wave issues those instructions once
  // either way), then share the equations and the reduction
  const int g = COOP ? (int)threadIdx.x >> 2 : (int)threadIdx.x;
  const int qs = (int)threadIdx.x & 3;
  const int h = blockIdx.x * lanes + g;
  const bool act = g < lanes && h < H;
  if (!COOP && !act) return;
  // The equation set (1784 B) lives in LDS, one record per hypothesis: the
  // reduction's pivoting indexes rows dynamically, which put it in scratch
  // (0.30 -> 0.13 ms per 32,768 hypotheses).  A 1784-B lane stride is 446
  // dwords, so the 16 lanes' doubles fall in distinct bank pairs.
  __shared__ Eqs s_eqs[kFrontLanes];
  Eqs& A = s_eqs[g];
  double q[5][2], qp[5][2];
  Lin Eb[9];
  if (act) {
    const int64_t n = pp.n[b];
    int64_t idx[5];
    sample5(seed, (uint32_t)h, n, idx);
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      const double4 v = src.load(b, idx[d]);
      q[d][0] = v.x; q[d][1] = v.y; qp[d][0] = v.z; qp[d][1] = v.w;
    }
    FRONT_STAMP(0);
    essential_basis(q, qp, Eb);
    FRONT_STAMP(1);
    if (COOP) {
      build_equations_quad(Eb, A, qs);
    } else {
      build_equations(Eb, A);
      FRONT_STAMP(2);
      reduce_equations(A);
    }
  }
  if (COOP) {
    __syncthreads();                           // the 16 records are written
    FRONT_STAMP(2);
    if (act) quad_reduce(A, qs);               // act is uniform per quad: its DPP exchanges stay within it
    __syncthreads();
    if (!act || qs != 0) return;
    raise_degree(A);
  }
  FRONT_STAMP(3);
  double poly[11];
  determinant_poly(A, poly);
  FRONT_STAMP(4);
  const size_t hb = (size_t)b * H + h;
#pragma unroll
  for (int e = 0; e < 9; ++e)
#pragma unroll
    for (int k = 0; k < 4; ++k) st_at(st, stride, kStEb + e * 4 + k, hb) = Eb[e].c[k];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      st_at(st, stride, kStA + i * 3 + j, hb) = A.e0[i][j];
      st_at(st, stride, kStA + 9 + i * 3 + j, hb) = A.e1[i][j];
      st_at(st, stride, kStA + 18 + i * 3 + j, hb) = A.e2[i][j];
      st_at(st, stride, kStA + 27 + i * 3 + j, hb) = A.e3[i][j];
    }
#pragma unroll
  for (int i = 0; i < 3; ++i) st_at(st, stride, kStA + 36 + i, hb) = A.e4[i];
#pragma unroll
  for (int d = 0; d < 5; ++d) {
    st_at(st, stride, kStQ + 4 * d + 0, hb) = q[d][0];
    st_at(st, stride, kStQ + 4 * d + 1, hb) = q[d][1];
    st_at(st, stride, kStQ + 4 * d + 2, hb) = qp[d][0];
    st_at(st, stride, kStQ + 4 * d + 3, hb) = qp[d][1];
  }
#pragma unroll
  for (int i = 0; i <= 10; ++i) st_at(st, stride, kStPoly + i, hb) = poly[i];
  FRONT_STAMP(5);
}

#ifdef SFM_ROOTS_STATS
__device__ unsigned long long g_roots_cycles[1 << 17];
extern "C" int sfm_experiment_roots_stats(unsigned int* evals, unsigned int* falsi, unsigned long long* cycles,
                                          unsigned long long* phases, int n, int reset) {
  if (reset) {
    static unsigned int z4[1 << 17];
    static unsigned long long z8[1 << 17];
    static unsigned long long zp[4][1 << 17];
    return (hipMemcpyToSymbol(HIP_SYMBOL(g_roots_evals), z4, sizeof(z4)) == hipSuccess &&
            hipMemcpyToSymbol(HIP_SYMBOL(g_roots_falsi), z4, sizeof(z4)) == hipSuccess &&
            hipMemcpyToSymbol(HIP_SYMBOL(g_roots_phase), zp, sizeof(zp)) == hipSuccess &&
            hipMemcpyToSymbol(HIP_SYMBOL(g_roots_cycles), z8, sizeof(z8)) == hipSuccess) ? 0 : 2;
  }
  return (hipMemcpyFromSymbol(evals, HIP_SYMBOL(g_roots_evals), n * 4) == hipSuccess &&
          hipMemcpyFromSymbol(falsi, HIP_SYMBOL(g_roots_falsi), n * 4) == hipSuccess &&
          hipMemcpyFromSymbol(phases, HIP_SYMBOL(g_roots_phase), 4 * (1 << 17) * 8) == hipSuccess &&
          hipMemcpyFromSymbol(cycles, HIP_SYMBOL(g_roots_cycles), n * 8) == hipSuccess) ? 0 : 2;
}
#endif

__global__ __launch_bounds__(64) void k_roots(int H, int lanes, double* __restrict__ st, size_t stride,
                                              int32_t* __restrict__ out_nroots) {
  const int b = blockIdx.y;
  if ((int)threadIdx.x >= lanes) return;
  const int h = blockIdx.x * lanes + threadIdx.x;
  if (h >= H) return;
#ifdef SFM_ROOTS_STATS
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  const size_t hb = (size_t)b * H + h;
  double poly[11];
#pragma unroll
  for (int i = 0; i <= 10; ++i) poly[i] = st_at(st, stride, kStPoly + i, hb);
#ifdef SFM_ROOTS_STATS
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long tl = __builtin_amdgcn_s_memtime();
  g_roots_cycles[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x + (1 << 16)] = tl - t0;
#endif
  double roots[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) roots[i] = 0.0;
  __shared__ double s_lohi[kStkDepth * 2 * kStkLanes];
  __shared__ int s_ints[kStkDepth * 4 * kStkLanes];
  const IsoStack stk{s_lohi + threadIdx.x, s_ints + threadIdx.x};
  const int nr = real_roots_r(poly, roots, stk);
#pragma unroll
  for (int i = 0; i < 10; ++i) st_at(st, stride, kStRoots + i, hb) = roots[i];
  out_nroots[hb] = nr;
#ifdef SFM_ROOTS_STATS
  g_roots_cycles[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x] =
      __builtin_amdgcn_s_memtime() - t0;
#endif
}

// SOLVE_COOP (tuning key solve_coop, default): one DPP quad per hypothesis,
// lane s taking roots s, s + 4, s + 8; the accepted roots' slots come from a
// quad-wide mask of the cheirality results, so the writes are the one-lane
// loop's (accepted E / P in root order; slot 0 = root 0's E when no root is
// accepted).  Four times the waves of the one-lane kernel, whose 512 waves
// left half the SIMDs idle and followed each wave's most-rooted hypothesis.
template <bool COOP>
__global__ __launch_bounds__(64) void k_solve_back(int H, int cheir, const double* __restrict__ st, size_t stride,
                                                   const int32_t* __restrict__ nroots,
                                                   int32_t* __restrict__ out_ncand, double* __restrict__ hypE,
                                                   double* __restrict__ hypP) {
  const int b = blockIdx.y;
  const int qs = COOP ? (int)threadIdx.x & 3 : 0;
  const int h = COOP ? blockIdx.x * 16 + ((int)threadIdx.x >> 2) : blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = h < H;
  if (!COOP && !act) return;
  const size_t hb = (size_t)b * H + (act ? h : 0);
  const int nr = act ? nroots[hb] : 0;
  const int nv = nr > 0 ? (nr < 10 ? nr : 10) : 0;
  Lin Eb[9];
  Eqs A;   // only the blocks compute_E_matrix reads
  double q[5][2], qp[5][2];
  if (act) {
#pragma unroll
    for (int e = 0; e < 9; ++e)
#pragma unroll
      for (int k = 0; k < 4; ++k) Eb[e].c[k] = st[(kStEb + e * 4 + k) * stride + hb];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        A.e0[i][j] = st[(kStA + i * 3 + j) * stride + hb];
        A.e1[i][j] = st[(kStA + 9 + i * 3 + j) * stride + hb];
        A.e2[i][j] = st[(kStA + 18 + i * 3 + j) * stride + hb];
        A.e3[i][j] = st[(kStA + 27 + i * 3 + j) * stride + hb];
      }
#pragma unroll
    for (int i = 0; i < 3; ++i) A.e4[i] = st[(kStA + 36 + i) * stride + hb];
#pragma unroll
    for (int d = 0; d < 5; ++d) {
      q[d][0] = st[(kStQ + 4 * d + 0) * stride + hb];
      q[d][1] = st[(kStQ + 4 * d + 1) * stride + hb];
      qp[d][0] = st[(kStQ + 4 * d + 2) * stride + hb];
      qp[d][1] = st[(kStQ + 4 * d + 3) * stride + hb];
    }
  }
  double* Eo = hypE + hb * kMaxSlots * 9;
  double* Po = hypP + hb * kMaxSlots * 12;
  if (!COOP) {
    int nc = 0;
    for (int m = 0; m < nv; ++m) {
      const double w = st[(kStRoots + m) * stride + hb];
      double E[9];
      essential_at_root(Eb, A, w, E);
      if (!cheir) {
#pragma unroll
        for (int e = 0; e < 9; ++e) Eo[m * 9 + e] = E[e];
        ++nc;
        continue;
      }
      double Pm[12];
      const bool ok = cheirality_P(E, q, qp, Pm);
      // compaction (cheirality.cu:142-146): accepted E's move to the front; if
      // none is accepted slot 0 keeps root 0's E.
      if (ok) {
#pragma unroll
        for (int e = 0; e < 9; ++e) Eo[nc * 9 + e] = E[e];
#pragma unroll
        for (int e = 0; e < 12; ++e) Po[nc * 12 + e] = Pm[e];
        ++nc;
      } else if (m == 0) {
#pragma unroll
        for (int e = 0; e < 9; ++e) Eo[e] = E[e];
      }
    }
    out_ncand[hb] = nc;
    return;
  }
  // quad: roots m = qs + 4t
  double E[3][9], Pm[3][12];
  int okbits = 0;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int m = qs + 4 * t;
    if (m < nv) {
      const double w = st[(kStRoots + m) * stride + hb];
      essential_at_root(Eb, A, w, E[t]);
      const bool ok = !cheir || cheirality_P(E[t], q, qp, Pm[t]);
      if (ok) okbits |= 1 << m;
    }
  }
  // the quad's accepted-root mask (roots 0..9), OR-reduced over the four lanes
  okbits |= __builtin_amdgcn_update_dpp(0, okbits, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  okbits |= __builtin_amdgcn_update_dpp(0, okbits, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  if (!act) return;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int m = qs + 4 * t;
    if (m < nv) {
      if ((okbits >> m) & 1) {
        const int slot = __popc(okbits & ((1 << m) - 1));
#pragma unroll
        for (int e = 0; e < 9; ++e) Eo[slot * 9 + e] = E[t][e];
        if (cheir)
#pragma unroll
          for (int e = 0; e < 12; ++e) Po[slot * 12 + e] = Pm[t][e];
      } else if (m == 0 && okbits == 0) {
#pragma unroll
        for (int e = 0; e < 9; ++e) Eo[e] = E[t][e];
      }
    }
  }
  if (qs == 0) out_ncand[hb] = __popc(okbits);
}

// ---------------------------------------------------------------------------
// Fast inlier decision: error bound (derivation in DESIGN.md, "Scoring").
//
// With u = 2^-53, R = sum |E_ij| and M = max(1, |x|, |y|, |x'|, |y'|), the
// FMA-evaluated quantities used below differ from the values the reference's
// operation order produces by at most
//     |a_f - a_r| <= 11 u M^2 R,   ||v_f - v_r|| <= 10.0002 u R M
// (v = (Ex0, Ex1, xE0, xE1), a = x'^T E x, D = ||v||^2).  Deciding
//     inlier  if a_f^2 < thr^2 (1 - 2^-22) D_f,
//     outlier if a_f^2 > thr^2 (1 + 2^-22) D_f
// is then provably identical to the reference's IEEE test whenever
//     D_f >= (u R M^2 G)^2,   G = 2^24 (11 + 11/thr),
// and 2^-40 <= thr < 1, 2^-100 <= R <= 2^100, M <= 2^100.  Every other
// (candidate, point) pair takes the exact path.  Per candidate the constant
// Kg = (u R G)^2 is stored in candE[9] (NaN disables the fast path); per
// point mm2 = M^4, so the guard is D_f >= Kg * mm2.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double guard_constant(const double* E, double g) {
  double R = 0.0;
#pragma unroll
  for (int e = 0; e < 9; ++e) R += fabs(E[e]);
  if (!(R >= 0x1p-100 && R <= 0x1p100) || !(g > 0.0)) return __builtin_nan("");
  const double k = 0x1p-53 * R * g;
  return k * k;
}

// ---------------------------------------------------------------------------
// Float32 pre-decision (k_score32).  With u = 2^-24, M = max(1, |x|, |y|,
// |x'|, |y'|) <= 2^12 and R = sum|E_ij| in [2^-30, 2^30], the float32 FMA
// evaluation (inputs rounded to float32) satisfies
//     |a_s - a*| <= alpha = 8 u R M^2,   ||v_s - v*|| <= beta = 8.1 u R M
// against the exact values a*, v* of the float64 inputs (7.1 u R M^2 and
// 8.02 u R M by the standard bounds; the reference's own float64 error is far
// below the slack).  Bounding the cross terms 2|a|alpha and 2 sqrt(D) beta by
// AM-GM with weight 2^7 turns the reference test into two sign tests:
//     inlier  if fma(-t2lo, D, a*a) < -eps1
//     outlier if fma(-t2hi, D, a*a) >  eps2
//     eps1 = 129 alpha^2 + 128 thr^2 beta^2           = A1 M^4 + B1 M^2
//     eps2 = (128 alpha^2 + 129 thr^2 beta^2)/(1-2^-7) = A2 M^4 + B2 M^2
//     t2lo = thr^2 (1 - 2^-6 - 2^-19),  t2hi = thr^2 (1 + 2^-7)/(1 - 2^-7) (1 + 2^-19)
// (rounding is monotone and +-eps are floats, so each compare implies the
// exact inequality on aa = fl(a^2); aa is within u of a^2, the same loss as
// rounding a^2 + eps once; derivation in DESIGN.md, "Scoring").  Anything else
// is undecided and re-evaluated by the float64 path.  A*, B* carry a 2^-20
// upward slack that covers their float32 rounding and the float32 operations
// forming eps; slots 14/15 hold -eps1 and eps2 at M = 1 (the common case).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fp32_constants(const double* E, double thr, bool enable, float* out) {
  double R = 0.0;
  bool finite = true;
#pragma unroll
  for (int e = 0; e < 9; ++e) {
    R += fabs(E[e]);
    finite = finite && isfinite(E[e]);
  }
  const bool ok = enable && finite && R >= 0x1p-30 && R <= 0x1p30;
#pragma unroll
  for (int e = 0; e < 9; ++e) out[e] = ok ? (float)E[e] : 0.0f;
  const double al = 8.0 * 0x1p-24 * R * (1.0 + 0x1p-20) + 0x1p-120;
  const double be = 8.1 * 0x1p-24 * R * (1.0 + 0x1p-20) + 0x1p-120;
  const double t2 = thr * thr, up = 1.0 + 0x1p-20;
  const double A1 = 129.0 * al * al * up, B1 = 128.0 * t2 * be * be * up;
  const double A2 = 128.0 * al * al / (1.0 - 0x1p-7) * up, B2 = 129.0 * t2 * be * be / (1.0 - 0x1p-7) * up;
  out[9] = ok ? (float)A1 : 0.0f;
  out[10] = ok ? (float)B1 : 0.0f;
  out[11] = ok ? (float)A2 : 0.0f;
  out[12] = ok ? (float)B2 : 0.0f;
  out[13] = ok ? 1.0f : 0.0f;
  out[14] = ok ? -(float)((A1 + B1) * up) : 0.0f;
  out[15] = ok ? (float)((A2 + B2) * up) : 0.0f;
}

// ---------------------------------------------------------------------------
// Phase 2: chains and the dense candidate list
//   k_chain  one block of 512 per pair: exclusive scan of the candidate counts
//            over chains (chain t owns hypotheses t*iters .. t*iters+iters-1)
//   k_cand   one thread per (hypothesis, slot): the candidate records
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kChains) void k_chain(int H, int iters, const int32_t* __restrict__ nroots,
                                                   const int32_t* __restrict__ ncand, int32_t* __restrict__ cand_off,
                                                   int32_t* __restrict__ chain_ref, int32_t* __restrict__ cand_total,
                                                   unsigned long long* __restrict__ skipped) {
  __shared__ int32_t s_sum[kChains / 64];
  const int b = blockIdx.x, t = threadIdx.x;
  // the call's pruning counter (first chunk only; it accumulates over chunks),
  // zeroed here rather than by a memset launch of its own
  if (skipped && b == 0 && t == 0) *skipped = 0ull;
  const size_t hb0 = (size_t)b * H + (size_t)t * iters;
  int cnt = 0;
  for (int i = 0; i < iters; ++i) {
    const int nc = ncand[hb0 + i];
    cnt += nc > 0 ? nc : 1;
  }
  const int lane = t & 63, wv = t >> 6;
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  if (lane == 63) s_sum[wv] = incl;
  __syncthreads();
  int off = incl - cnt;
  for (int w = 0; w < wv; ++w) off += s_sum[w];
  if (t == kChains - 1) cand_total[b] = off + cnt;
  // the same walk records, per hypothesis, the slot-0 state the reference
  // thread holds (kernel_functions.cu:154, 179): the chain's latest hypothesis
  // with a root (E) up to i, and with an accepted candidate (P) before i, so
  // that k_cand reads them in O(1) instead of looking back along the chain
  int ke = -1, kp = -1;
  for (int i = 0; i < iters; ++i) {
    const int nc = ncand[hb0 + i];
    if (nroots[hb0 + i] > 0) ke = i;
    cand_off[hb0 + i] = off;
    chain_ref[hb0 + i] = (ke + 1) | ((kp + 1) << 16);
    off += nc > 0 ? nc : 1;
    if (nc > 0) kp = i;
  }
}

// A hypothesis with no candidate rescores slot 0 as the reference thread
// holds it (kernel_functions.cu:154, 179-214): E of the chain's latest
// hypothesis with a root, P of its latest with an accepted candidate (zeros
// before any), as k_chain recorded them (chain_ref).
__global__ __launch_bounds__(256) void k_cand(int H, int iters, int cheir, const int32_t* __restrict__ chain_ref,
                                              const int32_t* __restrict__ ncand, const double* __restrict__ hypE,
                                              const double* __restrict__ hypP, double* __restrict__ hypP0,
                                              const int32_t* __restrict__ cand_off, double* __restrict__ candE,
                                              int cmax, double guard_g, double thr, int fast32,
                                              int32_t* __restrict__ cntT, int32_t* __restrict__ cntR) {
  const int b = blockIdx.y;
  const int g = blockIdx.x * 256 + threadIdx.x;
  const int h = g / kMaxSlots, j = g - h * kMaxSlots;
  if (h >= H) return;
  const size_t hb0 = (size_t)b * H;
  const size_t hb = hb0 + h;
  const int nc = ncand[hb];
  if (j >= (nc > 0 ? nc : 1)) return;
  const size_t ci = (size_t)b * cmax + cand_off[hb] + j;
  double* dst = candE + ci * kCandStride;
  // the scorers add into the counts of candidates < cand_total only: zeroing
  // them with their records replaces two memset launches per call
  cntT[ci] = 0;
  cntR[ci] = 0;
  if (nc > 0) {
    const double* Eh = hypE + (hb * kMaxSlots + j) * 9;
#pragma unroll
    for (int e = 0; e < 9; ++e) dst[e] = Eh[e];
  } else {
    const int i = h % iters;
    const size_t c0 = hb - i;   // the chain's first hypothesis
    const int ref = chain_ref[hb];
    const int ke = (ref & 0xffff) - 1, kp = cheir ? (ref >> 16) - 1 : -1;
#pragma unroll
    for (int e = 0; e < 9; ++e) dst[e] = ke >= 0 ? hypE[(c0 + ke) * kMaxSlots * 9 + e] : 0.0;
#pragma unroll
    for (int e = 0; e < 12; ++e) hypP0[hb * 12 + e] = kp >= 0 ? hypP[(c0 + kp) * kMaxSlots * 12 + e] : 0.0;
  }
  dst[9] = guard_constant(dst, guard_g);
  fp32_constants(dst, thr, fast32 != 0, reinterpret_cast<float*>(dst + 10));
}

// ---------------------------------------------------------------------------
// Phase 3: scoring
// ---------------------------------------------------------------------------
struct ScoreConsts {
  double thr, t2lo, t2hi;
  float t2lo32, t2hi32;
  int fast32;
  int prune;      // exact bound pruning on (PruneState)
  int interleave; // k_score32 item order: pairs interleaved (1) or one after another (0)
  int ws_batch;   // pairs the workspace was laid out for (locates PruneState)
};

// Exact bound pruning in k_score32 (tuning key score_prune; only when
// num_test == num_ransac_test, SFMnet's case, and no per-hypothesis scores
// are requested).  A candidate's final count is at most its count so far plus
// the points not yet scored for it.  Once that bound is below the largest
// count any candidate of the pair has reached so far, the candidate can be
// neither the winner nor decide it, so its remaining spans are skipped:
//   * best_lb only ever holds partial counts, each <= its candidate's final
//     count <= the winning score.
//   * a pruned candidate's true count is < best_lb.  If it loses its
//     hypothesis's preselection because its partial count is lower, that
//     hypothesis's true best is < best_lb too, so it cannot win.  Any
//     hypothesis or chain reaching the winning score has only unpruned, exact
//     counts (ties included).
//   * cov packs (count, points covered) in one 64-bit atomic, so every read
//     is a consistent snapshot.  Updates only lower count + (T - covered), and
//     only raise best_lb, so stale reads only prune less.
// The winner, its count, E and P are therefore identical with pruning on or
// off.  The per-hypothesis scores of losing hypotheses are lower bounds.
constexpr uint32_t kPrunedFlag = 0xBF800000u;   // record slot 10+13 (ok32) of a pruned candidate: -1.0f
constexpr int kBestStride = 64;                  // best_lb[b * kBestStride]: one 256-byte line per pair

// The pruning state follows cntR in the workspace (layout): cov [B][cmax]
// (count | points covered << 32), best_lb [64], skipped.  The score kernel
// derives it from cntR where it is used: its SGPRs are at the limit, and
// three more live pointers spill the hot loop.
struct PruneState {
  unsigned long long* cov;
  int32_t* best_lb;
  unsigned long long* skipped;
};
__host__ __device__ inline PruneState prune_state(int32_t* cntR, int ws_batch, int cmax) {
  char* p = reinterpret_cast<char*>(cntR) + align_up((size_t)ws_batch * cmax * 4);
  PruneState st;
  st.cov = reinterpret_cast<unsigned long long*>(p);
  p += align_up((size_t)ws_batch * cmax * 8);
  st.best_lb = reinterpret_cast<int32_t*>(p);
  p += align_up((size_t)SFM_MAX_BATCH * kBestStride * 4);
  st.skipped = reinterpret_cast<unsigned long long*>(p);
  return st;
}

// Exact reference evaluation (ComputeError, kernel_functions.cu:232-264).
__device__ __forceinline__ bool inlier_exact(double a, double D, double thr) {
  double e = a / sqrt(D);
  if (e < 0.0) e = -e;
  return e <= thr;
}

// Reference operation order, no contraction (ComputeError).
__device__ __forceinline__ bool inlier_reference(const double* E, double x, double y, double xp, double yp,
                                                 double thr) {
  const double ex0 = (E[0] * x + E[1] * y) + E[2];
  const double ex1 = (E[3] * x + E[4] * y) + E[5];
  const double ex2 = (E[6] * x + E[7] * y) + E[8];
  const double xe0 = (xp * E[0] + yp * E[3]) + E[6];
  const double xe1 = (xp * E[1] + yp * E[4]) + E[7];
  const double a = (xp * ex0 + yp * ex1) + ex2;
  const double D = ((ex0 * ex0 + ex1 * ex1) + xe0 * xe0) + xe1 * xe1;
  return inlier_exact(a, D, thr);
}

// mm2 = M^4 for the fast-path guard (NaN for non-finite / huge coordinates)
__device__ __forceinline__ double point_scale(double x, double y, double xp, double yp) {
  double M = fmax(fmax(fabs(x), fabs(y)), fmax(fabs(xp), fabs(yp)));
  M = fmax(M, 1.0);
  if (!(M <= 0x1p100)) return __builtin_nan("");
  const double M2 = M * M;
  return M2 * M2;
}

// Wave-uniform value copied into a VGPR: one VALU op may read only one SGPR,
// so the FMA-chain addends are broadcast once per candidate instead of being
// re-materialised for every point.
__device__ __forceinline__ double to_vgpr(double s) {
  double v;
  asm("v_mov_b64 %0, %1" : "=v"(v) : "s"(s));
  return v;
}

struct Addends { double e2, e5, e8, e6, e7; };

// UNITM: every point of the chunk has M = 1 (mm2 = 1), so the guard is D >= Kg
template <bool FAST, bool UNITM>
__device__ __forceinline__ bool inlier_test(const double* E, const Addends& ad, double Kg, double x, double y,
                                            double xp, double yp, double mm2, const ScoreConsts& k) {
  if (!FAST) return inlier_reference(E, x, y, xp, yp, k.thr);
  const double ex0 = fma(E[0], x, fma(E[1], y, ad.e2));
  const double ex1 = fma(E[3], x, fma(E[4], y, ad.e5));
  const double ex2 = fma(E[6], x, fma(E[7], y, ad.e8));
  const double xe0 = fma(xp, E[0], fma(yp, E[3], ad.e6));
  const double xe1 = fma(xp, E[1], fma(yp, E[4], ad.e7));
  const double a = fma(xp, ex0, fma(yp, ex1, ex2));
  const double D = fma(xe1, xe1, fma(xe0, xe0, fma(ex1, ex1, ex0 * ex0)));
  const double lhs = a * a;
  const bool g = UNITM ? (D >= Kg) : (D >= Kg * mm2);
  const bool fin = g && (lhs < k.t2lo * D);
  const bool fout = g && (lhs > k.t2hi * D);
  bool in = fin;
  if (!(fin || fout)) in = inlier_reference(E, x, y, xp, yp, k.thr);
  return in;
}

// Reduced-precision scoring (tuning key score_precision; BASELINE C5's fp32 vs
// fp16 inlier-set sweep).  Two forms; the reference itself only ever
// instantiates ComputeError<double> (kernel_functions.cu:193, 210), so neither
// has a reference output and both are pinned only to this build's oracle
// restatement (parity unpinned against the reference):
//   * "held in T" (score_precision 32 / 16, inlier_lowp below): this build's
//     own variant, NOT the reference's template.  E, q, qp and every
//     operation of ComputeError's expression tree in T (RNE, source order, no
//     contraction), sqrt and division correctly rounded in T.  E is first
//     scaled by a power of two (exact; the error is invariant to the scale of
//     E).  Inputs reach T through float32 (float64 -> float32 -> T).  For T =
//     half the sqrt and the division run in float32 and round once to half:
//     float32 carries 24 >= 2*11 + 2 bits, so that double rounding is exact.
//     oracle/ransac5_oracle.cpp:is_inlier_lp restates it.
//   * "template" (score_lowp_template 1, inlier_lowp_tpl): what a literal
//     ComputeError<T> instantiation computes with the reference's Ematrix =
//     double[3][3] (common.h:26).  q, qp are T; each E[k][l] * q[l] is a
//     double product (T widened exactly), `sum += ...` adds in double and
//     rounds the sum to T; xEx, D, sqrt and the division are T arithmetic.
//     No scaling of E.  oracle/ransac5_oracle.cpp:is_inlier_lp_tpl restates it.
// Both end with the call site's `error <= c_inlier_threshold` against the
// float64 threshold (kernel_functions.cu:193-194).
template <int PREC>
struct LowP { using T = float; };
template <>
struct LowP<16> { using T = _Float16; };
template <>
struct LowP<17> { using T = _Float16; };

// float64 -> binary16, rounded once (ties to even; subnormals; overflow to
// inf): the conversion of `T q_test[3] = {qs[..], ...}` for T = half.  The
// quantum arithmetic is exact in float64 (oracle: h16d).
__device__ __forceinline__ _Float16 h16_of_double(double v) {
  if (!(fabs(v) < 65520.0)) return (_Float16)(float)v;       // inf / nan / past max + half an ulp
  const double a = fabs(v);
  double q;
  if (a < 0x1p-14) {
    q = 0x1p-24;
  } else {
    int e;
    (void)frexp(a, &e);
    q = ldexp(1.0, e - 1 - 10);
  }
  return (_Float16)(float)copysign(rint(a / q) * q, v);      // representable: the conversions are exact
}
__device__ __forceinline__ float lowp_of_double(double v, float) { return (float)v; }
__device__ __forceinline__ _Float16 lowp_of_double(double v, _Float16) { return h16_of_double(v); }

// the literal template form (PREC 33 = float, 17 = half; see above)
template <int PREC>
__device__ __forceinline__ bool inlier_lowp_tpl(const double* E, double xd, double yd, double xpd, double ypd,
                                                double thr) {
  using T = typename LowP<PREC>::T;
  const T q[3] = {lowp_of_double(xd, T()), lowp_of_double(yd, T()), (T)1.0f};
  const T qp[3] = {lowp_of_double(xpd, T()), lowp_of_double(ypd, T()), (T)1.0f};
  T Ex[3], xE[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    T sum = (T)0.0f;
#pragma unroll
    for (int l = 0; l < 3; ++l) {
      const double p = E[3 * k + l] * (double)q[l];
      const double t = (double)sum + p;
      sum = lowp_of_double(t, T());
    }
    Ex[k] = sum;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    T sum = (T)0.0f;
#pragma unroll
    for (int l = 0; l < 3; ++l) {
      const double p = (double)qp[l] * E[3 * l + k];
      const double t = (double)sum + p;
      sum = lowp_of_double(t, T());
    }
    xE[k] = sum;
  }
  T xEx = (T)0.0f, m;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    m = qp[k] * Ex[k];
    xEx = xEx + m;
  }
  T D, m0, m1;
  m0 = Ex[0] * Ex[0]; m1 = Ex[1] * Ex[1]; D = m0 + m1;
  m0 = xE[0] * xE[0]; D = D + m0;
  m0 = xE[1] * xE[1]; D = D + m0;
  const T d = (T)sqrtf((float)D);
  T err = (T)((float)xEx / (float)d);
  if (err < (T)0.0f) err = -err;
  return (double)(float)err <= thr;
}

template <int PREC>
__device__ __forceinline__ bool inlier_lowp(const double* E, double xd, double yd, double xpd, double ypd,
                                            double thr) {
  using T = typename LowP<PREC>::T;
  // E scaled by a power of two to max |E_ij| in [0.5, 1): exact in float64,
  // and the Sampson error is invariant to the scale of E; without it a
  // five-point E of small norm underflows in half
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < 9; ++i) m = fmax(m, fabs(E[i]));
  int ex = 0;
  if (m > 0.0 && m < 0x1p1000) (void)frexp(m, &ex);
  T e[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) e[i] = (T)(float)ldexp(E[i], -ex);
  const T x = (T)(float)xd, y = (T)(float)yd, xp = (T)(float)xpd, yp = (T)(float)ypd;
  // every intermediate is a named T: assignment rounds each operation to T
  T m0, m1, s;
  m0 = e[0] * x; m1 = e[1] * y; s = m0 + m1; const T ex0 = s + e[2];
  m0 = e[3] * x; m1 = e[4] * y; s = m0 + m1; const T ex1 = s + e[5];
  m0 = e[6] * x; m1 = e[7] * y; s = m0 + m1; const T ex2 = s + e[8];
  m0 = xp * e[0]; m1 = yp * e[3]; s = m0 + m1; const T xe0 = s + e[6];
  m0 = xp * e[1]; m1 = yp * e[4]; s = m0 + m1; const T xe1 = s + e[7];
  m0 = xp * ex0; m1 = yp * ex1; s = m0 + m1; const T a = s + ex2;
  T D;
  m0 = ex0 * ex0; m1 = ex1 * ex1; D = m0 + m1;
  m0 = xe0 * xe0; D = D + m0;
  m0 = xe1 * xe1; D = D + m0;
  const T d = (T)sqrtf((float)D);
  T err = (T)((float)a / (float)d);
  if (err < (T)0.0f) err = -err;
  return (double)(float)err <= thr;
}

// Level-3 test (reference order), kept as a named call site for the drain.
__device__ __forceinline__
bool inlier_reference_call(const double* E, double x, double y, double xp, double yp,
                                                   double thr) {
  return inlier_reference(E, x, y, xp, yp, thr);
}

// One chunk (kPPL points per lane) against the tile's nc candidates.  One
// ballot per (candidate, point); the num_test / num_ransac_test prefixes are
// applied as precomputed wave masks (SAME: both prefixes equal, one count).
template <bool FAST, bool UNITM, bool SAME, int PREC>
__device__ __forceinline__ void score_chunk(const double* __restrict__ CE, int nc, const double (&x)[kPPL],
                                            const double (&y)[kPPL], const double (&xp)[kPPL],
                                            const double (&yp)[kPPL], const double (&mm2)[kPPL],
                                            const uint64_t (&mT)[kPPL], const uint64_t (&mR)[kPPL],
                                            const ScoreConsts& kc, int lane, int32_t (*cnt)[2]) {
  for (int c = 0; c < nc; ++c) {
    double E[9];
#pragma unroll
    for (int e = 0; e < 9; ++e) E[e] = CE[(size_t)c * kCandStride + e];
    const double Kg = CE[(size_t)c * kCandStride + 9];
    Addends ad;
    if (FAST) ad = Addends{to_vgpr(E[2]), to_vgpr(E[5]), to_vgpr(E[8]), to_vgpr(E[6]), to_vgpr(E[7])};
    int sT = 0, sR = 0;
#pragma unroll
    for (int k = 0; k < kPPL; ++k) {
      const bool in = PREC == 64 ? inlier_test<FAST, UNITM>(E, ad, Kg, x[k], y[k], xp[k], yp[k], mm2[k], kc)
                      : (PREC & 1) ? inlier_lowp_tpl<PREC>(E, x[k], y[k], xp[k], yp[k], kc.thr)
                                   : inlier_lowp<PREC>(E, x[k], y[k], xp[k], yp[k], kc.thr);
      const uint64_t m = __ballot(in);
      sT += __popcll(m & mT[k]);
      if (!SAME) sR += __popcll(m & mR[k]);
    }
    if (SAME) sR = sT;
    if (lane == 0) {
      cnt[c][0] += sT;
      cnt[c][1] += sR;
    }
  }
}

template <bool FAST, class Src, int PREC = 64>
__global__ __launch_bounds__(kScoreThreads) void k_score(const Src src, PairParams pp, int batch, int cmax,
                                                         const int32_t* __restrict__ cand_total,
                                                         const double* __restrict__ candE,
                                                         int32_t* __restrict__ cntT, int32_t* __restrict__ cntR,
                                                         ScoreConsts kc) {
  __shared__ int32_t s_cnt[kScoreThreads / 64][kKC][2];
  __shared__ int32_t s_items[SFM_MAX_BATCH + 1];
  __shared__ int32_t s_tiles[SFM_MAX_BATCH];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) {
    int acc = 0;
    for (int b = 0; b < batch; ++b) {
      const int tiles = (cand_total[b] + kKC - 1) / kKC;
      s_tiles[b] = tiles;
      s_items[b] = acc;
      acc += tiles * pp.splits[b];
    }
    s_items[batch] = acc;
  }
  for (int i = tid; i < (kScoreThreads / 64) * kKC * 2; i += kScoreThreads) (&s_cnt[0][0][0])[i] = 0;
  __syncthreads();
  const int total = s_items[batch];
  for (int item = blockIdx.x; item < total; item += gridDim.x) {
    int b = 0;
    while (item >= s_items[b + 1]) ++b;
    const int local = item - s_items[b];
    const int tiles = s_tiles[b];
    const int split = local / tiles, tile = local - split * tiles;
    const int ctot = cand_total[b];
    const int c0 = tile * kKC;
    const int nc = min(kKC, ctot - c0);
    const int T = pp.test[b], R = pp.rtest[b];
    const int M = max(T, R);
    const int p0 = split * kPtsPerItem;
    const int p1 = min(M, p0 + kPtsPerItem);
    const double* CE = candE + ((size_t)b * cmax + c0) * kCandStride;
    for (int cb = p0; cb < p1; cb += kChunk) {
      double x[kPPL], y[kPPL], xp[kPPL], yp[kPPL], mm2[kPPL];
      uint64_t mT[kPPL], mR[kPPL];
      bool unit = true;
#pragma unroll
      for (int k = 0; k < kPPL; ++k) {
        const int p = cb + k * kScoreThreads + tid;
        const bool ok = p < p1;
        const double4 v = src.load(b, ok ? p : p0);
        x[k] = v.x; y[k] = v.y; xp[k] = v.z; yp[k] = v.w;
        mm2[k] = point_scale(v.x, v.y, v.z, v.w);
        unit = unit && (mm2[k] == 1.0);
        mT[k] = __ballot(ok && p < T);
        mR[k] = __ballot(ok && p < R);
      }
      const bool all_unit = __all(unit);
      if (T == R) {
        if (all_unit) score_chunk<FAST, true, true, PREC>(CE, nc, x, y, xp, yp, mm2, mT, mR, kc, lane, s_cnt[wv]);
        else score_chunk<FAST, false, true, PREC>(CE, nc, x, y, xp, yp, mm2, mT, mR, kc, lane, s_cnt[wv]);
      } else {
        if (all_unit) score_chunk<FAST, true, false, PREC>(CE, nc, x, y, xp, yp, mm2, mT, mR, kc, lane, s_cnt[wv]);
        else score_chunk<FAST, false, false, PREC>(CE, nc, x, y, xp, yp, mm2, mT, mR, kc, lane, s_cnt[wv]);
      }
    }
    __syncthreads();
    if (tid < nc * 2) {
      const int c = tid >> 1, which = tid & 1;
      int s = 0;
#pragma unroll
      for (int w = 0; w < kScoreThreads / 64; ++w) { s += s_cnt[w][c][which]; s_cnt[w][c][which] = 0; }
      if (s) atomicAdd((which ? cntR : cntT) + (size_t)b * cmax + c0 + c, s);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Phase 3b: scoring with the float32 pre-decision (fp32_constants).
// Only float32 copies of the points stay in registers.  (Plain v_fma_f32
// issues at twice the fp64 rate on gfx950; packed v_pk_fma_f32 measured no
// faster.)  The kernel sits at the measured VALU issue ceiling
// (git-history scripts/probe_vgpr_bank.hip: ~1.15-1.3 ns per wave-FMA per SIMD at 4-8
// waves), so its cost is its VALU count: 21 per evaluation in the common
// path.  Undecided evaluations and lanes with a coordinate beyond 2^12 are
// queued and re-tested in float64.
// ---------------------------------------------------------------------------

#ifdef SFM_SCORE_STATS
// experiment builds only (git-history scripts/score_experiment.py): (candidate, point
// slot) wave iterations, those with an undecided lane, undecided evaluations
__device__ unsigned long long g_score_stats[3];
extern "C" int sfm_experiment_score_stats(unsigned long long* out3) {
  return hipMemcpyFromSymbol(out3, HIP_SYMBOL(g_score_stats), 24) == hipSuccess ? 0 : 2;
}
#endif

// float64 decision of one (reloaded) point; guard per point (any scale)
__device__ __forceinline__ bool inlier_f64v(const double* __restrict__ Ec, const double4 v, const ScoreConsts& kc) {
  double E[9];
#pragma unroll
  for (int e = 0; e < 9; ++e) E[e] = Ec[e];
  const double x = v.x, y = v.y, xp = v.z, yp = v.w;
  const double ex0 = fma(E[0], x, fma(E[1], y, E[2]));
  const double ex1 = fma(E[3], x, fma(E[4], y, E[5]));
  const double ex2 = fma(E[6], x, fma(E[7], y, E[8]));
  const double xe0 = fma(xp, E[0], fma(yp, E[3], E[6]));
  const double xe1 = fma(xp, E[1], fma(yp, E[4], E[7]));
  const double a = fma(xp, ex0, fma(yp, ex1, ex2));
  const double D = fma(xe1, xe1, fma(xe0, xe0, fma(ex1, ex1, ex0 * ex0)));
  const double lhs = a * a;
  const bool g = D >= Ec[9] * point_scale(x, y, xp, yp);
  const bool fin = g && (lhs < kc.t2lo * D);
  const bool fout = g && (lhs > kc.t2hi * D);
  if (fin || fout) return fin;
  return inlier_reference_call(E, x, y, xp, yp, kc.thr);
}

// Float32 pass.  Every decision is a wave mask straight out of one compare
// (inlier: din < -eps1, outlier: dout > eps2; all finite here since the
// lane's coordinates are within 2^12 and the candidate passed ok32), so the
// bookkeeping is scalar: counts by popcount, undecided = ~(in | out) per
// point.  Undecided points are queued and re-tested in float64.

// Lanes [0, n) of a wave (n may lie outside [0, 64]).
__device__ __forceinline__ uint64_t lane_prefix(int n) {
  return n >= 64 ? ~0ull : (n <= 0 ? 0ull : ((1ull << n) - 1ull));
}

constexpr int kQueue = 1024;        // undecided (candidate, point) entries per wave (LDS)
static_assert(kQueue >= 64 * kPPL32, "the queue takes one candidate's undecided points past its low mark");

// Append the wave's undecided lanes (mask und) of one point slot to the queue.
__device__ __forceinline__ void enqueue_undecided(uint64_t und, int c, int p, int lane, uint32_t* q, int& qn) {
#ifdef SFM_SCORE_STATS
  if (lane == 0) {
    atomicAdd(&g_score_stats[0], 1ull);
    if (und) atomicAdd(&g_score_stats[1], 1ull);
    atomicAdd(&g_score_stats[2], (unsigned long long)__popcll(und));
  }
#endif
  if (!und) return;                                     // wave-uniform
  if ((und >> lane) & 1ull) {
    const int pos = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(und >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)und, 0));
    q[pos] = ((uint32_t)c << 24) | (uint32_t)p;
  }
  qn += __popcll(und);
}

// One float32 pass of a wave over candidates [c, nc) of its chunk (lane l
// holds points cb + 64k + l).  Returns the first candidate not processed: nc,
// or one met with the queue past its low mark (the caller drains the queue,
// reloads the chunk and resumes there).  The float64 test stays out of this
// loop so that its registers stay out of the hot loop's footprint.
//   MASKED: the chunk crosses the num_test (nT) or num_ransac_test (nR)
//   prefix, counted from the chunk base; SAME: both prefixes are equal.
//   GEN: some lane has M != 1 or is bad; otherwise eps are the records'
//   precomputed M = 1 values.
template <bool SAME, bool MASKED, bool GEN>
__device__ __forceinline__ int score32_pass(const double* __restrict__ CE, int c, int nc, int pl, int nT, int nR,
                                            const float (&x)[kPPL32], const float (&y)[kPPL32],
                                            const float (&xp)[kPPL32], const float (&yp)[kPPL32], float M2,
                                            uint64_t bad, const ScoreConsts& kc, int lane, int32_t (*cnt)[2],
                                            uint32_t* q, int& qn) {
  const float nt2lo = -kc.t2lo32, nt2hi = -kc.t2hi32;
  const float M4 = M2 * M2;
  for (; c < nc; ++c) {
    if (qn > kQueue - 64 * kPPL32) break;               // drain first
    const float* F = reinterpret_cast<const float*>(CE + (size_t)c * kCandStride + 10);
    int sT = 0, sR = 0;
    uint64_t undk[kPPL32];
    const uint32_t ok32 = __builtin_amdgcn_readfirstlane(__float_as_uint(F[13]));   // 1.0f, 0.0f or pruned
    if (ok32 == kPrunedFlag) continue;                  // exact bound pruning (PruneState)
    if (ok32 != 0u) {
      const float e0 = F[0], e1 = F[1], e2 = F[2], e3 = F[3], e4 = F[4], e5 = F[5], e6 = F[6], e7 = F[7], e8 = F[8];
      float neps1, eps2;
      if (GEN) {
        neps1 = -__builtin_fmaf(F[9], M4, F[10] * M2);               // per lane: its points' M
        eps2 = __builtin_fmaf(F[11], M4, F[12] * M2);
      } else {
        neps1 = F[14];
        eps2 = F[15];
      }
      // stage by stage across the kPPL32 points: independent FMA chains
      float ex0[kPPL32], ex1[kPPL32], ex2[kPPL32], xe0[kPPL32], xe1[kPPL32], a[kPPL32], D[kPPL32], aa[kPPL32];
      float din[kPPL32], dout[kPPL32];
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) ex0[k] = __builtin_fmaf(e0, x[k], __builtin_fmaf(e1, y[k], e2));
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) ex1[k] = __builtin_fmaf(e3, x[k], __builtin_fmaf(e4, y[k], e5));
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) ex2[k] = __builtin_fmaf(e6, x[k], __builtin_fmaf(e7, y[k], e8));
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) xe0[k] = __builtin_fmaf(xp[k], e0, __builtin_fmaf(yp[k], e3, e6));
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) xe1[k] = __builtin_fmaf(xp[k], e1, __builtin_fmaf(yp[k], e4, e7));
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) a[k] = __builtin_fmaf(xp[k], ex0[k], __builtin_fmaf(yp[k], ex1[k], ex2[k]));
#pragma unroll
      for (int k = 0; k < kPPL32; ++k)
        D[k] = __builtin_fmaf(xe1[k], xe1[k], __builtin_fmaf(xe0[k], xe0[k], __builtin_fmaf(ex1[k], ex1[k], ex0[k] * ex0[k])));
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) aa[k] = a[k] * a[k];
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) din[k] = __builtin_fmaf(nt2lo, D[k], aa[k]);
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) dout[k] = __builtin_fmaf(nt2hi, D[k], aa[k]);
#pragma unroll
      for (int k = 0; k < kPPL32; ++k) {
        uint64_t mi = __ballot(din[k] < neps1);
        const uint64_t mo = __ballot(dout[k] > eps2);
        uint64_t und = ~(mi | mo);
        if (GEN) {
          mi &= ~bad;
          und |= bad;
        }
        if (MASKED) {
          const uint64_t mT = lane_prefix(nT - 64 * k), mR = lane_prefix(nR - 64 * k);
          und &= mT | mR;
          sT += __popcll(mi & mT);
          if (!SAME) sR += __popcll(mi & mR);
        } else {
          sT += __popcll(mi);
        }
        undk[k] = und;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPPL32; ++k)                  // candidate outside the float32 range
        undk[k] = MASKED ? (lane_prefix(nT - 64 * k) | lane_prefix(nR - 64 * k)) : ~0ull;
    }
    // enqueue after the unrolled compares (enqueueing inside them splits the
    // FMA block per point and costs SGPRs)
#pragma unroll
    for (int k = 0; k < kPPL32; ++k) enqueue_undecided(undk[k], c, pl + 64 * k, lane, q, qn);   // pl: relative to the item
    if (SAME || !MASKED) sR = sT;
    if (lane == 0) {
      cnt[c][0] += sT;
      cnt[c][1] += sR;
    }
  }
  return c;
}

// Compacted float64 pass over the queued evaluations: 64 lanes x kDrainBatch
// entries per round, the point loads of a round issued together.
constexpr int kDrainBatch = 4;

template <class Src>
__device__ __forceinline__ void score32_drain(const double* __restrict__ CE, const Src& src, int b, int p0, int T,
                                              int R, const ScoreConsts& kc, int lane, int32_t (*cnt)[2],
                                              const uint32_t* q, int qn) {
#pragma unroll 1
  for (int i0 = 0; i0 < qn; i0 += 64 * kDrainBatch) {
    uint32_t e[kDrainBatch];
    double4 v[kDrainBatch];
#pragma unroll
    for (int j = 0; j < kDrainBatch; ++j) {
      const int i = i0 + 64 * j + lane;
      e[j] = i < qn ? q[i] : 0xffffffffu;
      v[j] = src.load(b, p0 + (e[j] != 0xffffffffu ? (int)(e[j] & 0xffffffu) : 0));
    }
#pragma unroll
    for (int j = 0; j < kDrainBatch; ++j) {
      if (e[j] == 0xffffffffu) continue;
      const int c = (int)(e[j] >> 24), p = p0 + (int)(e[j] & 0xffffffu);
      if (inlier_f64v(CE + (size_t)c * kCandStride, v[j], kc)) {
        if (p < T) atomicAdd(&cnt[c][0], 1);
        if (p < R) atomicAdd(&cnt[c][1], 1);
      }
    }
  }
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Work unit: one wave scores one (pair, 32-candidate tile, kPtsPerWave-point
// span) item on its own -- its own LDS copy of the tile's records, counts and
// queue, no block barrier -- so a wave that drains a long queue never holds up
// the other waves of its block.  The queue collects the whole item's
// undecided evaluations (drained at the item's end, or earlier when past its
// low mark), so drains run in full 64-lane rounds.
constexpr int kPtsPerWave = kPPL32 * 64 * 4;

template <class Src>
__global__ __launch_bounds__(kScoreThreads) __attribute__((amdgpu_waves_per_eu(4, 4)))
void k_score32(const Src src, PairParams pp, int batch, int cmax, const int32_t* __restrict__ cand_total,
               const double* __restrict__ candE, int32_t* __restrict__ cntT, int32_t* __restrict__ cntR,
               ScoreConsts kc) {
  constexpr int kWaves = kScoreThreads / 64;
  __shared__ int32_t s_cnt[kWaves][kKC][2];
  __shared__ int32_t s_items[SFM_MAX_BATCH + 1];   // items per pair; [batch] = total
  __shared__ int32_t s_first[SFM_MAX_BATCH + 1];   // pair-major order: first item of each pair
  __shared__ int32_t s_tiles[SFM_MAX_BATCH];
  __shared__ double2 s_cand[kWaves][kKC * kCandStride / 2];
  __shared__ uint32_t s_queue[kWaves][kQueue];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) {
    int most = 0, acc = 0;
    for (int b = 0; b < batch; ++b) {
      const int tiles = (cand_total[b] + kKC - 1) / kKC;
      const int splits = (max(pp.test[b], pp.rtest[b]) + kPtsPerWave - 1) / kPtsPerWave;
      s_tiles[b] = tiles;
      s_items[b] = tiles * splits;
      s_first[b] = acc;
      acc += tiles * splits;
      most = max(most, tiles * splits);
    }
    s_first[batch] = acc;
    s_items[batch] = kc.interleave ? most * batch : acc;
  }
  for (int i = tid; i < kWaves * kKC * 2; i += kScoreThreads) (&s_cnt[0][0][0])[i] = 0;
  __syncthreads();
  int32_t(*cnt)[2] = s_cnt[wv];
  uint32_t* queue = s_queue[wv];
  const double* CE = reinterpret_cast<const double*>(s_cand[wv]);
  const int total = __builtin_amdgcn_readfirstlane(s_items[batch]);
  const int gw = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wv);
  // Items run split-major within a pair (every candidate of a pair advances
  // through its points together), pairs one after another, or interleaved
  // (item % batch, tuning key score_interleave).
  unsigned long long skipped = 0;                               // evaluations pruned by this wave
  for (int item = gw; item < total; item += gridDim.x * kWaves) {
    int b, local;
    if (kc.interleave) {
      b = __builtin_amdgcn_readfirstlane(item % batch);
      local = item / batch;
      if (local >= __builtin_amdgcn_readfirstlane(s_items[b])) continue;   // ragged batch: this pair is done
    } else {
      b = 0;
      while (item >= s_first[b + 1]) ++b;
      b = __builtin_amdgcn_readfirstlane(b);                    // wave-uniform (LDS-derived)
      local = item - __builtin_amdgcn_readfirstlane(s_first[b]);
    }
    const int tiles = __builtin_amdgcn_readfirstlane(s_tiles[b]);
    const int split = local / tiles, tile = local - split * tiles;
    const int ctot = cand_total[b];
    const int c0 = tile * kKC;
    const int nc = min(kKC, ctot - c0);
    const int T = pp.test[b], R = pp.rtest[b];
    const int M = max(T, R);
    const int p0 = split * kPtsPerWave;
    const int p1 = min(M, p0 + kPtsPerWave);
    {
      // this wave's copy of the tile's candidate records (nc x 144 B)
      const double2* srcc = reinterpret_cast<const double2*>(candE + ((size_t)b * cmax + c0) * kCandStride);
      for (int i = lane; i < nc * (kCandStride / 2); i += 64) s_cand[wv][i] = srcc[i];
    }
    wave_sync();
    // candidates whose bound count + (T - covered) is below the pair's best
    // count so far: flagged in this wave's LDS record (score32_pass skips them)
    bool all_pruned = false;
    int lb = 0;
    if (kc.prune) {
      const PruneState st = prune_state(cntR, kc.ws_batch, cmax);
      lb = __hip_atomic_load(st.best_lb + (size_t)b * kBestStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bool pr = false;
      if (lane < nc) {
        const unsigned long long v = __hip_atomic_load(st.cov + (size_t)b * cmax + c0 + lane, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        pr = (long long)(uint32_t)v + (long long)T - (long long)(v >> 32) < (long long)lb;
        if (pr) reinterpret_cast<float*>(s_cand[wv])[(lane * kCandStride + 10) * 2 + 13] = __uint_as_float(kPrunedFlag);
      }
      all_pruned = __ballot(pr) == lane_prefix(nc);
      wave_sync();
    }
    int qn = 0;
    for (int cb = all_pruned ? p1 : p0; cb < p1; cb += 64 * kPPL32) {
      int c = 0;
      for (;;) {
        // (re)load the chunk: the points are dead while the queue drains
        float x[kPPL32], y[kPPL32], xp[kPPL32], yp[kPPL32];
        double Mx = 1.0;
        const int pl = cb + lane;
#pragma unroll
        for (int k = 0; k < kPPL32; ++k) {
          const double4 v = src.load(b, min(pl + 64 * k, p1 - 1));
          Mx = fmax(Mx, fmax(fmax(fabs(v.x), fabs(v.y)), fmax(fabs(v.z), fabs(v.w))));
          x[k] = (float)v.x; y[k] = (float)v.y; xp[k] = (float)v.z; yp[k] = (float)v.w;
        }
        // lanes with a coordinate beyond 2^12 (or NaN) take the float64 test for all their points
        const bool lane_bad = !(Mx <= 0x1p12);
        const uint64_t bad = __ballot(lane_bad);
        const bool unit = __ballot(Mx != 1.0) == 0;                  // every lane M = 1, none bad
        const float Mf = lane_bad ? 1.0f : (float)Mx;
        const float M2 = Mf * Mf;
        const int nT = min(p1, T) - cb, nR = min(p1, R) - cb;
        if (min(nT, nR) >= 64 * kPPL32) {                           // no prefix masking needed
          if (unit) c = score32_pass<true, false, false>(CE, c, nc, pl - p0, nT, nR, x, y, xp, yp, M2, bad, kc, lane, cnt, queue, qn);
          else c = score32_pass<true, false, true>(CE, c, nc, pl - p0, nT, nR, x, y, xp, yp, M2, bad, kc, lane, cnt, queue, qn);
        } else if (T == R) {
          c = score32_pass<true, true, true>(CE, c, nc, pl - p0, nT, nR, x, y, xp, yp, M2, bad, kc, lane, cnt, queue, qn);
        } else {
          c = score32_pass<false, true, true>(CE, c, nc, pl - p0, nT, nR, x, y, xp, yp, M2, bad, kc, lane, cnt, queue, qn);
        }
        c = __builtin_amdgcn_readfirstlane(c);
        if (c >= nc) break;
        wave_sync();                                      // queue past its low mark: drain, resume at c
        score32_drain(CE, src, b, p0, T, R, kc, lane, cnt, queue, qn);
        qn = 0;
        wave_sync();
      }
    }
    wave_sync();
    score32_drain(CE, src, b, p0, T, R, kc, lane, cnt, queue, qn);
    wave_sync();
    if (kc.prune) {
      // publish (count, covered) of the span; raise the pair's best count so far
      const PruneState st = prune_state(cntR, kc.ws_batch, cmax);
      int reached = 0, skip = 0;
      if (lane < nc) {
        const float* F = reinterpret_cast<const float*>(CE + (size_t)lane * kCandStride + 10);
        if (__float_as_uint(F[13]) == kPrunedFlag) {
          skip = p1 - p0;
        } else {
          const int sc = cnt[lane][0];
          const unsigned long long old = atomicAdd(st.cov + (size_t)b * cmax + c0 + lane,
                                                   ((unsigned long long)(p1 - p0) << 32) | (unsigned)sc);
          reached = (int)(uint32_t)old + sc;
        }
      }
#pragma unroll
      for (int d = 32; d >= 1; d >>= 1) {
        reached = max(reached, __shfl_xor(reached, d, 64));
        skip += __shfl_xor(skip, d, 64);
      }
      // only raise the shared bound when this item beat the value it read:
      // one hot line per pair, updated by few items
      if (lane == 0 && reached > lb) atomicMax(st.best_lb + (size_t)b * kBestStride, reached);
      skipped += (unsigned long long)skip;
    }
    {
      const int c = lane >> 1, which = lane & 1;
      if (c < nc) {
        const int s = cnt[c][which];
        cnt[c][which] = 0;
        if (s) atomicAdd((which ? cntR : cntT) + (size_t)b * cmax + c0 + c, s);
      }
    }
    wave_sync();
  }
  if (kc.prune && lane == 0 && skipped) atomicAdd(prune_state(cntR, kc.ws_batch, cmax).skipped, skipped);
}

// ---------------------------------------------------------------------------
// Phase 4: selection (one block per pair)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_select(int H, int cmax, int cheir,
                                                 const int32_t* __restrict__ ncand,
                                                 const int32_t* __restrict__ cand_off,
                                                 const int32_t* __restrict__ cntT,
                                                 const int32_t* __restrict__ cntR,
                                                 const double* __restrict__ candE,
                                                 const double* __restrict__ hypP,
                                                 const double* __restrict__ hypP0,
                                                 int32_t* __restrict__ score_out,
                                                 double* __restrict__ E_out, double* __restrict__ P_out,
                                                 int32_t* __restrict__ inliers_out, int32_t* __restrict__ winner_out) {
  __shared__ unsigned long long s_best[16];
  const int b = blockIdx.x, tid = threadIdx.x;
  const size_t hb0 = (size_t)b * H;
  const int32_t* cT = cntT + (size_t)b * cmax;
  const int32_t* cR = cntR + (size_t)b * cmax;
  unsigned long long best = 0ull;
  for (int h = tid; h < H; h += blockDim.x) {
    const int nc = ncand[hb0 + h], off = cand_off[hb0 + h];
    int bi = 0, bc = 0;
    for (int j = 0; j < nc; ++j) {
      const int c = cT[off + j];
      if (c > bc) { bc = c; bi = j; }
    }
    const int s = cR[off + bi];
    score_out[hb0 + h] = s;
    const unsigned long long key = ((unsigned long long)(uint32_t)s << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)h);
    best = key > best ? key : best;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(best, d, 64);
    best = o > best ? o : best;
  }
  if ((tid & 63) == 0) s_best[tid >> 6] = best;
  __syncthreads();
  if (tid != 0) return;
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) best = s_best[w] > best ? s_best[w] : best;
  const int s = (int)(best >> 32);
  double* Eo = E_out + (size_t)b * 9;
  double* Po = P_out ? P_out + (size_t)b * 12 : nullptr;
  if (s <= 0) {
    for (int e = 0; e < 9; ++e) Eo[e] = 0.0;
    if (Po) for (int e = 0; e < 12; ++e) Po[e] = 0.0;
    inliers_out[b] = 0;
    if (winner_out) winner_out[b] = -1;
    return;
  }
  const int h = (int)(0xFFFFFFFFu - (uint32_t)(best & 0xFFFFFFFFull));
  const int nc = ncand[hb0 + h], off = cand_off[hb0 + h];
  int bi = 0, bc = 0;
  for (int j = 0; j < nc; ++j) {
    const int c = cT[off + j];
    if (c > bc) { bc = c; bi = j; }
  }
  const double* Ew = candE + ((size_t)b * cmax + off + bi) * kCandStride;
  for (int e = 0; e < 9; ++e) Eo[e] = Ew[e];
  if (Po) {
    const double* Pw = nc > 0 ? hypP + ((hb0 + h) * kMaxSlots + bi) * 12 : hypP0 + (hb0 + h) * 12;
    for (int e = 0; e < 12; ++e) Po[e] = cheir ? Pw[e] : 0.0;
  }
  inliers_out[b] = s;
  if (winner_out) winner_out[b] = h;
}

// ---------------------------------------------------------------------------
// Auxiliary kernels
// ---------------------------------------------------------------------------
__global__ void k_inlier_mask(const double* __restrict__ pts, int64_t n_stride, PairParams pp,
                              const double* __restrict__ E, double thr, uint8_t* __restrict__ mask) {
  const int b = blockIdx.y;
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_stride) return;
  uint8_t m = 0;
  if (k < pp.n[b]) {
    const double4 v = *reinterpret_cast<const double4*>(pts + ((size_t)b * n_stride + k) * 4);
    m = inlier_reference(E + (size_t)b * 9, v.x, v.y, v.z, v.w, thr) ? 1 : 0;
  }
  mask[(size_t)b * n_stride + k] = m;
}

__global__ void k_pack(const double* __restrict__ q, const double* __restrict__ qp, int64_t n, double* __restrict__ out) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double2 a = reinterpret_cast<const double2*>(q)[k];
  const double2 c = reinterpret_cast<const double2*>(qp)[k];
  reinterpret_cast<double4*>(out)[k] = make_double4(a.x, a.y, c.x, c.y);
}

// flow2coord + margin crop + K^-1 (models/SFMnet.py:179-263, 298-318): the
// FlowSrc values, materialised
__global__ void k_flow_points(const FlowSrc src, int64_t N, double* __restrict__ out) {
  const int b = blockIdx.y;
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= N) return;
  reinterpret_cast<double4*>(out)[(size_t)b * N + k] = src.load(b, k);
}

// Sparse correspondences of SFMnet.pose_by_ransac (models/SFMnet.py:218-258):
//   mode 0 (default): flow at the rounded keypoints of the reference image,
//          pts1 = np.int32(np.round(kp))  ->  coord[:, y, x]           (250-253)
//   mode 1 (cfg.SAMPLE_SP): grid_sample of the coordinate grids at the
//          keypoints, align_corners=True, zeros padding             (242-247)
//   mode 2 (cfg.SIFT_POSE): the matched keypoints themselves        (218-224)
// followed by K^-1 (bmm, 3 rows) in float32 and the f64 widening of
// compute_P_matrix_ransac.  Rows >= n[b] of the output are not written.
struct KpCounts {
  int n[SFM_MAX_BATCH];
};

__device__ __forceinline__ float kp_tap(float v, bool ok) { return ok ? v : 0.0f; }

__global__ void k_keypoint_points(const float* __restrict__ flow, int H, int W, int h_side, int w_side,
                                  const float* __restrict__ kp1, const float* __restrict__ kp2, int64_t kp_stride,
                                  KpCounts cnt, int mode, const float* __restrict__ Kinv, double* __restrict__ out,
                                  int64_t n_stride) {
  const int b = blockIdx.y;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt.n[b]) return;
  const float* Ki = Kinv + b * 9;
  const float* F = flow + (size_t)b * 2 * H * W;
  const float kx = kp1[((size_t)b * kp_stride + k) * 2], ky = kp1[((size_t)b * kp_stride + k) * 2 + 1];
  float c1[3], c2[3];
  if (mode == 2) {
    c1[0] = kx; c1[1] = ky; c1[2] = 1.0f;
    c2[0] = kp2[((size_t)b * kp_stride + k) * 2]; c2[1] = kp2[((size_t)b * kp_stride + k) * 2 + 1]; c2[2] = 1.0f;
  } else if (mode == 0) {
    // round half to even (np.round); the caller validates the range (the
    // reference's indexing raises), the clamp only keeps the access in bounds
    const int x = min(max((int)rintf(kx), 0), w_side - 1);
    const int y = min(max((int)rintf(ky), 0), h_side - 1);
    const float fu = F[(size_t)y * W + x], fv = F[(size_t)H * W + (size_t)y * W + x];
    c1[0] = (float)x; c1[1] = (float)y; c1[2] = 1.0f;
    c2[0] = c1[0] + fu; c2[1] = c1[1] + fv; c2[2] = 1.0f;
  } else {
    // pts normalised in float32 as SFMnet.py:245, then grid_sample's
    // align_corners=True unnormalisation and zero-padded bilinear taps
    const float xn = 2.0f * kx / (float)max(w_side - 1, 1) - 1.0f;
    const float yn = 2.0f * ky / (float)max(h_side - 1, 1) - 1.0f;
    const float ix = ((xn + 1.0f) / 2.0f) * (float)(w_side - 1);
    const float iy = ((yn + 1.0f) / 2.0f) * (float)(h_side - 1);
    const float fx = floorf(ix), fy = floorf(iy);
    const int x0 = (int)fx, y0 = (int)fy, x1 = x0 + 1, y1 = y0 + 1;
    const float wnw = ((fx + 1.0f) - ix) * ((fy + 1.0f) - iy);
    const float wne = (ix - fx) * ((fy + 1.0f) - iy);
    const float wsw = ((fx + 1.0f) - ix) * (iy - fy);
    const float wse = (ix - fx) * (iy - fy);
    const int xs[4] = {x0, x1, x0, x1}, ys[4] = {y0, y0, y1, y1};
    const float wt[4] = {wnw, wne, wsw, wse};
    float a1[3] = {0.0f, 0.0f, 0.0f}, a2[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bool ok = xs[t] >= 0 && xs[t] < w_side && ys[t] >= 0 && ys[t] < h_side;
      const int xc = min(max(xs[t], 0), w_side - 1), yc = min(max(ys[t], 0), h_side - 1);
      const float gx = (float)xc, gy = (float)yc;
      const float fu = F[(size_t)yc * W + xc], fv = F[(size_t)H * W + (size_t)yc * W + xc];
      a1[0] = a1[0] + kp_tap(gx, ok) * wt[t];
      a1[1] = a1[1] + kp_tap(gy, ok) * wt[t];
      a1[2] = a1[2] + kp_tap(1.0f, ok) * wt[t];
      a2[0] = a2[0] + kp_tap(gx + fu, ok) * wt[t];
      a2[1] = a2[1] + kp_tap(gy + fv, ok) * wt[t];
      a2[2] = a2[2] + kp_tap(1.0f, ok) * wt[t];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) { c1[j] = a1[j]; c2[j] = a2[j]; }
  }
  const float x1n = (Ki[0] * c1[0] + Ki[1] * c1[1]) + Ki[2] * c1[2];
  const float y1n = (Ki[3] * c1[0] + Ki[4] * c1[1]) + Ki[5] * c1[2];
  const float x2n = (Ki[0] * c2[0] + Ki[1] * c2[1]) + Ki[2] * c2[2];
  const float y2n = (Ki[3] * c2[0] + Ki[4] * c2[1]) + Ki[5] * c2[2];
  reinterpret_cast<double4*>(out)[(size_t)b * n_stride + k] = make_double4(x1n, y1n, x2n, y2n);
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
#include "score_mf.h"
#include "score_mf2.h"

// The score-kernel choice (shared by the RANSAC driver and
// sfm_score_essentials): the split-f16 matrix-core scorers when the threshold
// and precision allow, else the float32 / float64 VALU scorers.
struct ScoreBufs {
  int32_t* cand_total;
  double* candE;
  _Float16* candF;
  int32_t* cntT;
  int32_t* cntR;
  unsigned long long* claim;   // [9] k_score_mf2's range-claim counters and finished-block count
  int32_t* cmap2 = nullptr;    // the one-sided pruning's second keep (k_mf2_keep_map)
  int32_t* cmap = nullptr;     // count-bound pruning (k_mf2_lead / _keep): kept candidates, the
  int32_t* lead = nullptr;     // leader records (their [3] = kept candidates), the evaluations skipped,
  unsigned long long* skipped = nullptr;
  int32_t* bnd = nullptr;      // the launches' span boundaries per pair (k_mf2_split)
};

// score_precision with the low-precision form folded in: 64, 32 / 16 (held in
// T), 33 / 17 (the literal template form, score_lowp_template)
static int lowp_prec() {
  const int p = tuning().score_precision;
  return (p != 64 && tuning().score_lowp_template) ? p + 1 : p;
}

template <class Src>
static void score_dispatch(const Src& src, const PairParams& pp, int bc, int cmax, const ScoreBufs& w,
                           const ScoreConsts& kc, const MfParams& mp, bool use_mf, bool same, int prec, bool fast,
                           bool fast32, int cus, int grid, hipStream_t s, int prune_pm = 0) {
  if (use_mf) {
    hipLaunchKernelGGL(k_mf_cands, dim3((cmax + 255) / 256, bc), dim3(256), 0, s, cmax, w.cand_total, w.candE,
                       w.candF, mp, w.claim, prune_pm > 0 ? w.lead : nullptr);
    const dim3 gmf(std::max(1, cus) * tuning().score_mf_blocks_per_cu);
    const dim3 g2(std::max(1, cus)), b2(kMf2Waves * 64), b2u(mf2_waves<true>() * 64);
    if (same && tuning().score_mf == 2 && prune_pm > 0) {
      // count-bound pruning: A every candidate on the first prune_pm per mille
      // of each pair's spans; k_mf2_split picks the pair's pruning point sB
      // from its inlier ratio; B every candidate up to sB; k_mf2_lead +
      // k_mf2_keep; C the kept candidates on the rest
      const int ch = tuning().score_mf_chunk;
      const int ch2 = tuning().score_mf_chunk2 ? tuning().score_mf_chunk2 : ch;
      if (tuning().score_mf_prune_upper) {
        // the one-sided pruning (round 6), counts = points not certainly
        // outliers (upper bounds):
        //   A every candidate one-sided on the first prune_pm per mille of the
        //     spans; k_mf2_split the pair's pruning point sB (round 5's rule)
        //     and the leader (the first max); B every candidate up to sB;
        //   k_mf2_lead the leader's exact count over every point (lb);
        //   k_mf2_keep the candidates whose upper bound (count + points left)
        //     reaches lb; A2 those one-sided on the rest; k_mf2_keep_map those
        //     whose full upper count still reaches lb;
        //   their counts zeroed, then counted exactly: float64 (k_mf2_exact)
        //   for pairs with at most score_mf_exact_max of them, the two-sided
        //   matrix-core pass through the index map for the others (lead row 4)
        hipLaunchKernelGGL((k_score_mf2<Src, false, true>), g2, b2u, 0, s, src, pp, bc, cmax, w.cand_total, w.candE,
                           w.candF, w.cntT, kc, w.claim, (const int32_t*)nullptr, 0, prune_pm,
                           (const int32_t*)nullptr, 0, ch);
        hipLaunchKernelGGL(k_mf2_split, dim3(bc), dim3(1024), 0, s, pp, cmax, prune_pm,
                           tuning().score_mf_prune_margin, w.cand_total, w.cntT, w.bnd, w.lead);
        hipLaunchKernelGGL((k_score_mf2<Src, false, true>), g2, b2u, 0, s, src, pp, bc, cmax, w.cand_total, w.candE,
                           w.candF, w.cntT, kc, w.claim, (const int32_t*)nullptr, 0, 0, (const int32_t*)w.bnd, 1, ch);
        hipLaunchKernelGGL(k_mf2_lead<Src>, dim3(4 * kLeadBlocks, bc), dim3(1024), 0, s, src, pp, cmax,
                           (const int32_t*)w.bnd, w.cand_total, w.candE, w.cntT, kc, w.lead, 2);
        hipLaunchKernelGGL(k_mf2_keep, dim3((cmax + 1023) / 1024, bc), dim3(1024), 0, s, pp, cmax,
                           (const int32_t*)w.bnd, w.cand_total, w.cntT, w.lead, w.cmap, w.skipped, 0);
        hipLaunchKernelGGL((k_score_mf2<Src, true, true>), g2, b2u, 0, s, src, pp, bc, cmax,
                           w.lead + 3 * SFM_MAX_BATCH, w.candE, w.candF, w.cntT, kc, w.claim, (const int32_t*)w.cmap,
                           0, 0, (const int32_t*)w.bnd, 2, ch2);
        hipLaunchKernelGGL(k_mf2_keep_map, dim3(bc), dim3(1024), 0, s, cmax, (const int32_t*)w.cntT, w.lead,
                           (const int32_t*)w.cmap, w.cmap2, tuning().score_mf_exact_max);
        hipLaunchKernelGGL(k_mf2_zero_kept, dim3((cmax + 255) / 256, bc), dim3(256), 0, s, cmax,
                           (const int32_t*)w.lead, (const int32_t*)w.cmap2, w.cntT);
        hipLaunchKernelGGL(k_mf2_exact<Src>, dim3(kExactBlocks, bc), dim3(kExactThreads), 0, s, src, pp, cmax,
                           (const int32_t*)w.lead, (const int32_t*)w.cmap2, w.candE, kc, w.cntT,
                           tuning().score_mf_exact_max);
        hipLaunchKernelGGL((k_score_mf2<Src, true>), g2, b2, 0, s, src, pp, bc, cmax, w.lead + 4 * SFM_MAX_BATCH,
                           w.candE, w.candF, w.cntT, kc, w.claim, (const int32_t*)w.cmap2, 0, 1000,
                           (const int32_t*)nullptr, 0, ch2);
      } else {
        hipLaunchKernelGGL((k_score_mf2<Src, false>), g2, b2, 0, s, src, pp, bc, cmax, w.cand_total, w.candE, w.candF,
                           w.cntT, kc, w.claim, (const int32_t*)nullptr, 0, prune_pm, (const int32_t*)nullptr, 0, ch);
        hipLaunchKernelGGL(k_mf2_split, dim3(bc), dim3(1024), 0, s, pp, cmax, prune_pm,
                           tuning().score_mf_prune_margin, w.cand_total, w.cntT, w.bnd, (int32_t*)nullptr);
        hipLaunchKernelGGL((k_score_mf2<Src, false>), g2, b2, 0, s, src, pp, bc, cmax, w.cand_total, w.candE, w.candF,
                           w.cntT, kc, w.claim, (const int32_t*)nullptr, 0, 0, (const int32_t*)w.bnd, 1, ch);
        hipLaunchKernelGGL(k_mf2_lead<Src>, dim3(kLeadBlocks, bc), dim3(1024), 0, s, src, pp, cmax,
                           (const int32_t*)w.bnd, w.cand_total, w.candE, w.cntT, kc, w.lead, 0);
        hipLaunchKernelGGL(k_mf2_keep, dim3((cmax + 1023) / 1024, bc), dim3(1024), 0, s, pp, cmax,
                           (const int32_t*)w.bnd, w.cand_total, w.cntT, w.lead, w.cmap, w.skipped, 0);
        hipLaunchKernelGGL((k_score_mf2<Src, true>), g2, b2, 0, s, src, pp, bc, cmax, w.lead + 3 * SFM_MAX_BATCH,
                           w.candE, w.candF, w.cntT, kc, w.claim, (const int32_t*)w.cmap, 0, 0, (const int32_t*)w.bnd,
                           2, ch2);
      }
      set_last_scorer("k_score_mf2+prune");
    } else if (same && tuning().score_mf == 2) {
      hipLaunchKernelGGL((k_score_mf2<Src, false>), g2, b2, 0, s, src, pp, bc, cmax, w.cand_total, w.candE, w.candF, w.cntT,
                         kc, w.claim, (const int32_t*)nullptr, 0, 1000, (const int32_t*)nullptr, 0,
                         tuning().score_mf_chunk);
      set_last_scorer("k_score_mf2");
    } else if (same) {
      hipLaunchKernelGGL((k_score_mf<Src, true>), gmf, dim3(kMfWaves * 64), 0, s, src, pp, bc, cmax,
                         w.cand_total, w.candE, w.candF, w.cntT, w.cntR, kc);
      set_last_scorer("k_score_mf");
    } else {
      hipLaunchKernelGGL((k_score_mf<Src, false>), gmf, dim3(kMfWaves * 64), 0, s, src, pp, bc, cmax,
                         w.cand_total, w.candE, w.candF, w.cntT, w.cntR, kc);
      set_last_scorer("k_score_mf");
    }
  } else if (prec == 32) {
    hipLaunchKernelGGL((k_score<false, Src, 32>), dim3(grid), dim3(kScoreThreads), 0, s, src, pp, bc, cmax,
                       w.cand_total, w.candE, w.cntT, w.cntR, kc);
    set_last_scorer("k_score<32>");
  } else if (prec == 16) {
    hipLaunchKernelGGL((k_score<false, Src, 16>), dim3(grid), dim3(kScoreThreads), 0, s, src, pp, bc, cmax,
                       w.cand_total, w.candE, w.cntT, w.cntR, kc);
    set_last_scorer("k_score<16>");
  } else if (prec == 33) {
    hipLaunchKernelGGL((k_score<false, Src, 33>), dim3(grid), dim3(kScoreThreads), 0, s, src, pp, bc, cmax,
                       w.cand_total, w.candE, w.cntT, w.cntR, kc);
    set_last_scorer("k_score<33>");
  } else if (prec == 17) {
    hipLaunchKernelGGL((k_score<false, Src, 17>), dim3(grid), dim3(kScoreThreads), 0, s, src, pp, bc, cmax,
                       w.cand_total, w.candE, w.cntT, w.cntR, kc);
    set_last_scorer("k_score<17>");
  } else if (fast32) {
    hipLaunchKernelGGL(k_score32<Src>, dim3(grid), dim3(kScoreThreads), 0, s, src, pp, bc, cmax, w.cand_total,
                       w.candE, w.cntT, w.cntR, kc);
    set_last_scorer(kc.prune ? "k_score32+prune" : "k_score32");
  } else if (fast) {
    hipLaunchKernelGGL((k_score<true, Src>), dim3(grid), dim3(kScoreThreads), 0, s, src, pp, bc, cmax,
                       w.cand_total, w.candE, w.cntT, w.cntR, kc);
    set_last_scorer("k_score<fma>");
  } else {
    hipLaunchKernelGGL((k_score<false, Src>), dim3(grid), dim3(kScoreThreads), 0, s, src, pp, bc, cmax,
                       w.cand_total, w.candE, w.cntT, w.cntR, kc);
    set_last_scorer("k_score<ref>");
  }
}

// Candidate records of given essential matrices (sfm_score_essentials): E,
// the float64 guard constant and the float32 constants, as k_cand writes them.
__global__ __launch_bounds__(256) void k_fill_cands(const double* __restrict__ E, int ncand, int cmax,
                                                    double guard_g, double thr, int fast32,
                                                    double* __restrict__ candE, int32_t* __restrict__ cand_total) {
  const int b = blockIdx.y;
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c == 0) cand_total[b] = ncand;
  if (c >= ncand) return;
  double* dst = candE + ((size_t)b * cmax + c) * kCandStride;
  const double* src = E + ((size_t)b * ncand + c) * 9;
#pragma unroll
  for (int e = 0; e < 9; ++e) dst[e] = src[e];
  dst[9] = guard_constant(dst, guard_g);
  fp32_constants(dst, thr, fast32 != 0, reinterpret_cast<float*>(dst + 10));
}

// k_roots with the split isolation (five_point.h, isolate_p1 / falsi_tasks /
// bisect_deferred): lanes [0, lanes) of each wave own one hypothesis each
// through phase 1; phases 2 and 3 run over a task list on every lane.  NW = 1
// (roots_split 1, the default): one wave per block and its own list, so the
// launch lasts as long as its busiest wave (profiles/r03_roots_split_stats.txt:
// 245 k cycles per wave on average, 313-325 k at most).  NW = 4 (roots_split
// 2, opt-in): the block's four waves append to and claim from one pool (LDS
// counters), so the tail averages over four waves' tasks -- measured 2-6 %
// slower (profiles/r04_roots_pool_ab.txt).  Phase 1 stays per hypothesis, and
// every node's root goes to its fixed slot: the workspace is byte-identical.
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_roots_split(int H, int lanes, double* __restrict__ st, size_t stride,
                                                         int32_t* __restrict__ out_nroots) {
  const int b = blockIdx.y;
  const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
  const int h = (blockIdx.x * NW + wv) * lanes + lane;
  const bool own = lane < lanes && h < H;
  const int owner = wv * kStkLanes + lane;                  // the hypothesis' slot in the pool
  __shared__ double s_lohi[NW][kStkDepth * 2 * kStkLanes];
  __shared__ int s_meta[NW][kStkDepth * kStkLanes];
  __shared__ RootsSharedT<kStkLanes * NW> sh;
  if (lane < kStkLanes) {
#pragma unroll
    for (int i = 0; i < 10; ++i) sh.roots[i][owner] = 0.0;
  }
  if (threadIdx.x == 0) { sh.ntask = 0; sh.ndl = 0; sh.next2 = 0; sh.next3 = 0; }
  __syncthreads();
#ifdef SFM_ROOTS_STATS
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  const size_t hb = (size_t)b * H + h;
  int nr = 0;
  double fac = 1.0;
  if (own) {
    double poly[11];
#pragma unroll
    for (int i = 0; i <= 10; ++i) poly[i] = st_at(st, stride, kStPoly + i, hb);
    double roots[10];
    SturmR R;
    const IsoStack stk{nullptr, nullptr};
    const IsoStackP stkp{s_lohi[wv] + lane, s_meta[wv] + lane};
    nr = real_roots_t<true>(poly, roots, stk, R, &sh, &stkp, owner, &fac);
  }
#ifdef SFM_ROOTS_STATS
  // split stats: cycles at the end of phase 1 / phase 2 in the second half of g_roots_cycles / g_roots_phase[0]
  const size_t si = ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
  if (own) g_roots_cycles[si + (1 << 16)] = __builtin_amdgcn_s_memtime() - t0;
#endif
  __syncthreads();
  falsi_tasks<(NW > 1)>(sh, lane);
  __syncthreads();
#ifdef SFM_ROOTS_STATS
  if (own) g_roots_phase[0][si] = __builtin_amdgcn_s_memtime() - t0;
#endif
  bisect_deferred<(NW > 1)>(sh, lane);
  __syncthreads();
  if (own) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      double r = sh.roots[i][owner];
      if (i < nr) r /= fac;
      st_at(st, stride, kStRoots + i, hb) = r;
    }
    out_nroots[hb] = nr;
  }
#ifdef SFM_ROOTS_STATS
  if (own) g_roots_cycles[si] = __builtin_amdgcn_s_memtime() - t0;
#endif
}

// Score fence (sfm_score_fence_enable / _wait): an event recorded on the
// RANSAC stream right before the scoring phase, so that a second stream can
// start pose-independent memory work (the cost volume's reference half) beside
// the compute-bound scorer instead of beside the latency-bound solve.  One
// event per device, created on that device (the device of the stream it is
// recorded on / waited from, never the caller's current device); recording is
// on while any enable(1) is not matched by an enable(0).
constexpr int kFenceDevices = 64;
static std::mutex g_fence_mu;
static hipEvent_t g_fence[kFenceDevices] = {};
static int g_fence_refs = 0;

static int stream_device(hipStream_t s, int* dev) {
  if (hipStreamGetDevice(s, dev) != hipSuccess) SFM_HIP(hipGetDevice(dev));
  SFM_REQUIRE(*dev >= 0 && *dev < kFenceDevices, "score fence: device index out of range");
  return SFM_OK;
}

// the fence of the stream's device (created there on first use); g_fence_mu held
static int fence_of(hipStream_t s, hipEvent_t* ev) {
  int dev = 0;
  if (int rc = stream_device(s, &dev)) return rc;
  if (!g_fence[dev]) {
    int cur = 0;
    SFM_HIP(hipGetDevice(&cur));
    SFM_HIP(hipSetDevice(dev));
    const hipError_t e = hipEventCreateWithFlags(&g_fence[dev], hipEventDisableTiming);
    SFM_HIP(hipSetDevice(cur));
    SFM_HIP(e);
  }
  *ev = g_fence[dev];
  return SFM_OK;
}

static int record_score_fence(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_fence_mu);
  if (g_fence_refs <= 0) return SFM_OK;
  hipEvent_t ev = nullptr;
  if (int rc = fence_of(s, &ev)) return rc;
  SFM_HIP(hipEventRecord(ev, s));
  return SFM_OK;
}

// Score gate (sfm_score_gate): a library-owned event per (device, waiting
// stream), recorded on the caller's (side) stream; the next RANSAC call issued
// on that waiting stream waits for it right before its scoring phase
// (one-shot), so that a pipelined caller can run the previous step's
// HBM-bound sweep beside this step's latency-bound solve while keeping the
// compute-bound scorer to itself.  RANSAC calls on any other stream -- another
// hot path on the same device, a plain computeP -- neither wait for nor
// consume it.
constexpr int kGates = 32;
struct ScoreGate {
  int dev = -1;                  // -1: free slot
  hipStream_t waiter = nullptr;  // the stream whose next scoring phase waits
  hipEvent_t ev = nullptr;       // kept when the slot is freed (reused on evdev)
  int evdev = -1;                // the device ev was created on
  bool armed = false;
};
static ScoreGate g_gates[kGates];

static int wait_score_gate(hipStream_t s) {
  std::lock_guard<std::mutex> lk(g_fence_mu);
  int dev = 0;
  if (int rc = stream_device(s, &dev)) return rc;
  for (ScoreGate& g : g_gates)
    if (g.armed && g.dev == dev && g.waiter == s) {
      g.armed = false;
      g.dev = -1;
      SFM_HIP(hipStreamWaitEvent(s, g.ev, 0));
    }
  return SFM_OK;
}

template <class Src>
static int run_chunk(const Src& src, const int64_t* n, int bc, int num_test,
                     int num_ransac_test, int iters, double thr, uint64_t seed, int cheir,
                     const Workspace& w, int ws_batch, double* E_out, double* P_out, int32_t* inliers_out,
                     int32_t* winner_out, int32_t* score_out, hipStream_t s, bool first_chunk) {
  const int H = kChains * iters;
  const int cmax = H * kMaxSlots;
  PairParams pp{};
  for (int b = 0; b < bc; ++b) {
    pp.n[b] = n[b];
    pp.test[b] = (int32_t)(num_test > 0 ? num_test : n[b]);
    pp.rtest[b] = (int32_t)(num_ransac_test > 0 ? num_ransac_test : n[b]);
    const int M = std::max(pp.test[b], pp.rtest[b]);
    pp.splits[b] = (M + kPtsPerItem - 1) / kPtsPerItem;
  }
  {
    ProfScope ps("ransac_solve", s);
    // lane counts bounded by the kernels' per-lane LDS records (the key validators enforce it too)
    const int lanes = std::min(tuning().solve_lanes, kFrontLanes);
    const int rlanes = std::min(tuning().roots_lanes, kStkLanes);
    const size_t stride = (size_t)bc * H;
    if (tuning().solve_coop)
      hipLaunchKernelGGL((k_solve_front<Src, true>), dim3((H + lanes - 1) / lanes, bc), dim3(64), 0, s, src, pp, H,
                         seed, lanes, w.sstate, stride);
    else
      hipLaunchKernelGGL((k_solve_front<Src, false>), dim3((H + lanes - 1) / lanes, bc), dim3(64), 0, s, src, pp, H,
                         seed, lanes, w.sstate, stride);
    if (tuning().roots_split == 2)
      hipLaunchKernelGGL(k_roots_split<4>, dim3((H + 4 * rlanes - 1) / (4 * rlanes), bc), dim3(256), 0, s, H, rlanes,
                         w.sstate, stride, w.nroots);
    else if (tuning().roots_split)
      hipLaunchKernelGGL(k_roots_split<1>, dim3((H + rlanes - 1) / rlanes, bc), dim3(64), 0, s, H, rlanes, w.sstate,
                         stride, w.nroots);
    else
      hipLaunchKernelGGL(k_roots, dim3((H + rlanes - 1) / rlanes, bc), dim3(64), 0, s, H, rlanes, w.sstate, stride,
                         w.nroots);
    if (tuning().solve_coop)
      hipLaunchKernelGGL(k_solve_back<true>, dim3((H + 15) / 16, bc), dim3(64), 0, s, H, cheir, w.sstate, stride,
                         w.nroots, w.ncand, w.hypE, w.hypP);
    else
      hipLaunchKernelGGL(k_solve_back<false>, dim3((H + 63) / 64, bc), dim3(64), 0, s, H, cheir, w.sstate, stride,
                         w.nroots, w.ncand, w.hypE, w.hypP);
  }
  SFM_LAUNCHED();
  const int prec = lowp_prec();
  // reduced precision: no exactness guards; the plain ComputeError<T> kernel
  const bool fast = prec == 64 && thr >= 0x1p-40 && thr < 1.0;
  const double guard_g = fast ? 0x1p24 * (11.0 + 11.0 / thr) : 0.0;
  const bool fast32 = fast && thr >= 0x1p-20 && tuning().score_fp32;
  {
    ProfScope ps("ransac_chain", s);
    hipLaunchKernelGGL(k_chain, dim3(bc), dim3(kChains), 0, s, H, iters, w.nroots, w.ncand, w.cand_off, w.chain_ref,
                       w.cand_total, first_chunk ? w.skipped : nullptr);
    hipLaunchKernelGGL(k_cand, dim3((H * kMaxSlots + 255) / 256, bc), dim3(256), 0, s, H, iters, cheir, w.chain_ref,
                       w.ncand, w.hypE, w.hypP, w.hypP0, w.cand_off, w.candE, cmax, guard_g, thr, fast32 ? 1 : 0,
                       w.cntT, w.cntR);
  }
  SFM_LAUNCHED();
  ScoreConsts kc;
  kc.thr = thr;
  kc.t2lo = (thr * thr) * (1.0 - 0x1p-22);
  kc.t2hi = (thr * thr) * (1.0 + 0x1p-22);
  // float32 thresholds with directed slack (see fp32_constants)
  kc.t2lo32 = (float)((thr * thr) * (1.0 - 0x1p-6 - 0x1p-19));
  kc.t2hi32 = (float)((thr * thr) * (1.0 + 0x1p-7) / (1.0 - 0x1p-7) * (1.0 + 0x1p-19));
  kc.fast32 = fast32 ? 1 : 0;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = std::max(1, cus) * tuning().score_blocks_per_cu;
  // exact bound pruning: SFMnet's num_test == num_ransac_test, no per-hypothesis scores requested
  bool same = true;
  for (int b = 0; b < bc; ++b) same = same && pp.test[b] == pp.rtest[b];
  MfParams mp{};
  const bool use_mf = fast32 && tuning().score_mf && mf_params(thr, &mp);
  kc.prune = (fast32 && !use_mf && same && !score_out && tuning().score_prune) ? 1 : 0;
  // count-bound pruning in k_score_mf2 (k_mf2_lead / _keep): same condition, and
  // every pair long enough that the second launch has spans to skip
  int min_spans = INT32_MAX;
  for (int b = 0; b < bc; ++b) min_spans = std::min(min_spans, mf2_spans(std::max(pp.test[b], pp.rtest[b])));
  const int mf2_pm = (use_mf && same && !score_out && tuning().score_mf == 2 && min_spans >= kMf2PruneMinSpans)
                         ? tuning().score_mf_prune : 0;
  kc.ws_batch = ws_batch;
  kc.interleave = tuning().score_interleave;
  SFM_REQUIRE(prune_state(w.cntR, ws_batch, cmax).skipped == w.skipped, "internal: pruning state layout");
  if (kc.prune) {
    SFM_HIP(hipMemsetAsync(w.cov, 0, (size_t)bc * cmax * 8, s));
    SFM_HIP(hipMemsetAsync(w.best_lb, 0, SFM_MAX_BATCH * kBestStride * 4, s));
  }
  if (int rc = record_score_fence(s)) return rc;
  if (int rc = wait_score_gate(s)) return rc;
  {
    ProfScope ps("ransac_score", s);
    ScoreBufs sb{w.cand_total, w.candE, w.candF, w.cntT, w.cntR, w.claim};
    sb.cmap = w.cmap;
    sb.cmap2 = w.cmap2;
    sb.lead = w.lead;
    sb.bnd = w.bnd;
    sb.skipped = w.skipped;
    score_dispatch(src, pp, bc, cmax, sb, kc, mp, use_mf, same, prec, fast, fast32, cus, grid, s, mf2_pm);
  }
  SFM_LAUNCHED();
  {
    ProfScope ps("ransac_select", s);
    // k_score_mf2 publishes one count array (its runs have num_test == num_ransac_test)
    const bool one_cnt = use_mf && same && tuning().score_mf == 2;
    hipLaunchKernelGGL(k_select, dim3(bc), dim3(1024), 0, s, H, cmax, cheir, w.ncand, w.cand_off, w.cntT,
                       one_cnt ? w.cntT : w.cntR, w.candE, w.hypP, w.hypP0, score_out ? score_out : w.score, E_out, P_out,
                       inliers_out, winner_out);
  }
  SFM_LAUNCHED();
  return SFM_OK;
}

static int check_common(int iters, double thr, int batch) {
  SFM_REQUIRE(batch >= 1, "batch must be >= 1");
  SFM_REQUIRE(iters >= 1 && iters <= 4096, "iters must be in [1, 4096]");
  SFM_REQUIRE(thr > 0.0, "inlier threshold must be > 0");
  return SFM_OK;
}

template <class Src>
static int run_src(const Src& src, const int64_t* n, int batch, int num_test, int num_ransac_test, int iters,
                   double thr, uint64_t seed, int cheir, void* ws, size_t ws_bytes, double* E_out, double* P_out,
                   int32_t* inliers_out, int32_t* winner_out, int32_t* score_out, hipStream_t s) {
  const int bc = std::min(batch, SFM_MAX_BATCH);
  const size_t need = layout(nullptr, bc, 0, iters, nullptr);
  if (!ws || ws_bytes < need) {
    set_error("workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  Workspace w;
  layout((char*)ws, bc, 0, iters, &w);
  const int H = kChains * iters;
  for (int b0 = 0; b0 < batch; b0 += bc) {
    const int nb = std::min(bc, batch - b0);
    if (int rc = run_chunk(src.shifted(b0), n + b0, nb, num_test, num_ransac_test, iters, thr, seed, cheir, w, bc,
                           E_out + (size_t)b0 * 9, P_out ? P_out + (size_t)b0 * 12 : nullptr, inliers_out + b0,
                           winner_out ? winner_out + b0 : nullptr,
                           score_out ? score_out + (size_t)b0 * H : nullptr, s, b0 == 0))
      return rc;
  }
  return SFM_OK;
}

static int run_packed(const double* pts, int64_t n_stride, const int64_t* n, int batch, int num_test,
                      int num_ransac_test, int iters, double thr, uint64_t seed, int cheir, void* ws,
                      size_t ws_bytes, double* E_out, double* P_out, int32_t* inliers_out, int32_t* winner_out,
                      int32_t* score_out, hipStream_t s) {
  if (int rc = check_common(iters, thr, batch)) return rc;
  SFM_REQUIRE(pts && n && E_out && inliers_out, "null pointer argument");
  SFM_REQUIRE(cheir == 0 || P_out, "P_out required when cheirality is on");
  SFM_REQUIRE(n_stride >= 1 && n_stride <= (int64_t)INT32_MAX, "n_stride out of range");
  for (int b = 0; b < batch; ++b) {
    SFM_REQUIRE(n[b] >= 1 && n[b] <= n_stride, "each n[b] must be in [1, n_stride]");
    SFM_REQUIRE(num_test <= n[b] && num_ransac_test <= n[b],
                "num_test_points / num_ransac_test_points must not exceed the number of points");
  }
  return run_src(PackedSrc{pts, n_stride}, n, batch, num_test, num_ransac_test, iters, thr, seed, cheir, ws,
                 ws_bytes, E_out, P_out, inliers_out, winner_out, score_out, s);
}

}  // namespace sfm

using namespace sfm;

extern "C" {

size_t sfm_ransac5_workspace_bytes(int batch, int64_t n_max, int iters) {
  if (batch < 1 || iters < 1) return 0;
  return layout(nullptr, std::min(batch, SFM_MAX_BATCH), n_max, iters, nullptr);
}

int sfm_ransac5(const double* q, const double* qp, int64_t n, int num_test, int num_ransac_test, int iters,
                double thr, uint64_t seed, int cheirality, void* workspace, size_t workspace_bytes,
                double* E_out, double* P_out, int32_t* inliers_out, int32_t* winner_out, void* stream) {
  SFM_REQUIRE(q && qp, "null point arrays");
  SFM_REQUIRE(n >= 1, "need at least one correspondence");
  SFM_REQUIRE(num_test >= 1 && num_ransac_test >= 1, "num_test_points and num_ransac_test_points must be >= 1");
  const size_t need = layout(nullptr, 1, n, iters < 1 ? 1 : iters, nullptr);
  if (!workspace || workspace_bytes < need) {
    set_error("workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  Workspace w;
  layout((char*)workspace, 1, n, iters < 1 ? 1 : iters, &w);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, q, qp, n, w.pack);
  SFM_LAUNCHED();
  const int64_t nn[1] = {n};
  return run_packed(w.pack, n, nn, 1, num_test, num_ransac_test, iters, thr, seed, cheirality, workspace,
                    workspace_bytes, E_out, P_out, inliers_out, winner_out, nullptr, s);
}

int sfm_ransac5_packed(const double* pts, int64_t n_stride, const int64_t* n, int batch, int num_test,
                       int num_ransac_test, int iters, double thr, uint64_t seed, int cheirality,
                       void* workspace, size_t workspace_bytes, double* E_out, double* P_out,
                       int32_t* inliers_out, int32_t* winner_out, int32_t* hyp_score_out, void* stream) {
  return run_packed(pts, n_stride, n, batch, num_test, num_ransac_test, iters, thr, seed, cheirality, workspace,
                    workspace_bytes, E_out, P_out, inliers_out, winner_out, hyp_score_out, (hipStream_t)stream);
}

int sfm_ransac5_flow(const float* flow, int batch, int H, int W, int h_side, int w_side, int margin,
                     const float* Kinv, int num_test, int num_ransac_test, int iters, double thr, uint64_t seed,
                     int cheirality, void* workspace, size_t workspace_bytes, double* E_out, double* P_out,
                     int32_t* inliers_out, int32_t* winner_out, int32_t* hyp_score_out, void* stream) {
  if (int rc = check_common(iters, thr, batch)) return rc;
  SFM_REQUIRE(flow && Kinv && E_out && inliers_out, "null pointer argument");
  SFM_REQUIRE(cheirality == 0 || P_out, "P_out required when cheirality is on");
  SFM_REQUIRE(H >= 1 && W >= 1 && h_side >= 1 && h_side <= H && w_side >= 1 && w_side <= W,
              "h_side/w_side out of range");
  SFM_REQUIRE(margin >= 0 && 2 * margin < h_side && 2 * margin < w_side, "margin leaves no pixels");
  const int64_t N = (int64_t)(h_side - 2 * margin) * (w_side - 2 * margin);
  SFM_REQUIRE(N >= 5 && N <= (int64_t)INT32_MAX, "point count out of range");
  SFM_REQUIRE(num_test <= N && num_ransac_test <= N,
              "num_test_points / num_ransac_test_points must not exceed the number of points");
  std::vector<int64_t> n((size_t)batch, N);
  const FlowSrc src{flow, Kinv, H, W, w_side - 2 * margin, margin, 1.0 / (double)(w_side - 2 * margin)};
  return run_src(src, n.data(), batch, num_test, num_ransac_test, iters, thr, seed, cheirality, workspace,
                 workspace_bytes, E_out, P_out, inliers_out, winner_out, hyp_score_out, (hipStream_t)stream);
}

int sfm_score_fence_enable(int on) {
  std::lock_guard<std::mutex> lk(g_fence_mu);
  g_fence_refs = on ? g_fence_refs + 1 : std::max(0, g_fence_refs - 1);
  return SFM_OK;
}

int sfm_score_fence_wait(void* stream) {
  std::lock_guard<std::mutex> lk(g_fence_mu);
  SFM_REQUIRE(g_fence_refs > 0, "score fence not enabled");
  hipEvent_t ev = nullptr;
  if (int rc = fence_of((hipStream_t)stream, &ev)) return rc;
  SFM_HIP(hipStreamWaitEvent((hipStream_t)stream, ev, 0));
  return SFM_OK;
}

int sfm_score_gate(void* stream, void* waiter, int arm) {
  std::lock_guard<std::mutex> lk(g_fence_mu);
  int dev = 0;
  if (int rc = stream_device((hipStream_t)stream, &dev)) return rc;
  ScoreGate* slot = nullptr;
  for (ScoreGate& g : g_gates)
    if (g.dev == dev && g.waiter == (hipStream_t)waiter) slot = &g;
  if (!arm) {
    if (slot) {
      slot->armed = false;
      slot->dev = -1;
    }
    return SFM_OK;
  }
  if (!slot) {
    for (ScoreGate& g : g_gates)                             // a free slot, one with this device's event first
      if (g.dev < 0 && (!slot || (g.evdev == dev && slot->evdev != dev))) slot = &g;
    SFM_REQUIRE(slot != nullptr, "score gate: too many armed (device, stream) gates");
  }
  if (slot->evdev != dev) {
    if (slot->ev) {                                          // an event of another device
      hipEvent_t old = slot->ev;
      slot->ev = nullptr;
      slot->evdev = -1;
      SFM_HIP(hipEventDestroy(old));
    }
    int cur = 0;
    SFM_HIP(hipGetDevice(&cur));
    SFM_HIP(hipSetDevice(dev));
    const hipError_t e = hipEventCreateWithFlags(&slot->ev, hipEventDisableTiming);
    SFM_HIP(hipSetDevice(cur));
    SFM_HIP(e);
    slot->evdev = dev;
  }
  SFM_HIP(hipEventRecord(slot->ev, (hipStream_t)stream));
  slot->dev = dev;
  slot->waiter = (hipStream_t)waiter;
  slot->armed = true;
  return SFM_OK;
}

size_t sfm_score_essentials_workspace_bytes(int batch, int ncand) {
  if (batch < 1 || batch > SFM_MAX_BATCH || ncand < 1) return 0;
  const size_t c = (size_t)batch * ncand;
  return align_up(SFM_MAX_BATCH * 4) + align_up(c * kCandStride * 8) + align_up(c * kMfRec * 2) + align_up(c * 4) +
         align_up(kMf2ClaimBytes);
}

int sfm_score_essentials(const double* pts, int64_t n_stride, const int64_t* n, int batch, const double* E,
                         int ncand, double thr, int32_t* counts, void* workspace, size_t workspace_bytes,
                         void* stream) {
  SFM_REQUIRE(pts && n && E && counts, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && batch <= SFM_MAX_BATCH, "batch must be in [1, 64]");
  SFM_REQUIRE(ncand >= 1 && ncand <= (1 << 20), "ncand must be in [1, 2^20]");
  SFM_REQUIRE(thr > 0.0, "inlier threshold must be > 0");
  SFM_REQUIRE(n_stride >= 1 && n_stride <= (int64_t)INT32_MAX, "n_stride out of range");
  for (int b = 0; b < batch; ++b) SFM_REQUIRE(n[b] >= 1 && n[b] <= n_stride, "each n[b] must be in [1, n_stride]");
  const size_t need = sfm_score_essentials_workspace_bytes(batch, ncand);
  if (!workspace || workspace_bytes < need) {
    set_error("workspace too small: need " + std::to_string(need) + " bytes");
    return SFM_ERR_WORKSPACE;
  }
  hipStream_t s = (hipStream_t)stream;
  char* p = (char*)workspace;
  const size_t c = (size_t)batch * ncand;
  ScoreBufs w;
  w.cand_total = (int32_t*)p;
  p += align_up(SFM_MAX_BATCH * 4);
  w.candE = (double*)p;
  p += align_up(c * kCandStride * 8);
  w.candF = (_Float16*)p;
  p += align_up(c * kMfRec * 2);
  w.cntR = (int32_t*)p;
  p += align_up(c * 4);
  w.claim = (unsigned long long*)p;
  w.cntT = counts;
  PairParams pp{};
  for (int b = 0; b < batch; ++b) {
    pp.n[b] = n[b];
    pp.test[b] = pp.rtest[b] = (int32_t)n[b];
    pp.splits[b] = (int32_t)((n[b] + kPtsPerItem - 1) / kPtsPerItem);
  }
  const int prec = lowp_prec();
  const bool fast = prec == 64 && thr >= 0x1p-40 && thr < 1.0;
  const double guard_g = fast ? 0x1p24 * (11.0 + 11.0 / thr) : 0.0;
  const bool fast32 = fast && thr >= 0x1p-20 && tuning().score_fp32;
  ScoreConsts kc{};
  kc.thr = thr;
  kc.t2lo = (thr * thr) * (1.0 - 0x1p-22);
  kc.t2hi = (thr * thr) * (1.0 + 0x1p-22);
  kc.t2lo32 = (float)((thr * thr) * (1.0 - 0x1p-6 - 0x1p-19));
  kc.t2hi32 = (float)((thr * thr) * (1.0 + 0x1p-7) / (1.0 - 0x1p-7) * (1.0 + 0x1p-19));
  kc.fast32 = fast32 ? 1 : 0;
  kc.prune = 0;
  kc.ws_batch = batch;
  kc.interleave = tuning().score_interleave;
  MfParams mp{};
  const bool use_mf = fast32 && tuning().score_mf && mf_params(thr, &mp);
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = std::max(1, cus) * tuning().score_blocks_per_cu;
  SFM_HIP(hipMemsetAsync(w.cntT, 0, c * 4, s));
  SFM_HIP(hipMemsetAsync(w.cntR, 0, c * 4, s));
  hipLaunchKernelGGL(k_fill_cands, dim3((ncand + 255) / 256, batch), dim3(256), 0, s, E, ncand, ncand, guard_g, thr,
                     fast32 ? 1 : 0, w.candE, w.cand_total);
  ProfScope ps("score_essentials", s);
  score_dispatch(PackedSrc{pts, n_stride}, pp, batch, ncand, w, kc, mp, use_mf, true, prec, fast, fast32, cus, grid,
                 s);
  SFM_LAUNCHED();
  return SFM_OK;
}

int sfm_ransac5_inlier_mask(const double* pts, int64_t n_stride, const int64_t* n, int batch, const double* E,
                            double thr, uint8_t* mask, void* stream) {
  SFM_REQUIRE(pts && n && E && mask, "null pointer argument");
  SFM_REQUIRE(batch >= 1, "batch must be >= 1");
  hipStream_t s = (hipStream_t)stream;
  for (int b0 = 0; b0 < batch; b0 += SFM_MAX_BATCH) {
    const int nb = std::min(SFM_MAX_BATCH, batch - b0);
    PairParams pp{};
    for (int b = 0; b < nb; ++b) {
      SFM_REQUIRE(n[b0 + b] >= 0 && n[b0 + b] <= n_stride, "n[b] must be in [0, n_stride]");
      pp.n[b] = n[b0 + b];
    }
    hipLaunchKernelGGL(k_inlier_mask, dim3((unsigned)((n_stride + 255) / 256), nb), dim3(256), 0, s,
                       pts + (size_t)b0 * n_stride * 4, n_stride, pp, E + (size_t)b0 * 9, thr,
                       mask + (size_t)b0 * n_stride);
    SFM_LAUNCHED();
  }
  return SFM_OK;
}

int sfm_ransac5_candidate_counts(const void* workspace, size_t workspace_bytes, int batch, int iters,
                                 int32_t* counts_host) {
  SFM_REQUIRE(workspace && counts_host && batch >= 1 && batch <= SFM_MAX_BATCH && iters >= 1, "invalid arguments");
  const int bc = batch;
  SFM_REQUIRE(workspace_bytes >= layout(nullptr, bc, 0, iters, nullptr), "workspace too small");
  Workspace w;
  layout((char*)workspace, bc, 0, iters, &w);
  SFM_HIP(hipMemcpy(counts_host, w.cand_total, sizeof(int32_t) * batch, hipMemcpyDeviceToHost));
  return SFM_OK;
}

int sfm_ransac5_skipped_evaluations(const void* workspace, size_t workspace_bytes, int batch, int iters,
                                    unsigned long long* skipped_host) {
  SFM_REQUIRE(workspace && skipped_host && batch >= 1 && iters >= 1, "invalid arguments");
  const int bc = std::min(batch, SFM_MAX_BATCH);
  SFM_REQUIRE(workspace_bytes >= layout(nullptr, bc, 0, iters, nullptr), "workspace too small");
  Workspace w;
  layout((char*)workspace, bc, 0, iters, &w);
  SFM_HIP(hipMemcpy(skipped_host, w.skipped, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return SFM_OK;
}

int sfm_ransac5_kept_candidates(const void* workspace, size_t workspace_bytes, int batch, int iters,
                                int32_t* kept_host, int32_t* points_host) {
  SFM_REQUIRE(workspace && kept_host && batch >= 1 && batch <= SFM_MAX_BATCH && iters >= 1, "invalid arguments");
  SFM_REQUIRE(workspace_bytes >= layout(nullptr, batch, 0, iters, nullptr), "workspace too small");
  Workspace w;
  layout((char*)workspace, batch, 0, iters, &w);
  SFM_HIP(hipMemcpy(kept_host, w.lead + 3 * SFM_MAX_BATCH, sizeof(int32_t) * batch, hipMemcpyDeviceToHost));
  if (points_host) {
    SFM_HIP(hipMemcpy(points_host, w.bnd + 2 * SFM_MAX_BATCH, sizeof(int32_t) * batch, hipMemcpyDeviceToHost));
    for (int b = 0; b < batch; ++b) points_host[b] *= kMf2Span;   // spans -> points (the caller clamps at N)
  }
  return SFM_OK;
}

int sfm_pack_points(const double* q, const double* qp, int64_t n, double* pts_out, void* stream) {
  SFM_REQUIRE(q && qp && pts_out && n >= 0, "invalid arguments");
  if (n == 0) return SFM_OK;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, q, qp, n,
                     pts_out);
  SFM_LAUNCHED();
  return SFM_OK;
}

int sfm_flow_to_points(const float* flow, int batch, int H, int W, int h_side, int w_side, int margin,
                       const float* Kinv, double* pts_out, void* stream) {
  SFM_REQUIRE(flow && Kinv && pts_out, "null pointer argument");
  SFM_REQUIRE(batch >= 1 && H >= 1 && W >= 1, "invalid flow shape");
  SFM_REQUIRE(h_side >= 1 && h_side <= H && w_side >= 1 && w_side <= W, "h_side/w_side out of range");
  SFM_REQUIRE(margin >= 0 && 2 * margin < h_side && 2 * margin < w_side, "margin leaves no pixels");
  const int64_t N = (int64_t)(h_side - 2 * margin) * (w_side - 2 * margin);
  hipStream_t s = (hipStream_t)stream;
  for (int b0 = 0; b0 < batch; b0 += 65535) {
    const int nb = std::min(65535, batch - b0);
    ProfScope ps("flow_to_points", s);
    const FlowSrc src{flow + (size_t)b0 * 2 * H * W, Kinv + (size_t)b0 * 9, H, W, w_side - 2 * margin, margin,
                      1.0 / (double)(w_side - 2 * margin)};
    hipLaunchKernelGGL(k_flow_points, dim3((unsigned)((N + 255) / 256), nb), dim3(256), 0, s, src, N,
                       pts_out + (size_t)b0 * N * 4);
  }
  SFM_LAUNCHED();
  return SFM_OK;
}

int sfm_keypoints_to_points(const float* flow, int batch, int H, int W, int h_side, int w_side,
                            const float* kp1, const float* kp2, int64_t kp_stride, const int64_t* n, int mode,
                            const float* Kinv, double* pts_out, int64_t n_stride, void* stream) {
  SFM_REQUIRE(kp1 && n && Kinv && pts_out, "null pointer argument");
  SFM_REQUIRE(mode >= 0 && mode <= 2, "mode must be 0 (rounded gather), 1 (SAMPLE_SP) or 2 (SIFT_POSE)");
  SFM_REQUIRE(mode == 2 || flow, "null flow");
  SFM_REQUIRE(mode != 2 || kp2, "SIFT_POSE needs the target keypoints");
  SFM_REQUIRE(batch >= 1 && H >= 1 && W >= 1, "invalid flow shape");
  SFM_REQUIRE(h_side >= 1 && h_side <= H && w_side >= 1 && w_side <= W, "h_side/w_side out of range");
  int64_t nmax = 0;
  for (int b = 0; b < batch; ++b) {
    SFM_REQUIRE(n[b] >= 0 && n[b] <= kp_stride && n[b] <= n_stride && n[b] < (1 << 30),
                "keypoint count out of range");
    nmax = std::max(nmax, n[b]);
  }
  hipStream_t s = (hipStream_t)stream;
  ProfScope ps("keypoints_to_points", s);
  for (int b0 = 0; b0 < batch; b0 += SFM_MAX_BATCH) {
    const int nb = std::min(SFM_MAX_BATCH, batch - b0);
    KpCounts c;
    int64_t m = 0;
    for (int b = 0; b < nb; ++b) { c.n[b] = (int)n[b0 + b]; m = std::max(m, n[b0 + b]); }
    if (m == 0) continue;
    hipLaunchKernelGGL(k_keypoint_points, dim3((unsigned)((m + 255) / 256), nb), dim3(256), 0, s,
                       mode == 2 ? nullptr : flow + (size_t)b0 * 2 * H * W, H, W, h_side, w_side,
                       kp1 + (size_t)b0 * kp_stride * 2, mode == 2 ? kp2 + (size_t)b0 * kp_stride * 2 : nullptr,
                       kp_stride, c, mode, Kinv + (size_t)b0 * 9, pts_out + (size_t)b0 * n_stride * 4, n_stride);
  }
  (void)nmax;
  SFM_LAUNCHED();
  return SFM_OK;
}

}  // extern "C"
