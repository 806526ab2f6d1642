// Phase 3e of the RANSAC (included by ransac5.hip after score_mf.h): the
// span-major split-f16 matrix-core scorer, k_score_mf2 (default for SFMnet's
// num_test == num_ransac_test; tuning key score_mf = 2).
//
// Same arithmetic and decisions as k_score_mf (the A rows of k_mf_cands, the
// B columns of mf_stage_point, mf_tile_mfma, mf_tile_decide, the float64
// re-test of the undecided band), so every count is identical; what changes
// is how the work is laid out on the chip:
//
//   * Work units are (pair, 1024-point span, 32-candidate tile), ordered
//     span-major within a pair, and each persistent block takes one
//     contiguous range of ~U / grid units.  The block stages a span once
//     (B fragments + float64 points, one LDS image) and its 12 waves run
//     every candidate tile of that span in its range, 25-26 each per span at
//     KITTI size; one LDS barrier pair per span, not per candidate group.
//     The per-pair tail of k_score_mf (the last candidate group of a pair
//     leaving up to half the waves of an item idle) does not exist: the
//     range split is exact to one unit.
//   * Logical block ranges are contiguous per XCD (block id % 8 picks the
//     XCD), so an XCD's blocks work on one or two pairs and that pair's A
//     rows (1.3 MB) and E rows stay in its L2.
//   * The tile loop keeps the matrix pipe and the vector issue busy together
//     from one wave: round 2's decisions ran two accumulator sets (tile t+1's
//     four MFMAs before tile t's 64 decision VALU; scripts/probe_tile.hip: 247
//     -> 213 SIMD cycles per tile at 3 waves per SIMD); the folded decisions
//     (SFM_MF2_FOLD, default) pipeline a / aa+z / signs over three tiles with
//     48 decision VALU per tile.  Spans are 32 tiles: the 32-bit
//     decision strings are full, and a run's fixed costs (A rows, queue,
//     float64 drain, count reduction) spread over 32 tiles instead of 24.
//   * The next run's A rows load right after the tile loop, under the
//     queue / drain / reduction of the current run.
//
// Registers (gfx950, 3 waves per SIMD = 168 VGPRs): 2 x 48 accumulators + 16
// A + 12 B + 32 decision strings in the loop.
#ifndef SFM_MF2_SCHED
#define SFM_MF2_SCHED 1
#endif
#ifndef SFM_MF2_EARLY_CLAIM
#define SFM_MF2_EARLY_CLAIM 0
#endif
#ifndef SFM_MF2_SPAN
#define SFM_MF2_SPAN 1024
#endif
#ifndef SFM_MF2_WAVES
#define SFM_MF2_WAVES 12
#endif
// Per-block LDS count table (round 4): a run's counts are added into an LDS
// table of the pair's candidates (tile k of a span belongs to one wave, and a
// block barrier separates spans, so the adds need no atomics); the table goes
// to the global counts with one atomic per nonzero candidate when the block
// moves to another pair or ends.  Round 3 published every (span, candidate)
// with two global atomics: 0.27 GB of atomic traffic per launch at C2.
// SFM_MF2_TBL 2: 16-bit counts, two per LDS word (ds_add_u32 of d or d << 16:
// a half never carries, because the table is flushed before any candidate's
// count can pass 63 spans x 1024 points), so the table fits beside the LDS
// copy of the span's points.
#ifndef SFM_MF2_TBL
#define SFM_MF2_TBL 2
#endif
// the float64 drain reads its points from global memory (L2) instead of an LDS
// copy of the span: the 32 KB make room for the count table
#ifndef SFM_MF2_GPTS
#define SFM_MF2_GPTS (SFM_MF2_TBL == 1)
#endif
#ifndef SFM_MF2_FOLD
#define SFM_MF2_FOLD 1
#endif
// Experiment builds only (timing of the parts; WRONG counts): bit 1 skips the
// undecided queue and float64 drain, bit 2 the count reduction and publishing
// (the decision strings go to a sink instead), bit 4 the per-run A-row reloads
// (every run reuses its first rows), bit 8 the span staging after a block's
// first span (profiles/r04_mf2_parts_ab.txt).
#ifndef SFM_MF2_EXP
#define SFM_MF2_EXP 0
#endif
// (Round 4 also measured, and dropped: aa as packed v_pk_mul_f32; s_setprio
// around the MFMA groups; the sign harvest as v_perm_b32 + v_bitop3_b32; a
// lane pointer walking the span -- profiles/r04_mf2_prio_pk_ab.txt.)
// the tile loop's fragment addresses from one lane base per two tiles (1;
// measured 0.8 % slower than the lane id per tile, 0: profiles/r04_mf2_ln1_ab.txt)
#ifndef SFM_MF2_LN1
#define SFM_MF2_LN1 0
#endif
#ifndef SFM_MF2_BPRE
#define SFM_MF2_BPRE 0
#endif
// queue build: each word's first undecided bit written straight-line, the
// rare further bits of the same word in a loop behind a wave-uniform test
#ifndef SFM_MF2_DYN
#define SFM_MF2_DYN 1
#endif
#ifndef SFM_MF2_MINCHUNK
#define SFM_MF2_MINCHUNK 128
#endif
constexpr int kMf2MinChunk = SFM_MF2_MINCHUNK;               // smallest claimed unit range (candidate tiles)
#ifndef SFM_MF2_ALIGN
#define SFM_MF2_ALIGN 0   // 1 measured slower (profiles/r03_mf2_align_ab.txt)
#endif
#ifndef SFM_MF2_GUIDE
#define SFM_MF2_GUIDE 2
#endif
constexpr int kMf2Guide = SFM_MF2_GUIDE;                     // a claim takes remainder / (guide x blocks per XCD)
#ifndef SFM_MF2_QB
#define SFM_MF2_QB 0   // 1 measured slower (profiles/r03_mf2_qb_ab.txt)
#endif
constexpr int kMf2Waves = SFM_MF2_WAVES;       // 12: 3 per SIMD, two accumulator sets; 16: 4 per SIMD, one
constexpr int kMf2Wpe = kMf2Waves / 4;
constexpr int kMf2Span = SFM_MF2_SPAN;         // points per staged span
constexpr int kMf2Tiles = kMf2Span / 32;       // tiles per span (every run decides all of them)
#ifndef SFM_MF2_QLEN
#define SFM_MF2_QLEN (SFM_MF2_TBL == 2 ? 128 : (SFM_MF2_TBL || SFM_MF2_WAVES > 12) ? 256 : 512)
#endif
#ifndef SFM_MF2_TBLCAP
#define SFM_MF2_TBLCAP (SFM_MF2_TBL == 2 ? 352 : 384)
#endif
constexpr int kMf2Queue = SFM_MF2_QLEN;        // undecided entries per wave and drain window (LDS)
// candidate tiles the LDS count table holds (tiles past it publish per run)
constexpr int kMf2TblTiles = SFM_MF2_TBL ? SFM_MF2_TBLCAP : 1;
constexpr int kMf2TblWords = SFM_MF2_TBL == 2 ? kMf2TblTiles * kKC / 2 : kMf2TblTiles * kKC;
constexpr int kMf2TblSpans = 63;               // TBL 2: spans between flushes (63 x 1024 < 2^16)
static_assert(SFM_MF2_TBL != 2 || kMf2Span <= 1024, "16-bit table counts");
static_assert(kMf2Tiles <= 32 && kMf2Tiles % 2 == 0, "32-bit decision strings, tiles in pairs");

#ifdef SFM_MF_STATS
// experiment builds only: [0] undecided evaluations, [1] evaluations decided by the tile loop
__device__ unsigned long long g_mf2_stats[2];
extern "C" int sfm_experiment_mf_stats(unsigned long long* out, int reset) {
  if (reset) {
    unsigned long long z[2] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_mf2_stats), z, sizeof(z)) == hipSuccess ? 0 : 2;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mf2_stats), 16) == hipSuccess ? 0 : 2;
}
#endif

// The float64 test of queued (row, span-relative point) entries; E rows from
// the candidate records in global memory (L1/L2-resident: the tile's 32
// records), points from the staged span.
__device__ __forceinline__ void mf2_drain(const double* __restrict__ Erow0, const double4* __restrict__ spts,
                                          const ScoreConsts& kc, int lane, int32_t* cnt, const uint32_t* q, int qn) {
#pragma unroll 1
  for (int i = lane; i < qn; i += 64) {
    const uint32_t e = q[i];
    const int c = (int)(e >> 24), r = (int)(e & 0xffffffu);
    if (inlier_f64v(Erow0 + (size_t)c * kCandStride, spts[r], kc)) atomicAdd(&cnt[c], 1);
  }
}

// The same test with each entry's point read from global memory (SFM_MF2_GPTS;
// the span's points are L2-resident: the block staged them from there)
template <class Src>
__device__ __forceinline__ void mf2_drain_src(const double* __restrict__ Erow0, const Src& src, int b, int p0,
                                              const ScoreConsts& kc, int lane, int32_t* cnt, const uint32_t* q,
                                              int qn) {
#pragma unroll 1
  for (int i = lane; i < qn; i += 64) {
    const uint32_t e = q[i];
    const int c = (int)(e >> 24), r = (int)(e & 0xffffffu);
    if (inlier_f64v(Erow0 + (size_t)c * kCandStride, src.load(b, (int64_t)p0 + r), kc)) atomicAdd(&cnt[c], 1);
  }
}
// (Round 3 measured a queue carried across runs, SFM_MF2_CARRY, and dropped
// it: profiles/r03_mf2_carry_ab.txt.)

// mf_tile_decide with each register's decisions kept together (scheduling
// barriers): the compiler otherwise hoists all 32 FMAs of a tile ahead of the
// shifts, 32 temporaries that the two accumulator sets leave no room for
__device__ __forceinline__ void mf2_decide(const MfAcc& r, uint32_t (&s1)[16], uint32_t (&s2)[16]) {
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const float z1 = __builtin_fmaf(r.a[g], r.a[g], -r.lo[g]);
    const float z2 = __builtin_fmaf(-r.a[g], r.a[g], r.hi[g]);
    s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(z1), 31);
    s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(z2), 31);
#if SFM_MF2_SCHED
    __builtin_amdgcn_sched_barrier(0);
#endif
  }
}

// SFM_MF2_FOLD (12-wave build): a^2 folded into the band MFMAs (the bound:
// score_mf.h, kMfFoldLo / kMfFoldHi).  Per tile a = two MFMAs as before, then
// aa = a * a (16 VALU) becomes the C operand of z1 = aa - Ylo and z2 = aa - Yhi
// (the A rows of Ylo / Yhi negated once per run), and the decisions are the
// two sign bits alone: 48 VALU per tile instead of 64 (the two FMAs per
// evaluation become one multiply).  s1 holds inlier bits (z1 < 0) as before;
// s2 holds NOT-outlier bits (z2 < 0), so undecided = s2 & ~s1.
// Pipelined over three tiles: tile t+1's a MFMAs, tile t's aa and z MFMAs and
// tile t-1's sign bits in one step.
struct MfAB {                                                 // a fragments of one tile (ds_read_b128 x 2)
  mf_half8 b1, b2;
};
__device__ __forceinline__ MfAB mf2_load_ab(const _Float16* frag_tile, int lane) {
  MfAB b;
  b.b1 = *reinterpret_cast<const mf_half8*>(frag_tile + (size_t)(0 * 64 + lane) * 8);
  b.b2 = *reinterpret_cast<const mf_half8*>(frag_tile + (size_t)(1 * 64 + lane) * 8);
  return b;
}
__device__ __forceinline__ mf_half8 mf2_load_d(const _Float16* frag_tile, int lane) {
  return *reinterpret_cast<const mf_half8*>(frag_tile + (size_t)(2 * 64 + lane) * 8);
}
__device__ __forceinline__ mf_float16 mf2_a(const MfAB& B, mf_half8 A1, mf_half8 A2) {
  mf_float16 z;
#pragma unroll
  for (int g = 0; g < 16; ++g) z[g] = 0.0f;
  const mf_float16 a = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B.b1, z, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(A2, B.b2, a, 0, 0, 0);
}
struct MfZ {
  mf_float16 z1, z2;
};
#ifndef SFM_MF2_PK
#define SFM_MF2_PK 0   // measured slower (profiles/r03_mf2_pk_ab.txt)
#endif
typedef float mf_float2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ MfZ mf2_z(mf_half8 bd, mf_half8 NL, mf_half8 NH, const mf_float16& a) {
  mf_float16 aa;
#if SFM_MF2_PK
  // aa = a * a as eight packed multiplies (v_pk_mul_f32: two IEEE float32
  // products per instruction, the same bits as v_mul_f32)
#pragma unroll
  for (int g = 0; g < 16; g += 2) {
    mf_float2 v = {a[g], a[g + 1]};
    v = v * v;
    aa[g] = v.x;
    aa[g + 1] = v.y;
  }
#else
#pragma unroll
  for (int g = 0; g < 16; ++g) aa[g] = a[g] * a[g];
#endif
  MfZ r;
  r.z1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(NL, bd, aa, 0, 0, 0);
  r.z2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(NH, bd, aa, 0, 0, 0);
  return r;
}
__device__ __forceinline__ void mf2_signs(const MfZ& r, uint32_t (&s1)[16], uint32_t (&s2)[16]) {
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    s1[g] = __builtin_amdgcn_alignbit(s1[g], __float_as_uint(r.z1[g]), 31);
    s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(r.z2[g]), 31);
  }
}
constexpr bool kMf2Fold = SFM_MF2_FOLD;

// queue entry (candidate row << 24 | span-relative point) of the lowest set
// bit j of a string: bit j = tile kMf2Tiles - 1 - j
__device__ __forceinline__ uint32_t mf2_qbase(int g, int hl, int rl) {
  return ((uint32_t)mf_row(g, hl) << 24) | (uint32_t)(32 * (kMf2Tiles - 1) + rl);
}
__device__ __forceinline__ uint32_t mf2_qentry(uint32_t base, uint32_t uu) {
  return base - 32u * (uint32_t)__builtin_ctz(uu);
}
// undecided evaluations of a decision-string pair
__device__ __forceinline__ uint32_t mf2_undecided(uint32_t s1, uint32_t s2) {
  return kMf2Fold ? (s2 & ~s1) : ~(s1 | s2);
}

// the lane id, recomputed where it is used (v_mbcnt) instead of kept live
// across the tile loop, where every VGPR is taken
__device__ __forceinline__ int mf2_lane() {
  int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(l));
  return l;
}

#ifdef SFM_MF2_BLOCKT
__device__ unsigned long long g_mf2_blockt[3 * 4096];
extern "C" int sfm_experiment_mf2_blockt(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mf2_blockt), (size_t)3 * n * 8) == hipSuccess ? 0 : 2;
}
#endif
template <class Src>
__global__ __launch_bounds__(kMf2Waves * 64) __attribute__((amdgpu_waves_per_eu(kMf2Wpe, kMf2Wpe))) void k_score_mf2(
    const Src src, PairParams pp, int batch, int cmax, const int32_t* __restrict__ cand_total,
    const double* __restrict__ candE, const _Float16* __restrict__ candF, int32_t* __restrict__ cntT,
    ScoreConsts kc, unsigned long long* __restrict__ claim) {
  // one count array: this kernel runs only when num_test == num_ransac_test,
  // so the preselection count is the score and k_select reads cntT for both
  __shared__ __attribute__((aligned(16))) _Float16 s_frag[kMf2Tiles][3][64][8];
#if !SFM_MF2_GPTS
  __shared__ double4 s_pts[kMf2Span];
#endif
#if SFM_MF2_TBL
  __shared__ int32_t s_tbl[kMf2TblWords];                    // the block's counts of pair tb's candidates
#endif
  __shared__ uint32_t s_queue[kMf2Waves][kMf2Queue];
  __shared__ int32_t s_cnt[kMf2Waves][kKC];                  // float64 drain counts
  __shared__ long long s_first[SFM_MAX_BATCH + 1];           // first unit of each pair
  __shared__ int32_t s_tiles[SFM_MAX_BATCH];                 // candidate tiles per pair
  __shared__ int32_t s_ctot[SFM_MAX_BATCH];
  __shared__ int32_t s_claim;                                // next candidate tile of the span to claim
  __shared__ long long s_range[2];                           // the block's current unit range
  const int tid = threadIdx.x, wv = tid >> 6;
  if (tid == 0) {
    long long acc = 0;
    for (int b = 0; b < batch; ++b) {
      const int ct = cand_total[b];
      const int tiles = (ct + kKC - 1) / kKC;
      const long long spans = (max(pp.test[b], pp.rtest[b]) + kMf2Span - 1) / kMf2Span;
      s_first[b] = acc;
      s_tiles[b] = tiles;
      s_ctot[b] = ct;
      acc += spans * tiles;
    }
    s_first[batch] = acc;
  }
  for (int i = tid; i < kMf2Waves * kKC; i += kMf2Waves * 64) (&s_cnt[0][0])[i] = 0;
#if SFM_MF2_TBL
  for (int i = tid; i < kMf2TblWords; i += kMf2Waves * 64) s_tbl[i] = 0;
  int tb = -1;                                               // the pair the table holds (block-uniform)
  int tspans = 0;                                            // spans added since the last flush
  // the table to pair fb's global counts (all threads, between block barriers)
  auto flush = [&](int fb) {
    const int nt = min(s_tiles[fb], kMf2TblTiles) * kKC;
    int32_t* dst = cntT + (size_t)fb * cmax;
    if (SFM_MF2_TBL == 2) {
      for (int i = tid; i < nt / 2; i += kMf2Waves * 64) {
        const uint32_t v = (uint32_t)s_tbl[i];
        if (v) {
          if (v & 0xffffu) atomicAdd(dst + 2 * i, (int)(v & 0xffffu));
          if (v >> 16) atomicAdd(dst + 2 * i + 1, (int)(v >> 16));
          s_tbl[i] = 0;
        }
      }
    } else {
      for (int i = tid; i < nt; i += kMf2Waves * 64) {
        const int v = s_tbl[i];
        if (v) {
          atomicAdd(dst + i, v);
          s_tbl[i] = 0;
        }
      }
    }
  };
#endif
  __syncthreads();
#ifdef SFM_MF2_BLOCKT
  const unsigned long long blk_t0 = __builtin_amdgcn_s_memrealtime();
#endif
  // Unit ranges: workgroup ids are dealt round-robin over the 8 XCDs, so
  // id % 8 names the XCD.  SFM_MF2_DYN (default): XCD x owns the x-th eighth
  // of the units (about one pair, whose A rows then stay in that XCD's L2),
  // and its blocks claim guided chunks of it from a global counter (half the
  // remainder's per-block share, at least kMf2MinChunk units); a block whose
  // eighth is exhausted takes chunks of the next XCDs' eighths.  Static
  // contiguous ranges left blocks idle for 6 % of the launch on average
  // (scripts/mf2_blockt.py): units cost unequal time across pairs and XCDs.
  const int G = gridDim.x;
  const long long U = s_first[batch];
#if SFM_MF2_DYN
  const int nx = (G % 8 == 0) ? 8 : 1;
  const int xcd = (int)(blockIdx.x % (unsigned)nx);
  const int per_x = G / nx;
  int victim = 0;                                            // XCDs after our own already drained
  long long units_done = 0;
#else
  const int per_xcd = G / 8;
  const int logical = (G % 8 == 0) ? (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const long long u_beg = U * logical / G, u_end = U * (logical + 1) / G;
#endif
  int32_t* cnt = s_cnt[wv];
  uint32_t* queue = s_queue[wv];
  const _Float16* fr = &s_frag[0][0][0][0];
  constexpr int kTileHalves = 3 * 64 * 8;
#if SFM_MF2_EXP
  uint32_t exp_sink = 0u;
  bool exp_first = true;
#endif
  int b = 0;
#if !SFM_MF2_DYN
  long long u = u_beg;
#endif
  mf_half8 A1, A2, AL, AH;
#ifdef SFM_MF_STAMPS
  // experiment builds (scripts/mf_stamps.py): [0] staging, [1] tile loop,
  // [2] queue build, [3] float64 drain, [4] reduction + atomics, [5] span
  // barriers, [6] A-row load issue, [7] runs
  unsigned long long mf_t0_ = __builtin_amdgcn_s_memtime();
  unsigned long long mf_acc_[kMfStamps] = {};
#endif
  // A rows of candidate tile k of pair b (absent rows: every evaluation a decided outlier)
  auto load_rows = [&](int bb, int k, int ctot) {
    const int ln = mf2_lane();
    const int lh = ln >> 5, lr = ln & 31;
    const int c = k * kKC + lr;
    if (c < ctot) {
      const mf_half8* rec = reinterpret_cast<const mf_half8*>(candF + ((size_t)bb * cmax + c) * kMfRec);
      A1 = rec[0 + lh];
      A2 = rec[2 + lh];
      AL = rec[4 + lh];
      AH = rec[6 + lh];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        A1[j] = (_Float16)0.0f; A2[j] = (_Float16)0.0f; AL[j] = (_Float16)0.0f; AH[j] = (_Float16)0.0f;
      }
      if (lh == 0) {
        AL[2] = (_Float16)(-1.0f); AH[2] = (_Float16)(-1.0f);
      } else {
        AL[6] = (_Float16)(-1.0f); AL[7] = (_Float16)(-1.0f);
        AH[6] = (_Float16)(-1.0f); AH[7] = (_Float16)(-1.0f);
      }
    }
  };
#if SFM_MF2_DYN
  for (;;) {
    if (tid == 0) {
      long long st = U, en = U;
      for (; victim < nx; ++victim) {
        const int x = (xcd + victim) % nx;
        const long long seg_beg = U * x / nx, seg_end = U * (x + 1) / nx;
        // the floor never exceeds a block's static share of the eighth (small
        // launches, e.g. 2,048 keypoints: a 128-unit floor would idle most blocks)
        const long long floor_c = max(min((long long)kMf2MinChunk, (seg_end - seg_beg + per_x - 1) / per_x), 1ll);
#if SFM_MF2_ALIGN
        // chunks of a span or more end on a span boundary, so that a span is
        // staged by one block only (compare-and-swap on the claimed offset)
        unsigned long long cur = __hip_atomic_load(claim + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool done = false;
        while (seg_beg + (long long)cur < seg_end) {
          const long long start = seg_beg + (long long)cur, rem = seg_end - start;
          long long end = min(start + max(floor_c, rem / (kMf2Guide * per_x)), seg_end);
          int pb = 0;
          while (end > s_first[pb + 1]) ++pb;                  // the pair holding unit end - 1
          const long long tl = s_tiles[pb];
          if (end - start >= tl) {
            const long long loc = end - s_first[pb];
            end = min(s_first[pb] + (loc + tl - 1) / tl * tl, seg_end);
          }
          const unsigned long long want = (unsigned long long)(end - seg_beg);
          const unsigned long long seen = atomicCAS(claim + x, cur, want);
          if (seen == cur) {
            st = start;
            en = end;
            done = true;
            break;
          }
          cur = seen;
        }
        if (done) break;
#else
        const long long rem = seg_end - seg_beg - (long long)__hip_atomic_load(claim + x, __ATOMIC_RELAXED,
                                                                                __HIP_MEMORY_SCOPE_AGENT);
        if (rem <= 0) continue;
        const long long size = max(floor_c, rem / (kMf2Guide * per_x));
        const long long got = seg_beg + (long long)atomicAdd(claim + x, (unsigned long long)size);
        if (got < seg_end) {
          st = got;
          en = min(got + size, seg_end);
          break;
        }
#endif
      }
      s_range[0] = st;
      s_range[1] = en;
    }
    __syncthreads();
    long long u = s_range[0];
    const long long u_end = s_range[1];
    if (u >= u_end) break;
    units_done += u_end - u;
    if (u < s_first[b]) b = 0;                               // a stolen chunk may lie before our own
#endif
  while (u < u_end) {
    while (u >= s_first[b + 1]) ++b;
    b = __builtin_amdgcn_readfirstlane(b);
    const int tiles = s_tiles[b];
    const long long local = u - s_first[b];
    const int span = (int)(local / tiles);
    const int k0 = (int)(local - (long long)span * tiles);
    const int k1 = (int)min((long long)tiles, (long long)k0 + (u_end - u));   // this block's tiles of the span
    const int p0 = span * kMf2Span;
    const int np = min(max(pp.test[b], pp.rtest[b]) - p0, kMf2Span);     // live points of the span
#if SFM_MF2_TBL
    // a new pair: the table's counts go out first (every wave's adds to it
    // ended before the barrier that closed the previous span or claim)
    if (b != tb || (SFM_MF2_TBL == 2 && tspans == kMf2TblSpans)) {
      if (tb >= 0) flush(tb);
      tb = b;
      tspans = 0;
    }
    ++tspans;
#endif
    // 1. stage the span: B fragments for every slot (dead slots: the decided-outlier sentinel)
    if (tid == 0) s_claim = 0;
    for (int i = tid; i < kMf2Span; i += kMf2Waves * 64) {
      const bool live = i < np;
      const double4 v = src.load(b, live ? p0 + i : p0);
#if !SFM_MF2_GPTS
      s_pts[i] = v;
#endif
#if SFM_MF2_EXP & 8
      if (exp_first)
#endif
      mf_stage_point(v, live, &s_frag[i >> 5][0][0][0], i & 31);
    }
#if SFM_MF2_EXP & 8
    exp_first = false;
#endif
    MF_STAMP(0);
    lds_barrier();
    MF_STAMP(5);
    // 2. the span's candidate tiles, claimed one run at a time from an LDS
    // counter: the three waves of a SIMD progress at very different rates
    // (issue arbitration favours the oldest), so a static split left the
    // younger waves' tail for the others to wait out at the span barrier
    auto claim = [&]() {
      int j = 0;
      if (mf2_lane() == 0) j = atomicAdd(&s_claim, 1);
      return k0 + __builtin_amdgcn_readfirstlane(j);      // lane 0 is the first active lane
    };
    int k = claim();
    const int ctot = __builtin_amdgcn_readfirstlane(s_ctot[b]);   // the pair's candidates, in an SGPR
    if (k < k1) load_rows(b, k, ctot);
#pragma unroll 1
    while (k < k1) {
#ifdef SFM_MF_STAMPS
      mf_acc_[7] += 1;
#endif
      const int c0 = k * kKC;
      uint32_t s1[16], s2[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) { s1[g] = 0u; s2[g] = 0u; }
#if SFM_MF2_EARLY_CLAIM
      // the next run's claim flies during this run's tile loop
      int jn = 0;
      if (mf2_lane() == 0) jn = atomicAdd(&s_claim, 1);
#endif
      {
#if SFM_MF2_WAVES > 12
        // four waves per SIMD (128 VGPRs): one accumulator set, the B
        // fragments one tile ahead; the other waves cover the MFMA latency
        if (kMf2Fold) {
          // one register set; the other three waves of the SIMD cover the
          // a -> aa -> z -> signs dependency chain
          const mf_half8 NL = -AL, NH = -AH;
#pragma unroll 1
          for (int t = 0; t < kMf2Tiles; ++t) {
            const mf_float16 a = mf2_a(mf2_load_ab(fr + (size_t)t * kTileHalves, mf2_lane()), A1, A2);
            const MfZ z = mf2_z(mf2_load_d(fr + (size_t)t * kTileHalves, mf2_lane()), NL, NH, a);
            mf2_signs(z, s1, s2);
          }
        } else {
        MfB bn = mf_load_b(fr, mf2_lane());
#pragma unroll 1
        for (int t = 0; t < kMf2Tiles; ++t) {
          const MfB bc = bn;
          if (t + 1 < kMf2Tiles) bn = mf_load_b(fr + (size_t)(t + 1) * kTileHalves, mf2_lane());
          const MfAcc r = mf_tile_mfma(bc, A1, A2, AL, AH);
          mf2_decide(r, s1, s2);
        }
        }
#else
        if (kMf2Fold) {
          // step t: a(t+1) MFMAs, aa(t) -> z(t) MFMAs, sign bits of z(t-1)
          // (step 0 and the last step peeled; pairs of steps ping-pong the
          // a / z register sets)
          const mf_half8 NL = -AL, NH = -AH;
#if SFM_MF2_BPRE
          // B fragments one step ahead (12 more VGPRs: the 8-wave build)
          auto ldab = [&](int t) { return mf2_load_ab(fr + (size_t)min(t, kMf2Tiles - 1) * kTileHalves, mf2_lane()); };
          auto ldd = [&](int t) { return mf2_load_d(fr + (size_t)min(t, kMf2Tiles - 1) * kTileHalves, mf2_lane()); };
          MfAB ab1 = ldab(1);
          mf_half8 d0 = ldd(0);
          mf_float16 aA = mf2_a(ldab(0), A1, A2), aB;
          MfZ zA, zB;
          aB = mf2_a(ab1, A1, A2);
          ab1 = ldab(2);
          zA = mf2_z(d0, NL, NH, aA);
          d0 = ldd(1);
#pragma unroll 1
          for (int t = 1; t < kMf2Tiles - 1; t += 2) {
            aA = mf2_a(ab1, A1, A2);                      // a(t + 1)
            ab1 = ldab(t + 2);
            zB = mf2_z(d0, NL, NH, aB);                   // z(t)
            d0 = ldd(t + 1);
            mf2_signs(zA, s1, s2);                        // t - 1
            aB = mf2_a(ab1, A1, A2);                      // a(t + 2)
            ab1 = ldab(t + 3);
            zA = mf2_z(d0, NL, NH, aA);                   // z(t + 1)
            d0 = ldd(t + 2);
            mf2_signs(zB, s1, s2);                        // t
          }
          zB = mf2_z(d0, NL, NH, aB);
          mf2_signs(zA, s1, s2);
          mf2_signs(zB, s1, s2);
        } else if (kMf2Fold) {
          const mf_half8 NL = -AL, NH = -AH;
#endif
          mf_float16 aA = mf2_a(mf2_load_ab(fr, mf2_lane()), A1, A2), aB;
          MfZ zA, zB;
          aB = mf2_a(mf2_load_ab(fr + (size_t)1 * kTileHalves, mf2_lane()), A1, A2);
          zA = mf2_z(mf2_load_d(fr, mf2_lane()), NL, NH, aA);
#pragma unroll 1
          for (int t = 1; t < kMf2Tiles - 1; t += 2) {
#if SFM_MF2_LN1
            // one lane address per two tiles: the four fragment loads use
            // immediate offsets from it (round 3 recomputed it per load)
            const int ln = mf2_lane();
#define MF2_LN ln
#else
#define MF2_LN mf2_lane()
#endif
            aA = mf2_a(mf2_load_ab(fr + (size_t)(t + 1) * kTileHalves, MF2_LN), A1, A2);
            zB = mf2_z(mf2_load_d(fr + (size_t)t * kTileHalves, MF2_LN), NL, NH, aB);
            mf2_signs(zA, s1, s2);
            aB = mf2_a(mf2_load_ab(fr + (size_t)(t + 2) * kTileHalves, MF2_LN), A1, A2);
            zA = mf2_z(mf2_load_d(fr + (size_t)(t + 1) * kTileHalves, MF2_LN), NL, NH, aA);
            mf2_signs(zB, s1, s2);
#undef MF2_LN
          }
          zB = mf2_z(mf2_load_d(fr + (size_t)(kMf2Tiles - 1) * kTileHalves, mf2_lane()), NL, NH, aB);
          mf2_signs(zA, s1, s2);
          mf2_signs(zB, s1, s2);
        } else {
        // two accumulator sets: tile t+1's MFMAs beside tile t's decisions
        // (the last pair peeled, so the loop body has no conditional MFMA)
        MfB B = mf_load_b(fr, mf2_lane());
        MfAcc ra = mf_tile_mfma(B, A1, A2, AL, AH), rb;
#pragma unroll 1
        for (int t = 0; t < kMf2Tiles - 2; t += 2) {
          B = mf_load_b(fr + (size_t)(t + 1) * kTileHalves, mf2_lane());
          rb = mf_tile_mfma(B, A1, A2, AL, AH);
          mf2_decide(ra, s1, s2);
          B = mf_load_b(fr + (size_t)(t + 2) * kTileHalves, mf2_lane());
          ra = mf_tile_mfma(B, A1, A2, AL, AH);
          mf2_decide(rb, s1, s2);
        }
        B = mf_load_b(fr + (size_t)(kMf2Tiles - 1) * kTileHalves, mf2_lane());
        rb = mf_tile_mfma(B, A1, A2, AL, AH);
        mf2_decide(ra, s1, s2);
        mf2_decide(rb, s1, s2);
        }
#endif
      }
      MF_STAMP(1);
      const int lane = mf2_lane(), hl = lane >> 5, rl = lane & 31;
      // the next run's rows load under this run's queue, drain and reduction
#if SFM_MF2_EARLY_CLAIM
      const int kn = k0 + __builtin_amdgcn_readfirstlane(jn);
#else
      const int kn = claim();
#endif
      if (!(SFM_MF2_EXP & 4) && kn < k1) load_rows(b, kn, ctot);
      MF_STAMP(6);
      // 3. undecided evaluations -> the queue -> float64.  Bit j of a string
      // is tile kMf2Tiles-1-j, point 32 (kMf2Tiles-1-j) + rl of the span.
      int nl = 0;
#if SFM_MF2_EXP & 1
      if (false)
#endif
#pragma unroll
      for (int g = 0; g < 16; ++g) nl += __popc(mf2_undecided(s1[g], s2[g]));
      const int incl = mf_wave_scan(nl, lane);
      const int qtotal = __builtin_amdgcn_readlane(incl, 63);
#ifdef SFM_MF_STATS
      if (lane == 0) {
        atomicAdd(&g_mf2_stats[0], (unsigned long long)qtotal);
        atomicAdd(&g_mf2_stats[1], (unsigned long long)kKC * kMf2Span);
      }
#endif
      const double* Erow0 = candE + ((size_t)b * cmax + c0) * kCandStride;
      for (int base = 0; base < qtotal; base += kMf2Queue) {
        int pos = incl - nl - base;
        if (qtotal <= kMf2Queue) {
          uint32_t* q = queue + pos;
#if SFM_MF2_QB
          uint32_t more = 0u;                                 // words with a second bit (rare)
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const uint32_t uu = mf2_undecided(s1[g], s2[g]);
            const uint32_t top = mf2_qbase(g, hl, rl);
            if (uu) {
              *q++ = mf2_qentry(top, uu);
              more |= (uu & (uu - 1u)) ? (1u << g) : 0u;
            }
          }
          if (__builtin_expect(__builtin_amdgcn_ballot_w64(more != 0u) != 0, 0)) {
#pragma unroll
            for (int g = 0; g < 16; ++g) {
              if (more & (1u << g)) {
                uint32_t uu = mf2_undecided(s1[g], s2[g]);
                uu &= uu - 1u;
                const uint32_t top = mf2_qbase(g, hl, rl);
                while (uu) {
                  *q++ = mf2_qentry(top, uu);
                  uu &= uu - 1u;
                }
              }
            }
          }
#else
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            uint32_t uu = mf2_undecided(s1[g], s2[g]);
            const uint32_t top = mf2_qbase(g, hl, rl);
            while (uu) {
              *q++ = mf2_qentry(top, uu);
              uu &= uu - 1u;
            }
          }
#endif
        } else {
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            uint32_t uu = mf2_undecided(s1[g], s2[g]);
            const uint32_t top = mf2_qbase(g, hl, rl);
            while (uu) {
              if (pos >= 0 && pos < kMf2Queue) queue[pos] = mf2_qentry(top, uu);
              uu &= uu - 1u;
              ++pos;
            }
          }
        }
        wave_sync();
        MF_STAMP(2);
#if SFM_MF2_GPTS
        mf2_drain_src(Erow0, src, b, p0, kc, lane, cnt, queue, min(kMf2Queue, qtotal - base));
#else
        mf2_drain(Erow0, s_pts, kc, lane, cnt, queue, min(kMf2Queue, qtotal - base));
#endif
        wave_sync();
        MF_STAMP(3);
      }
      MF_STAMP(2);
      // 4. counts: popcounts of the inlier strings over the 32 points of each half + the float64 counts
#if SFM_MF2_EXP & 2
#pragma unroll
      for (int g = 0; g < 16; ++g) exp_sink ^= s1[g] ^ s2[g];
      if (false) {
#endif
      int cT[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) cT[g] = __popc(s1[g]);
      const int sumT = mf_half_reduce(cT, lane);
      if ((lane & 1) == 0) {
        const int c = mf_row((rl >> 1) & 15, hl);
        const int d = sumT + cnt[c];
        cnt[c] = 0;
        if (d && c0 + c < ctot) {
#if SFM_MF2_TBL
          if (k < kMf2TblTiles) {
            if (SFM_MF2_TBL == 2)                             // two candidates per word: an LDS atomic
              atomicAdd(&s_tbl[(c0 + c) >> 1], d << (16 * ((c0 + c) & 1)));
            else
              s_tbl[c0 + c] += d;                             // tile k of this span is this wave's alone
          } else
#endif
            atomicAdd(cntT + (size_t)b * cmax + c0 + c, d);
        }
      }
#if SFM_MF2_EXP & 2
      }
#endif
      wave_sync();
      MF_STAMP(4);
      k = kn;
    }
    u += k1 - k0;
    lds_barrier();                                            // the span is re-staged next
    MF_STAMP(5);
  }
#if SFM_MF2_DYN
  }
#endif
#if SFM_MF2_TBL
  // (DYN: the loop left right after a block barrier; static ranges: after the
  // last span's barrier)
  if (tb >= 0) flush(tb);
#endif
#if SFM_MF2_EXP
  if (exp_sink == 0x9e3779b9u) cntT[0] = 1;                 // keeps the sinked strings live
#endif
#if SFM_MF2_DYN
  // the last block out zeroes the counters (claim[8] counts finished blocks),
  // so the workspace holds no schedule-dependent bytes after the launch
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    if (atomicAdd(claim + 8, 1ull) == (unsigned long long)G - 1ull) {
#pragma unroll
      for (int i = 0; i < 9; ++i) claim[i] = 0ull;
    }
  }
#endif
#ifdef SFM_MF_STAMPS
  if (mf2_lane() == 0)
    for (int i = 0; i < kMfStamps; ++i) atomicAdd(&g_mf_stamps[i], mf_acc_[i]);
#endif
#ifdef SFM_MF2_BLOCKT
  // experiment builds (scripts/mf2_blockt.py): each block's start and end on
  // the 100 MHz clock and its unit count, for the cross-block balance
  __syncthreads();
  if (tid == 0) {
    g_mf2_blockt[blockIdx.x * 3 + 0] = blk_t0;
    g_mf2_blockt[blockIdx.x * 3 + 1] = __builtin_amdgcn_s_memrealtime();
#if SFM_MF2_DYN
    g_mf2_blockt[blockIdx.x * 3 + 2] = (unsigned long long)units_done;
#else
    g_mf2_blockt[blockIdx.x * 3 + 2] = (unsigned long long)(u_end - u_beg);
#endif
  }
#endif
}
