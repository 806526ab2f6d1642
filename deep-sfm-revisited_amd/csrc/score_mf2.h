// Phase 3e of the RANSAC (included by ransac5.hip after score_mf.h): the
// span-major split-f16 matrix-core scorer, k_score_mf2 (default for SFMnet's
// num_test == num_ransac_test; tuning key score_mf = 2).
//
// Same arithmetic and decisions as k_score_mf (the A rows of k_mf_cands, the
// B columns of mf_stage_point, the float64 re-test of the undecided band), so
// every count is identical; what changes is how the work is laid out on the
// chip:
//
//   * Work units are (pair, 1024-point span, 32-candidate tile), ordered
//     span-major within a pair.  XCD x owns the x-th eighth of the units
//     (about one pair, whose A rows then stay in that XCD's L2) and its
//     blocks claim guided chunks of it from a global counter.  The block
//     stages a span once (B fragments + float64 points, one LDS image) and
//     its 12 waves claim the span's candidate tiles from an LDS counter; one
//     LDS barrier pair per span.
//   * The tile loop keeps the matrix pipe and the vector issue busy together
//     from one wave: a = x'^T E x (two MFMAs), aa = a * a as the accumulator
//     input of the two band MFMAs z1 = aa - Ylo, z2 = aa - Yhi, and the two
//     sign bits of each, pipelined over three tiles (48 decision VALU per
//     tile).  Spans are 32 tiles, so the 32-bit decision strings are full.
//   * The next run's A rows load right after the tile loop, under the queue /
//     drain / reduction of the current run.
//   * Counts go to a per-block LDS table (16-bit halves) flushed with one
//     global atomic per nonzero candidate when the block moves to another
//     pair or ends.
//
// Count-bound pruning (round 5, tuning key score_mf_prune): the launch can
// cover only a range of each pair's spans (sp_lo .. sp_hi, in per mille of
// the span count, or per-pair boundaries in device memory), and the
// candidates can be a compacted subset whose counts go to cntT[cmap[j]]
// (k_mf2_split / k_mf2_lead / k_mf2_keep below).
//
// Registers (gfx950, 3 waves per SIMD = 168 VGPRs): 2 x 48 accumulators + 16
// A + 12 B + 32 decision strings in the loop.  The round 2-4 schedule and
// layout variants that measured slower are described in DESIGN_HISTORY.md
// and the profiles/r0*_mf2_* A/B records; their code is gone.
constexpr int kMf2Waves = 12;                  // 3 per SIMD, two accumulator sets
constexpr int kMf2Wpe = kMf2Waves / 4;
// the one-sided pass (kUpper) holds fewer registers (z2 alone): its block
// size, waves per SIMD = SFM_MF2_UP_WAVES / 4
#ifndef SFM_MF2_UP_WAVES
#define SFM_MF2_UP_WAVES 16
#endif
template <bool kUpper> constexpr int mf2_waves() { return kUpper ? SFM_MF2_UP_WAVES : kMf2Waves; }
constexpr int kMf2Span = 1024;                 // points per staged span
constexpr int kMf2Tiles = kMf2Span / 32;       // tiles per span (every run decides all of them)
constexpr int kMf2Guide = 2;                   // a claim takes remainder / (guide x blocks per XCD)
constexpr int kMf2Queue = 128;                 // undecided entries per wave and drain window (LDS)
#ifndef SFM_MF2_WQ
#define SFM_MF2_WQ 1                           // the two-phase (word, then lane-parallel bit) queue build
#endif
constexpr int kMf2WordSlots = kMf2Queue / 2;   // word slots (two words each) of the two-phase build
// candidate tiles the LDS count table holds (tiles past it publish per run)
constexpr int kMf2TblTiles = 352;
constexpr int kMf2TblWords = kMf2TblTiles * kKC / 2;   // 16-bit counts, two per word
constexpr int kMf2TblSpans = 63;               // spans between flushes (63 x 1024 < 2^16: a half never carries)
constexpr int kMf2PruneMinSpans = 32;         // count-bound pruning only for pairs of >= 32 spans
static_assert(kMf2Span <= 1024, "16-bit table counts");
static_assert(kMf2Tiles <= 32 && kMf2Tiles % 2 == 0, "32-bit decision strings, tiles in pairs");

// the first span of a launch's range: spans * pm / 1000 (k_score_mf2 and
// k_mf2_lead / k_mf2_keep agree on it)
__host__ __device__ inline int mf2_span_at(int spans, int pm) { return (int)(((long long)spans * pm) / 1000); }
__host__ __device__ inline int mf2_spans(int points) { return (points + kMf2Span - 1) / kMf2Span; }

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
// records; through the pair's index map in a pruned launch), points from the
// staged span.
__device__ __forceinline__ void mf2_drain(const double* __restrict__ Epair, const int32_t* __restrict__ mpair,
                                          int c0, const double4* __restrict__ spts, const ScoreConsts& kc, int lane,
                                          int32_t* cnt, const uint32_t* q, int qn) {
#pragma unroll 1
  for (int i = lane; i < qn; i += 64) {
    const uint32_t e = q[i];
    const int c = (int)(e >> 24), r = (int)(e & 0xffffffu);
    const int ci = mpair ? mpair[c0 + c] : c0 + c;
    if (inlier_f64v(Epair + (size_t)ci * kCandStride, spts[r], kc)) atomicAdd(&cnt[c], 1);
  }
}

// a^2 folded into the band MFMAs (the bound: score_mf.h, kMfFoldLo /
// kMfFoldHi).  Per tile a = two MFMAs, then aa = a * a (16 VALU) becomes the
// C operand of z1 = aa - Ylo and z2 = aa - Yhi (the A rows of Ylo / Yhi
// negated once per run), and the decisions are the two sign bits alone.  s1
// holds inlier bits (z1 < 0); s2 holds NOT-outlier bits (z2 < 0), so
// undecided = s2 & ~s1.
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
__device__ __forceinline__ MfZ mf2_z(mf_half8 bd, mf_half8 NL, mf_half8 NH, const mf_float16& a) {
  mf_float16 aa;
#pragma unroll
  for (int g = 0; g < 16; ++g) aa[g] = a[g] * a[g];
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

// the upper-bound (one-sided) form: z2 alone and its sign bits
__device__ __forceinline__ mf_float16 mf2_zhi(mf_half8 bd, mf_half8 NH, const mf_float16& a) {
  mf_float16 aa;
#pragma unroll
  for (int g = 0; g < 16; ++g) aa[g] = a[g] * a[g];
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(NH, bd, aa, 0, 0, 0);
}
__device__ __forceinline__ void mf2_signs_hi(const mf_float16& z2, uint32_t (&s2)[16]) {
#pragma unroll
  for (int g = 0; g < 16; ++g) s2[g] = __builtin_amdgcn_alignbit(s2[g], __float_as_uint(z2[g]), 31);
}

// queue entry (candidate row << 24 | span-relative point) of the lowest set
// bit j of a string: bit j = tile kMf2Tiles - 1 - j
__device__ __forceinline__ uint32_t mf2_qbase(int g, int hl, int rl) {
  return ((uint32_t)mf_row(g, hl) << 24) | (uint32_t)(32 * (kMf2Tiles - 1) + rl);
}
__device__ __forceinline__ uint32_t mf2_qentry(uint32_t base, uint32_t uu) {
  return base - 32u * (uint32_t)__builtin_ctz(uu);
}
// undecided evaluations of a decision-string pair
__device__ __forceinline__ uint32_t mf2_undecided(uint32_t s1, uint32_t s2) { return s2 & ~s1; }

// the lane id, recomputed where it is used (v_mbcnt) instead of kept live
// across the tile loop, where every VGPR is taken
__device__ __forceinline__ int mf2_lane() {
  int l = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(l));
  return l;
}

// the global count slot of compacted candidate j of pair b (cmap: the
// pruned launch's index map; null: the identity)
__device__ __forceinline__ int32_t* mf2_count_slot(int32_t* cntT, const int32_t* cmap, int b, int cmax, int j) {
  const size_t i = (size_t)b * cmax + j;
  return cntT + (size_t)b * cmax + (cmap ? cmap[i] : j);
}

// kUpper (round 6): the one-sided pass of count-bound pruning -- z2 only (3
// MFMAs and 32 VALU per tile instead of 4 and 48), each count the number of
// points NOT certainly outliers (sign of z2), an upper bound on the inlier
// count; no undecided queue, no float64 drain.
template <class Src, bool kMap, bool kUpper = false>
__global__ __launch_bounds__(mf2_waves<kUpper>() * 64)
__attribute__((amdgpu_waves_per_eu(mf2_waves<kUpper>() / 4, mf2_waves<kUpper>() / 4))) void k_score_mf2(
    const Src src, PairParams pp, int batch, int cmax, const int32_t* __restrict__ cand_total,
    const double* __restrict__ candE, const _Float16* __restrict__ candF, int32_t* __restrict__ cntT,
    ScoreConsts kc, unsigned long long* __restrict__ claim, const int32_t* __restrict__ cmap_arg, int sp_lo,
    int sp_hi, const int32_t* __restrict__ bnd, int phase, int min_chunk) {
  // one count array: this kernel runs only when num_test == num_ransac_test,
  // so the preselection count is the score and k_select reads cntT for both
  __shared__ __attribute__((aligned(16))) _Float16 s_frag[kMf2Tiles][3][64][8];
  __shared__ double4 s_pts[kMf2Span];
  __shared__ int32_t s_tbl[kMf2TblWords];                    // the block's counts of pair tb's candidates
  constexpr int NW = mf2_waves<kUpper>();
  __shared__ uint32_t s_queue[kUpper ? 1 : NW][kMf2Queue];   // (the one-sided pass: neither queue nor drain)
  __shared__ int32_t s_cnt[kUpper ? 1 : NW][kKC];           // float64 drain counts
  __shared__ long long s_first[SFM_MAX_BATCH + 1];           // first unit of each pair
  __shared__ int32_t s_tiles[SFM_MAX_BATCH];                 // candidate tiles per pair
  __shared__ int32_t s_ctot[SFM_MAX_BATCH];
  __shared__ int32_t s_span0[SFM_MAX_BATCH];                 // the pair's first span in this launch
  __shared__ int32_t s_claim;                                // next candidate tile of the span to claim
  __shared__ long long s_range[2];                           // the block's current unit range
  // the compacted candidates' index map: a compile-time null in the launches
  // without one, so that its address arithmetic costs the tile loop no registers
  const int32_t* __restrict__ const cmap = kMap ? cmap_arg : nullptr;
  const int tid = threadIdx.x, wv = tid >> 6;
  if (tid == 0) {
    long long acc = 0;
    for (int b = 0; b < batch; ++b) {
      const int ct = cand_total[b];
      const int tiles = (ct + kKC - 1) / kKC;
      const int all = mf2_spans(max(pp.test[b], pp.rtest[b]));
      // the launch's spans: per mille of the pair's spans, or (bnd) the span
      // boundaries phase and phase + 1 that k_mf2_split chose for the pair
      const int s0 = bnd ? bnd[phase * SFM_MAX_BATCH + b] : mf2_span_at(all, sp_lo);
      const int s1 = bnd ? bnd[(phase + 1) * SFM_MAX_BATCH + b] : mf2_span_at(all, sp_hi);
      s_first[b] = acc;
      s_tiles[b] = tiles;
      s_ctot[b] = ct;
      s_span0[b] = s0;
      acc += (long long)(s1 - s0) * tiles;
    }
    s_first[batch] = acc;
  }
  __syncthreads();
  // nothing to score (the one-sided pruning's matrix-core pass when every
  // pair's kept candidates went to k_mf2_exact): out before the table set-up.
  // No block claims a unit, so the counters stay as the last launch left them.
  if (s_first[batch] == 0) return;
  for (int i = tid; i < (kUpper ? 1 : NW) * kKC; i += NW * 64) (&s_cnt[0][0])[i] = 0;
  for (int i = tid; i < kMf2TblWords; i += NW * 64) s_tbl[i] = 0;
  int tb = -1;                                               // the pair the table holds (block-uniform)
  int tspans = 0;                                            // spans added since the last flush
  // the table to pair fb's global counts (all threads, between block barriers)
  auto flush = [&](int fb) {
    const int nt = min(s_tiles[fb], kMf2TblTiles) * kKC;
    for (int i = tid; i < nt / 2; i += NW * 64) {
      const uint32_t v = (uint32_t)s_tbl[i];
      if (v) {
        if (v & 0xffffu) atomicAdd(mf2_count_slot(cntT, cmap, fb, cmax, 2 * i), (int)(v & 0xffffu));
        if (v >> 16) atomicAdd(mf2_count_slot(cntT, cmap, fb, cmax, 2 * i + 1), (int)(v >> 16));
        s_tbl[i] = 0;
      }
    }
  };
  __syncthreads();
  // Unit ranges: workgroup ids are dealt round-robin over the 8 XCDs, so
  // id % 8 names the XCD.  XCD x owns the x-th eighth of the units and its
  // blocks claim guided chunks of it from a global counter (half the
  // remainder's per-block share, at least min_chunk units); a block whose
  // eighth is exhausted takes chunks of the next XCDs' eighths.  Static
  // contiguous ranges left blocks idle for 6 % of the launch on average
  // (round 3): units cost unequal time across pairs and XCDs.
  const int G = gridDim.x;
  const long long U = s_first[batch];
  const int nx = (G % 8 == 0) ? 8 : 1;
  const int xcd = (int)(blockIdx.x % (unsigned)nx);
  const int per_x = G / nx;
  int victim = 0;                                            // XCDs after our own already drained
  int32_t* cnt = s_cnt[kUpper ? 0 : wv];
  uint32_t* queue = s_queue[kUpper ? 0 : wv];
  const _Float16* fr = &s_frag[0][0][0][0];
  constexpr int kTileHalves = 3 * 64 * 8;
  int b = 0;
  mf_half8 A1, A2, AL, AH;
  // A rows of candidate tile k of pair b (absent rows: every evaluation a decided outlier)
  auto load_rows = [&](int bb, int k, int ctot) {
    const int ln = mf2_lane();
    const int lh = ln >> 5, lr = ln & 31;
    const int c = k * kKC + lr;
    if (c < ctot) {
      const int ci = cmap ? cmap[(size_t)bb * cmax + c] : c;
      const mf_half8* rec = reinterpret_cast<const mf_half8*>(candF + ((size_t)bb * cmax + ci) * kMfRec);
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
  for (;;) {
    if (tid == 0) {
      long long st = U, en = U;
      for (; victim < nx; ++victim) {
        const int x = (xcd + victim) % nx;
        const long long seg_beg = U * x / nx, seg_end = U * (x + 1) / nx;
        // the floor never exceeds a block's static share of the eighth (small
        // launches, e.g. 2,048 keypoints: a 128-unit floor would idle most blocks)
        const long long floor_c = max(min((long long)min_chunk, (seg_end - seg_beg + per_x - 1) / per_x), 1ll);
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
      }
      s_range[0] = st;
      s_range[1] = en;
    }
    __syncthreads();
    long long u = s_range[0];
    const long long u_end = s_range[1];
    if (u >= u_end) break;
    if (u < s_first[b]) b = 0;                               // a stolen chunk may lie before our own
    while (u < u_end) {
      while (u >= s_first[b + 1]) ++b;
      b = __builtin_amdgcn_readfirstlane(b);
      const int tiles = s_tiles[b];
      const long long local = u - s_first[b];
      const int span_l = (int)(local / tiles);
      const int k0 = (int)(local - (long long)span_l * tiles);
      const int k1 = (int)min((long long)tiles, (long long)k0 + (u_end - u));   // this block's tiles of the span
      const int p0 = (s_span0[b] + span_l) * kMf2Span;
      const int np = min(max(pp.test[b], pp.rtest[b]) - p0, kMf2Span);     // live points of the span
      // a new pair: the table's counts go out first (every wave's adds to it
      // ended before the barrier that closed the previous span or claim)
      if (b != tb || tspans == kMf2TblSpans) {
        if (tb >= 0) flush(tb);
        tb = b;
        tspans = 0;
      }
      ++tspans;
      // 1. stage the span: B fragments for every slot (dead slots: the decided-outlier sentinel)
      if (tid == 0) s_claim = 0;
      for (int i = tid; i < kMf2Span; i += NW * 64) {
        const bool live = i < np;
        const double4 v = src.load(b, live ? p0 + i : p0);
        if constexpr (!kUpper) s_pts[i] = v;                 // (the float64 points serve the drain only)
        mf_stage_point(v, live, &s_frag[i >> 5][0][0][0], i & 31);
      }
      lds_barrier();
      // 2. the span's candidate tiles, claimed one run at a time from an LDS
      // counter: the three waves of a SIMD progress at very different rates
      // (issue arbitration favours the oldest), so a static split left the
      // younger waves' tail for the others to wait out at the span barrier
      auto claim_tile = [&]() {
        int j = 0;
        if (mf2_lane() == 0) j = atomicAdd(&s_claim, 1);
        return k0 + __builtin_amdgcn_readfirstlane(j);      // lane 0 is the first active lane
      };
      int k = claim_tile();
      const int ctot = __builtin_amdgcn_readfirstlane(s_ctot[b]);   // the pair's candidates, in an SGPR
      if (k < k1) load_rows(b, k, ctot);
#pragma unroll 1
      while (k < k1) {
        const int c0 = k * kKC;
        uint32_t s1[16], s2[16];
#pragma unroll
        for (int g = 0; g < 16; ++g) { s1[g] = 0u; s2[g] = 0u; }
        if constexpr (kUpper) {
          // the same pipeline with z2 alone: a(t+1) MFMAs, z2(t), sign bits of z2(t-1)
          const mf_half8 NH = -AH;
          mf_float16 aA = mf2_a(mf2_load_ab(fr, mf2_lane()), A1, A2), aB;
          mf_float16 zA, zB;
          aB = mf2_a(mf2_load_ab(fr + (size_t)1 * kTileHalves, mf2_lane()), A1, A2);
          zA = mf2_zhi(mf2_load_d(fr, mf2_lane()), NH, aA);
#pragma unroll 1
          for (int t = 1; t < kMf2Tiles - 1; t += 2) {
            const _Float16* lp = fr + (size_t)t * kTileHalves + (size_t)mf2_lane() * 8;
            aA = mf2_a(mf2_load_ab(lp + kTileHalves, 0), A1, A2);
            zB = mf2_zhi(mf2_load_d(lp, 0), NH, aB);
            mf2_signs_hi(zA, s2);
            aB = mf2_a(mf2_load_ab(lp + 2 * kTileHalves, 0), A1, A2);
            zA = mf2_zhi(mf2_load_d(lp + kTileHalves, 0), NH, aA);
            mf2_signs_hi(zB, s2);
          }
          zB = mf2_zhi(mf2_load_d(fr + (size_t)(kMf2Tiles - 1) * kTileHalves, mf2_lane()), NH, aB);
          mf2_signs_hi(zA, s2);
          mf2_signs_hi(zB, s2);
        } else {
          // step t: a(t+1) MFMAs, aa(t) -> z(t) MFMAs, sign bits of z(t-1)
          // (step 0 and the last step peeled; pairs of steps ping-pong the
          // a / z register sets)
          const mf_half8 NL = -AL, NH = -AH;
          mf_float16 aA = mf2_a(mf2_load_ab(fr, mf2_lane()), A1, A2), aB;
          MfZ zA, zB;
          aB = mf2_a(mf2_load_ab(fr + (size_t)1 * kTileHalves, mf2_lane()), A1, A2);
          zA = mf2_z(mf2_load_d(fr, mf2_lane()), NL, NH, aA);
#pragma unroll 1
          for (int t = 1; t < kMf2Tiles - 1; t += 2) {
            // one lane address per two tiles: the six fragment reads of the
            // step are immediate offsets from it (round 5: 98 instead of 104
            // VALU per two tiles, the scorer 0.8 - 1.3 % faster in three
            // alternating rounds, profiles/r05_mf2_lane_ptr_ab.txt)
            const _Float16* lp = fr + (size_t)t * kTileHalves + (size_t)mf2_lane() * 8;
            aA = mf2_a(mf2_load_ab(lp + kTileHalves, 0), A1, A2);
            zB = mf2_z(mf2_load_d(lp, 0), NL, NH, aB);
            mf2_signs(zA, s1, s2);
            aB = mf2_a(mf2_load_ab(lp + 2 * kTileHalves, 0), A1, A2);
            zA = mf2_z(mf2_load_d(lp + kTileHalves, 0), NL, NH, aA);
            mf2_signs(zB, s1, s2);
          }
          zB = mf2_z(mf2_load_d(fr + (size_t)(kMf2Tiles - 1) * kTileHalves, mf2_lane()), NL, NH, aB);
          mf2_signs(zA, s1, s2);
          mf2_signs(zB, s1, s2);
        }
        const int lane = mf2_lane(), hl = lane >> 5, rl = lane & 31;
        // the next run's rows load under this run's queue, drain and reduction
        const int kn = claim_tile();
        if (kn < k1) load_rows(b, kn, ctot);
        if constexpr (kUpper) {
          // not-certain-outlier bits are the count: s1 := s2, nothing undecided
#pragma unroll
          for (int g = 0; g < 16; ++g) s1[g] = s2[g];
        } else {
        // 3. undecided evaluations -> the queue -> float64.  Bit j of a string
        // is tile kMf2Tiles-1-j, point 32 (kMf2Tiles-1-j) + rl of the span.
        int nl = 0;
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
        const double* Epair = candE + (size_t)b * cmax * kCandStride;
        const int32_t* mpair = cmap ? cmap + (size_t)b * cmax : nullptr;
#if SFM_MF2_WQ
        if (qtotal <= kMf2WordSlots) {
          // Two-phase build (round 6): (1) every lane appends its non-empty
          // undecided words as (word, entry base) pairs -- no per-bit loop --
          // at its first bit's queue position (the wave scan of the bit
          // counts), leaving a hole for each further bit; (2) lane i expands
          // the word at slot i, if any, into entries i, i+1, ... (lane-parallel:
          // the per-bit loop runs as many times as the fullest word has bits).
          uint32_t* qw = queue;                              // 64 slots of two words, then 4-byte entries
          qw[2 * lane] = 0u;                                 // holes: an empty word
          int pos = incl - nl;
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const uint32_t uu = mf2_undecided(s1[g], s2[g]);
            if (uu) {
              qw[2 * pos] = uu;
              qw[2 * pos + 1] = mf2_qbase(g, hl, rl);
              pos += __popc(uu);
            }
          }
          wave_sync();
          uint32_t uu = qw[2 * lane];
          const uint32_t top = qw[2 * lane + 1];
          wave_sync();                                       // every slot read before the entries overwrite them
          for (int p = lane; uu; ++p) {
            qw[p] = mf2_qentry(top, uu);
            uu &= uu - 1u;
          }
          wave_sync();
          mf2_drain(Epair, mpair, c0, s_pts, kc, lane, cnt, queue, qtotal);
          wave_sync();
        } else
#endif
        for (int base = 0; base < qtotal; base += kMf2Queue) {
          int pos = incl - nl - base;
          if (qtotal <= kMf2Queue) {
            uint32_t* q = queue + pos;
#pragma unroll
            for (int g = 0; g < 16; ++g) {
              uint32_t uu = mf2_undecided(s1[g], s2[g]);
              const uint32_t top = mf2_qbase(g, hl, rl);
              while (uu) {
                *q++ = mf2_qentry(top, uu);
                uu &= uu - 1u;
              }
            }
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
          mf2_drain(Epair, mpair, c0, s_pts, kc, lane, cnt, queue, min(kMf2Queue, qtotal - base));
          wave_sync();
        }
        }
        // 4. counts: popcounts of the inlier strings over the 32 points of each half + the float64 counts
        int cT[16];
#pragma unroll
        for (int g = 0; g < 16; ++g) cT[g] = __popc(s1[g]);
        const int sumT = mf_half_reduce(cT, lane);
        if ((lane & 1) == 0) {
          const int c = mf_row((rl >> 1) & 15, hl);
          const int d = sumT + cnt[c];
          cnt[c] = 0;
          if (d && c0 + c < ctot) {
            if (k < kMf2TblTiles)                             // two candidates per word: an LDS atomic
              atomicAdd(&s_tbl[(c0 + c) >> 1], d << (16 * ((c0 + c) & 1)));
            else
              atomicAdd(mf2_count_slot(cntT, cmap, b, cmax, c0 + c), d);
          }
        }
        wave_sync();
        k = kn;
      }
      u += k1 - k0;
      lds_barrier();                                          // the span is re-staged next
    }
  }
  // (the loop left right after a block barrier)
  if (tb >= 0) flush(tb);
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
}

// Count-bound pruning (tuning key score_mf_prune = pm; only for SFMnet's
// num_test == num_ransac_test without per-hypothesis scores).  Launches A
// and B score every candidate of pair b on its first n1 points (spans [0,
// sB), k_mf2_split above); then
//   k_mf2_lead  (kLeadBlocks blocks per pair) takes the leader, the first
//               candidate with the largest partial count, and counts its
//               inliers on the remaining points [n1, M) with the exact
//               float64 test (inlier_f64v, the drain's), each block a slice:
//               lb = partial + rest is the leader's final count, a lower
//               bound on the pair's winning count;
//   k_mf2_keep  (one block per 1024 candidates) keeps candidate c iff its
//               bound (M - n1) + count(c) -- every point not yet scored an
//               inlier -- is >= lb, writing the kept indices to cmap in
//               candidate order (each block counts the kept candidates
//               before its own range for its offset).
// The second launch scores the kept candidates on the remaining spans.  A
// dropped candidate's true count is < lb <= the winning count, so it can be
// neither a winner nor tie one: every candidate that reaches the winning
// count is kept and counted exactly, and k_select's first-max choices
// (within each hypothesis, then over hypotheses) are unchanged.  The counts
// of dropped candidates stay partial (lower
// than their true counts), which is why pruning is off when per-hypothesis
// scores are requested.  `skipped` gains (dropped candidates) x (M - n1).
// lead[k * SFM_MAX_BATCH + b], k = 0: partial count of the leader, 1: its
// index, 2: its rest count (zeroed by k_mf_cands at the start of the scoring
// phase), 3: kept candidates (the second launch's cand_total).
constexpr int kLeadBlocks = 32;
constexpr int kExactMaxKept = 256;   // kept candidates per pair k_mf2_exact can count (score_mf_exact_max)

// the points the launches before the pruning scored: spans [0, bnd[2][b])
__device__ __forceinline__ int mf2_n1(const PairParams& pp, int b, const int32_t* bnd) {
  const int M = max(pp.test[b], pp.rtest[b]);
  return min(bnd[2 * SFM_MAX_BATCH + b] * kMf2Span, M);
}

// k_mf2_split (one block per pair), after the first launch (spans [0, sA),
// sA = spans * pm / 1000): the pair's inlier ratio estimated from its largest
// partial count, rho = max_c count(c) / nA, sets where the pruning happens.
// A candidate with inlier ratio r can only be dropped after a share f of the
// points with f (1 - r) > 1 - rho (its outliers so far must exceed every
// point the winner does not hold), so the pruning point is f = 1 - rho +
// margin (per mille; at least pm, and no pruning -- all spans before it --
// when f would pass 990): 0.88 on the KITTI bench pairs (rho ~ 0.145), 0.92
// on the indoor ones (rho ~ 0.105), where the fixed 0.88 of the first round-5
// build could drop nothing and cost an extra launch boundary.  Writes the
// boundaries bnd[0..3][b] = 0, sA, sB, spans for the launches A [0, sA), B
// [sA, sB) (every candidate) and, after k_mf2_lead / k_mf2_keep at sB, C
// [sB, spans) (the kept candidates).
// (The one-sided pruning of round 6 runs it with pm = 1000: its pruning point
// is the end of the pair, sA = sB = spans.)
// leader (the one-sided pruning, counts final): also the leader -- the first
// candidate with the largest count, as k_mf2_lead picks it -- into lead rows
// 0 (0: the partial count of a full count) and 1 (its index).
__global__ __launch_bounds__(1024) void k_mf2_split(PairParams pp, int cmax, int pm, int margin,
                                                   const int32_t* __restrict__ cand_total,
                                                   const int32_t* __restrict__ cntT, int32_t* __restrict__ bnd,
                                                   int32_t* __restrict__ leader) {
  __shared__ unsigned long long s_key[16];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = max(pp.test[b], pp.rtest[b]);
  const int all = mf2_spans(M);
  const int sA = mf2_span_at(all, pm);
  const int nA = min(sA * kMf2Span, M);
  const int ctot = cand_total[b];
  const int32_t* cnt = cntT + (size_t)b * cmax;
  // key = count << 32 | ~c: the max is the first of the largest
  unsigned long long key = 0ull;
  for (int c = tid; c < ctot; c += 1024) {
    const unsigned long long k = ((unsigned long long)(uint32_t)cnt[c] << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)c);
    key = k > key ? k : key;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(key, d, 64);
    key = o > key ? o : key;
  }
  if (lane == 0) s_key[wv] = key;
  __syncthreads();
  if (tid != 0) return;
  for (int w = 0; w < 16; ++w) key = s_key[w] > key ? s_key[w] : key;
  int mx = (int)(key >> 32);
  if (leader && ctot > 0) {
    leader[0 * SFM_MAX_BATCH + b] = 0;
    leader[1 * SFM_MAX_BATCH + b] = (int)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
  }
  // f = 1 - rho + margin in per mille, rounded up; >= pm; > 990: no pruning
  const long long rho_pm = nA > 0 ? ((long long)mx * 1000) / nA : 0;
  long long f = 1000 - rho_pm + margin;
  f = max(f, (long long)pm);
  const int sB = f > 990 ? all : max(sA, mf2_span_at(all, (int)f));
  bnd[0 * SFM_MAX_BATCH + b] = 0;
  bnd[1 * SFM_MAX_BATCH + b] = sA;
  bnd[2 * SFM_MAX_BATCH + b] = sB;
  bnd[3 * SFM_MAX_BATCH + b] = all;
}

// full (the one-sided pruning of round 6, whose counts are upper bounds):
// the leader's exact count over every point [0, M), its partial count
// recorded as 0, so that lb = lead[0] + lead[2] is still its exact count.
template <class Src>
__global__ __launch_bounds__(1024) void k_mf2_lead(const Src src, PairParams pp, int cmax, const int32_t* __restrict__ bnd,
                                                  const int32_t* __restrict__ cand_total,
                                                  const double* __restrict__ candE, const int32_t* __restrict__ cntT,
                                                  ScoreConsts kc, int32_t* __restrict__ lead, int full) {
  __shared__ unsigned long long s_key[16];
  __shared__ int s_part[16];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int M = max(pp.test[b], pp.rtest[b]);
  const int n1 = full ? 0 : mf2_n1(pp, b, bnd);
  const int ctot = cand_total[b];
  if (ctot <= 0) return;
  const int32_t* cnt = cntT + (size_t)b * cmax;
  if (full == 2) {
    // the leader from k_mf2_split (lead rows 0 / 1): its exact count alone
    const int ldr = lead[1 * SFM_MAX_BATCH + b];
    const int k0 = (int)((long long)M * blockIdx.x / gridDim.x);
    const int k1 = (int)((long long)M * (blockIdx.x + 1) / gridDim.x);
    const double* El = candE + ((size_t)b * cmax + ldr) * kCandStride;
    int r = 0;
    const int T = (int)blockDim.x;
    for (int k = k0 + tid; k < k1; k += 2 * T) {             // two independent chains per pass
      const bool ob = k + T < k1;
      const double4 va = src.load(b, k), vb = src.load(b, ob ? k + T : k);
      r += inlier_f64v(El, va, kc) ? 1 : 0;
      r += (ob && inlier_f64v(El, vb, kc)) ? 1 : 0;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) r += __shfl_xor(r, d, 64);
    if (lane == 0) s_part[wv] = r;
    __syncthreads();
    if (tid == 0) {                                          // one global atomic per block
      int t = 0;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += s_part[w];
      if (t) atomicAdd(&lead[2 * SFM_MAX_BATCH + b], t);
    }
    return;
  }
  // the leader (key count << 32 | ~c: the first of the largest); every block
  // finds the same one
  unsigned long long key = 0ull;
  for (int c = tid; c < ctot; c += 1024) {
    const unsigned long long k = ((unsigned long long)(uint32_t)cnt[c] << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)c);
    key = k > key ? k : key;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const unsigned long long o = __shfl_xor(key, d, 64);
    key = o > key ? o : key;
  }
  if (lane == 0) s_key[wv] = key;
  __syncthreads();
  key = s_key[0];
  for (int w = 1; w < 16; ++w) key = s_key[w] > key ? s_key[w] : key;
  const int ld = (int)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
  // this block's slice of the points the first launch did not score
  const int rest_n = M - n1;
  const int k0 = n1 + (int)((long long)rest_n * blockIdx.x / gridDim.x);
  const int k1 = n1 + (int)((long long)rest_n * (blockIdx.x + 1) / gridDim.x);
  const double* El = candE + ((size_t)b * cmax + ld) * kCandStride;
  int rest = 0;
  for (int k = k0 + tid; k < k1; k += 1024) rest += inlier_f64v(El, src.load(b, k), kc) ? 1 : 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) rest += __shfl_xor(rest, d, 64);
  if (lane == 0) s_part[wv] = rest;
  __syncthreads();
  if (tid == 0) {
    int r = 0;
    for (int w = 0; w < 16; ++w) r += s_part[w];
    if (blockIdx.x == 0) {
      lead[0 * SFM_MAX_BATCH + b] = full ? 0 : (int)(key >> 32);
      lead[1 * SFM_MAX_BATCH + b] = ld;
    }
    if (r) atomicAdd(&lead[2 * SFM_MAX_BATCH + b], r);
  }
}

__global__ __launch_bounds__(1024) void k_mf2_keep(PairParams pp, int cmax, const int32_t* __restrict__ bnd,
                                                  const int32_t* __restrict__ cand_total,
                                                  const int32_t* __restrict__ cntT, int32_t* __restrict__ lead,
                                                  int32_t* __restrict__ cmap, unsigned long long* __restrict__ skipped,
                                                  int exact_max) {
  __shared__ int s_part[16];
  __shared__ int s_before[16];
  const int b = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ctot = cand_total[b];
  const int c0 = blockIdx.x * 1024;
  if (c0 >= ctot) return;
  const int M = max(pp.test[b], pp.rtest[b]);
  const int n1 = mf2_n1(pp, b, bnd);
  const long long lb = (long long)lead[0 * SFM_MAX_BATCH + b] + lead[2 * SFM_MAX_BATCH + b];
  const int32_t* cnt = cntT + (size_t)b * cmax;
  auto kept = [&](int c) { return (long long)(M - n1) + cnt[c] >= lb; };
  // this block's offset: the kept candidates before c0, counted here (a
  // deterministic order, so the workspace holds no schedule-dependent bytes)
  int before = 0;
  for (int c = tid; c < c0; c += 1024) before += kept(c) ? 1 : 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) before += __shfl_xor(before, d, 64);
  const int c = c0 + tid;
  const bool keep = c < ctot && kept(c);
  const unsigned long long bal = __ballot(keep);
  if (lane == 0) {
    s_part[wv] = __popcll(bal);
    s_before[wv] = before;
  }
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < 16; ++w) {
    base += s_before[w];
    tot += s_part[w];
  }
  if (keep) {
    int off = base + __popcll(bal & ((1ull << lane) - 1ull));
    for (int w = 0; w < wv; ++w) off += s_part[w];
    cmap[(size_t)b * cmax + off] = c;
  }
  if (tid == 0) {
    if (c0 + 1024 >= ctot) {                                  // the last block: the kept count
      lead[3 * SFM_MAX_BATCH + b] = base + tot;
      // the one-sided pruning: a pair with more kept candidates than the
      // float64 kernel takes goes to the two-sided matrix-core pass
      lead[4 * SFM_MAX_BATCH + b] = base + tot > exact_max ? base + tot : 0;
    }
    const int live = min(1024, ctot - c0);
    if (skipped && live > tot)
      atomicAdd(skipped, (unsigned long long)(live - tot) * (unsigned long long)(M - n1));
  }
}

// k_mf2_exact (the one-sided pruning, after k_mf2_zero_kept): the kept
// candidates' exact counts over every point with the drain's float64 test,
// for pairs with at most kExactMaxKept of them (the others: k_score_mf2 over
// every span through the index map).  Block (x, b) takes the x-th slice of
// pair b's points; every wave tests its points against each kept candidate in
// turn (E through uniform loads), the count of the wave's inliers goes to an
// LDS table by one lane, the table to cntT once per block.
constexpr int kExactBlocks = 128;    // blocks per pair
constexpr int kExactThreads = 1024;  // (latency-bound: every point a dependent float64 chain)

template <class Src>
__global__ __launch_bounds__(kExactThreads) void k_mf2_exact(const Src src, PairParams pp, int cmax,
                                                   const int32_t* __restrict__ lead, const int32_t* __restrict__ cmap,
                                                   const double* __restrict__ candE, ScoreConsts kc,
                                                   int32_t* __restrict__ cntT, int exact_max) {
  __shared__ int32_t s_cnt[kExactMaxKept];
  __shared__ double s_E[kExactMaxKept][10];                   // the kept candidates' E and guard constant
  const int b = blockIdx.y, tid = threadIdx.x;
  const int kept = lead[3 * SFM_MAX_BATCH + b];
  if (kept <= 0 || kept > exact_max) return;
  const int32_t* mp = cmap + (size_t)b * cmax;
  const double* Eb = candE + (size_t)b * cmax * kCandStride;
  for (int c = tid; c < kept; c += kExactThreads) s_cnt[c] = 0;
  for (int i = tid; i < kept * 10; i += kExactThreads) s_E[i / 10][i % 10] = Eb[(size_t)mp[i / 10] * kCandStride + i % 10];
  __syncthreads();
  const int M = max(pp.test[b], pp.rtest[b]);
  const int k0 = (int)((long long)M * blockIdx.x / gridDim.x);
  const int k1 = (int)((long long)M * (blockIdx.x + 1) / gridDim.x);
  const int lane = tid & 63;
  // two points per thread and pass (two independent float64 chains in
  // flight); the block's loop is uniform, so every lane takes part in the
  // ballots and lane 0 publishes
  for (int base = k0; base < k1; base += 2 * kExactThreads) {
    const int ka = base + tid, kb = base + kExactThreads + tid;
    const bool oa = ka < k1, ob = kb < k1;
    const double4 va = src.load(b, oa ? ka : k0), vb = src.load(b, ob ? kb : k0);
#pragma unroll 1
    for (int j = 0; j < kept; ++j) {
      const bool ia = inlier_f64v(&s_E[j][0], va, kc), ib = inlier_f64v(&s_E[j][0], vb, kc);
      const int n = (int)__popcll(__ballot(oa && ia)) + (int)__popcll(__ballot(ob && ib));
      if (lane == 0 && n) atomicAdd(&s_cnt[j], n);
    }
  }
  __syncthreads();
  for (int c = tid; c < kept; c += kExactThreads)
    if (s_cnt[c]) atomicAdd(cntT + (size_t)b * cmax + mp[c], s_cnt[c]);
}

// The one-sided pruning's second keep: of the candidates k_mf2_keep kept
// (cmap_in, lead row 3), those whose upper count -- now over every point --
// still reaches lb, compacted in order into cmap_out; lead rows 3 / 4 become
// their count (row 4: 0 when k_mf2_exact takes them).  One block per pair.
__global__ __launch_bounds__(1024) void k_mf2_keep_map(int cmax, const int32_t* __restrict__ cntT,
                                                      int32_t* __restrict__ lead, const int32_t* __restrict__ cmap_in,
                                                      int32_t* __restrict__ cmap_out, int exact_max) {
  __shared__ int s_part[16];
  __shared__ int s_base;
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = lead[3 * SFM_MAX_BATCH + b];
  const long long lb = (long long)lead[0 * SFM_MAX_BATCH + b] + lead[2 * SFM_MAX_BATCH + b];
  const int32_t* cnt = cntT + (size_t)b * cmax;
  const int32_t* in = cmap_in + (size_t)b * cmax;
  int32_t* out = cmap_out + (size_t)b * cmax;
  if (tid == 0) s_base = 0;
  __syncthreads();
  for (int j0 = 0; j0 < n; j0 += 1024) {
    const int j = j0 + tid;
    const int c = j < n ? in[j] : 0;
    const bool keep = j < n && (long long)cnt[c] >= lb;
    const unsigned long long bal = __ballot(keep);
    if (lane == 0) s_part[wv] = __popcll(bal);
    __syncthreads();
    int off = s_base + __popcll(bal & ((1ull << lane) - 1ull));
    for (int w = 0; w < wv; ++w) off += s_part[w];
    if (keep) out[off] = c;
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int w = 0; w < 16; ++w) t += s_part[w];
      s_base += t;
    }
    __syncthreads();
  }
  if (tid == 0) {
    lead[3 * SFM_MAX_BATCH + b] = s_base;
    lead[4 * SFM_MAX_BATCH + b] = s_base > exact_max ? s_base : 0;
  }
}

// After k_mf2_keep in the one-sided pruning: the kept candidates' (upper
// bound) counts are zeroed, so that the two-sided launch over every span
// leaves their exact counts in cntT (a separate launch: k_mf2_keep's blocks
// read every count below their range while they run).
__global__ __launch_bounds__(256) void k_mf2_zero_kept(int cmax, const int32_t* __restrict__ lead,
                                                      const int32_t* __restrict__ cmap, int32_t* __restrict__ cntT) {
  const int b = blockIdx.y;
  const int j = (int)(blockIdx.x * 256 + threadIdx.x);
  if (j < lead[3 * SFM_MAX_BATCH + b]) cntT[(size_t)b * cmax + cmap[(size_t)b * cmax + j]] = 0;
}
