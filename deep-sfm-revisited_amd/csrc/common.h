// Internal helpers shared by the libsfm_hip translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "sfm_hip.h"

namespace sfm {

void set_error(const std::string& msg);

// Launch-shape tuning knobs (sfm_tune_set); read by the launchers.
struct Tuning {
  int solve_lanes = 16;          // active lanes per k_solve_front wave (1..16: LDS records)
  int solve_coop = 1;            // k_solve_front's reduction on DPP quads (4 lanes per hypothesis); 0: one lane
  int roots_lanes = 32;          // active lanes per k_roots wave (1..32: LDS stack columns)
  int roots_split = 1;           // 1: k_roots_split (per-wave task pool); 2: k_roots_split<4> (a block's 4 waves, slower); 0: k_roots
  int sweep_items_per_block = 4; // consecutive (row, plane, window) items per sweep block
  int sweep_lane_pixels = 0;     // 1: warped lanes own 4 consecutive pixels (16-byte stores)
  int sweep_flat = 2;            // 1: 256-byte-aligned slab windows (k_sweep_flat); 2: narrow windows (k_sweep_tile); 0: per-row
  int sweep_nj = 1;              // k_sweep_tile (sweep_flat = 2): pixels per lane, window 256 * nj (bf16: even)
  int sweep_group = 8;           // warped channels per k_sweep_flat item (4 or 8; 8 measured stable in the bench loop)
  int sweep_buffer = 1;          // k_sweep_tile: buffer-addressed fast path for interior full-group windows
  int sweep_share = 0;           // k_sweep_tile fast path: right-hand taps from the next lane's left-hand taps (DPP)
  int sweep_store_wt = -1;       // 16-byte sweep stores' cache policy: 0 by sweep_store_nt, 1 sc1, 2 sc0 sc1, 3 nt sc1;
                                 // -1 (default): fp32 volumes 3, bf16 by sweep_store_nt
  int sweep_store_px = -1;       // k_sweep_tile fast path: 16-byte lane stores via LDS, 1/2/4/8 pixels per lane; 0: plain; -1: bf16 2, fp32 1
  int sweep_store_nt = 2;        // k_sweep_tile fast path: volume stores with sc0 nt (streaming); 2: bf16 volumes and
                                 // fp32 volumes of slabs <= 6 MiB (measured by shape)
  int sweep_run = 16;            // k_sweep_band (sweep_flat = 3): planes per block
  int sweep_band_rows = 16;      // k_sweep_band: most target rows staged in LDS (further clipped to 80 KB)
  int score_blocks_per_cu = 32;  // persistent score grid
  int score_fp32 = 1;            // packed float32 pre-decision in the score kernel
  int score_prune = 1;           // exact bound pruning in k_score32 (PruneState)
  int score_mf = 2;              // split-f16 MFMA scoring (exact by bound): 2 = k_score_mf2 (span-major, default
                                 // when num_test == num_ransac_test), 1 = k_score_mf (item-major), 0 = off
  int score_mf_chunk2 = 0;       // the same for the pruned second launch (0: score_mf_chunk)
  int score_mf_prune = 880;      // k_score_mf2 count-bound pruning: the first launch's share of each pair's
                                 // spans in per mille (0: off; one launch); later pruning points per pair from
                                 // k_mf2_split (an empty middle launch when the pair's own point is not later)
  int score_mf_prune_margin = 10; // the pruning point: 1 - (inlier ratio) + margin, per mille (k_mf2_split)
  int score_mf_prune_upper = 1;   // pruning passes one-sided (upper-bound counts), the kept candidates rescored (round 6)
  int score_mf_exact_max = 256;   // with upper: kept candidates per pair counted in float64 (k_mf2_exact); more: MFMA
  int score_mf_chunk = 64;       // k_score_mf2: smallest unit range a block claims (32-candidate tiles of a span);
                                 // 64 measured ~1 % faster than 128 with pruning (profiles/r05_prune_ab.txt)
  int score_mf_blocks_per_cu = 1; // k_score_mf persistent grid (LDS: one block per CU)
  int score_interleave = 0;      // k_score32 items: pairs interleaved (1) or pair after pair (0)
  int score_precision = 64;      // 64: exact (reference float64 decisions); 32 / 16: ComputeError<float> /
                                 // <half> semantics (approximate inlier sets, BASELINE C5)
  int score_lowp_template = 0;   // 32 / 16: 0 = E and every operation held in T (this build's variant);
                                 // 1 = the literal ComputeError<T> with double Ematrix (double products)
  int conv_rolling = 1;          // 1: cin-32 conv layers roll along the planes (k_conv3r); 0: k_conv3
};
Tuning& tuning();

// The score kernel the last RANSAC / score call dispatched (sfm_last_scorer):
// a static string literal.
void set_last_scorer(const char* name);
const char* last_scorer();

// Profiling hooks (capi.hip): record HIP events around a launch when enabled.
struct ProfScope {
  ProfScope(const char* name, hipStream_t s);
  ~ProfScope();
  int slot;
  hipStream_t stream;
};

}  // namespace sfm

#define SFM_REQUIRE(cond, msg)                 \
  do {                                         \
    if (!(cond)) {                             \
      ::sfm::set_error(msg);                   \
      return SFM_ERR_ARG;                      \
    }                                          \
  } while (0)

#define SFM_HIP(call)                                                             \
  do {                                                                            \
    hipError_t e_ = (call);                                                       \
    if (e_ != hipSuccess) {                                                       \
      ::sfm::set_error(std::string(#call) + ": " + hipGetErrorString(e_));        \
      return SFM_ERR_HIP;                                                         \
    }                                                                             \
  } while (0)

#define SFM_LAUNCHED()                                                            \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess) {                                                       \
      ::sfm::set_error(std::string("kernel launch: ") + hipGetErrorString(e_));   \
      return SFM_ERR_HIP;                                                         \
    }                                                                             \
  } while (0)
