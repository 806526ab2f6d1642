/*
 * sfm_hip.h — C ABI of the MI355X-native two-view SfM hot path
 * (libsfm_hip.so, built from deep-sfm-revisited_amd/csrc for gfx950).
 *
 * Drop-in boundary for jytime/Deep-SfM-Revisited:
 *   - the `essential_matrix` PyTorch extension (RANSAC_FiveP/essential_matrix/
 *     essential_matrix_wrapper.cpp:102-108) — initialise / computeP / optimise /
 *     decompose / decomposeUV;
 *   - the plane-sweep cost volume of models/PSNet.py:144-158 and the per-plane
 *     warp models/inverse_warp.py:121-153;
 *   - the dense correspondence build of models/SFMnet.py:176-263 (flow2coord
 *     298-318) feeding the RANSAC.
 *
 * Conventions
 *   - Every pointer marked [dev] is device memory on the current HIP device;
 *     [host] is host memory.  No torch types cross this boundary.
 *   - Device work is stream-ordered on `stream` (a hipStream_t, NULL = default
 *     stream).  Functions return before the work completes unless stated.
 *   - Return value: SFM_OK (0) or an SFM_ERR_* code; sfm_last_error() gives a
 *     message (thread-local).  Nothing calls exit() (the reference's
 *     CudaErrorCheck exit()s the process: essential_matrix.cu:17-24).
 *   - Scratch memory is caller-provided (`workspace`), sized by the matching
 *     *_workspace_bytes() query; no call allocates device memory, so every
 *     device entry point is hipGraph-capturable.
 */
#ifndef SFM_HIP_H
#define SFM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  SFM_OK = 0,
  SFM_ERR_ARG = 1,        /* invalid argument (shape, size, range)          */
  SFM_ERR_HIP = 2,        /* HIP runtime / launch error                     */
  SFM_ERR_WORKSPACE = 3   /* workspace missing or too small                 */
};

#define SFM_ABI_VERSION 1
#define SFM_RANSAC_CHAINS 512   /* reference: 8 blocks x 64 threads (essential_matrix.cu:201-203) */
#define SFM_MAX_BATCH 64        /* pairs per device launch (larger batches are chunked) */

int sfm_abi_version(void);
const char* sfm_last_error(void);

/* ------------------------------------------------------------------------
 * RANSAC five-point essential matrix
 * ------------------------------------------------------------------------
 * Hypotheses: H = SFM_RANSAC_CHAINS * iters; hypothesis h = t*iters + i is
 * iteration i of chain t (reference thread t).  Sampling: Philox4x32-10 keyed
 * by `seed`, counter {h, draw/4, 0, 0}, curand_uniform-style (0,1] floats
 * turned into indices by the reference's RandomInt arithmetic, clamped to n-1.
 * Selection: per hypothesis the best candidate on the first num_test points
 * (first strict max, default candidate 0), rescored on the first
 * num_ransac_test points; the winner is the first hypothesis (in h order)
 * with the maximal rescored count — exactly the reference's per-thread
 * strict-> update followed by the host max_element (kernel_functions.cu:
 * 141-226, essential_matrix.cu:248-265).  If no hypothesis has an inlier,
 * E = P = 0, inliers = 0, winner = -1 (the reference returns uninitialised
 * memory there).
 */

/* Workspace for up to `batch` pairs of at most n_max points and `iters`
 * RANSAC iterations per chain. */
size_t sfm_ransac5_workspace_bytes(int batch, int64_t n_max, int iters);

/* Single pair, reference layout.  Replaces ProjectionMatrixRansac
 * (essential_matrix.cu:190-280, cheirality=1) and EssentialMatrixInitialise
 * (essential_matrix.cu:110-184, cheirality=0).
 *   q, qp          [dev] n x 2 float64, row-major (x, y) — input1 / input2
 *   E_out          [dev] 3x3 float64; P_out [dev] 3x4 float64 (may be NULL
 *                  when cheirality == 0); inliers_out [dev] int32[1];
 *   winner_out     [dev] int32[1] or NULL.
 * Requires 1 <= num_test, num_ransac_test <= n (the reference reads out of
 * bounds otherwise), iters >= 1, thr > 0. */
int sfm_ransac5(const double* q, const double* qp, int64_t n,
                int num_test, int num_ransac_test, int iters, double thr,
                uint64_t seed, int cheirality,
                void* workspace, size_t workspace_bytes,
                double* E_out, double* P_out, int32_t* inliers_out, int32_t* winner_out,
                void* stream);

/* Batched pairs on packed correspondences.
 *   pts            [dev] batch x n_stride x 4 float64: (x, y, x', y') per point
 *   n              [host] batch int64: points of each pair (<= n_stride)
 *   num_test, num_ransac_test: per-call; values <= 0 mean "all n[b] points"
 *   E_out [dev] batch x 9, P_out [dev] batch x 12 (or NULL), inliers_out
 *   [dev] batch int32, winner_out [dev] batch int32 or NULL,
 *   hyp_score_out  [dev] batch x H int32 rescored count per hypothesis, or NULL.
 */
int sfm_ransac5_packed(const double* pts, int64_t n_stride, const int64_t* n, int batch,
                       int num_test, int num_ransac_test, int iters, double thr,
                       uint64_t seed, int cheirality,
                       void* workspace, size_t workspace_bytes,
                       double* E_out, double* P_out, int32_t* inliers_out, int32_t* winner_out,
                       int32_t* hyp_score_out, void* stream);

/* Fused dense path: RANSAC straight from the flow
 * field, no correspondence buffer.  Point k of each pair is pixel
 * (u, v) = (m + k % (w_side-2m), m + k / (w_side-2m)) of the crop, with the
 * values of sfm_flow_to_points (bit-identical results to
 * sfm_flow_to_points + sfm_ransac5_packed).
 *   flow [dev] batch x 2 x H x W float32; Kinv [dev] batch x 3 x 3 float32;
 *   other arguments and outputs as sfm_ransac5_packed. */
int sfm_ransac5_flow(const float* flow, int batch, int H, int W, int h_side, int w_side, int margin,
                     const float* Kinv, int num_test, int num_ransac_test, int iters, double thr,
                     uint64_t seed, int cheirality, void* workspace, size_t workspace_bytes,
                     double* E_out, double* P_out, int32_t* inliers_out, int32_t* winner_out,
                     int32_t* hyp_score_out, void* stream);

/* Inlier counts of given essential matrices over packed correspondences:
 * counts[b][c] = #{k < n[b] : e(E[b][c], point k) <= thr} with e the
 * reference's ComputeError<double> Sampson-style error
 * (kernel_functions.cu:232-264), through the same scorer the RANSAC uses
 * (split-f16 matrix-core decisions exact by bound + float64 re-test; the
 * float32 / float64 VALU scorers outside its threshold range), bit-exact.
 * The reference's scoring loop over a candidate set (kernel_functions.cu:
 * 187-214) without the sampling.
 *   pts [dev] batch x n_stride x 4 float64; n [host] batch;
 *   E [dev] batch x ncand x 9 float64; counts [dev] batch x ncand int32;
 *   workspace [dev] sfm_score_essentials_workspace_bytes(batch, ncand). */
size_t sfm_score_essentials_workspace_bytes(int batch, int ncand);
int sfm_score_essentials(const double* pts, int64_t n_stride, const int64_t* n, int batch, const double* E,
                         int ncand, double thr, int32_t* counts, void* workspace, size_t workspace_bytes,
                         void* stream);

/* Exact inlier mask of E (reference ComputeError + `<= thr`) for each point.
 *   pts [dev] batch x n_stride x 4; n [host] batch; E [dev] batch x 9;
 *   mask [dev] batch x n_stride uint8 (entries >= n[b] are written 0). */
int sfm_ransac5_inlier_mask(const double* pts, int64_t n_stride, const int64_t* n, int batch,
                            const double* E, double thr, uint8_t* mask, void* stream);

/* Dense flow -> packed normalised correspondences (models/SFMnet.py:179-263,
 * flow2coord 298-318): crop flow to h_side x w_side, drop a `margin` border,
 * q = (K^-1 (u, v, 1))[:2], qp = (K^-1 (u+fu, v+fv, 1))[:2] in float32 rows
 * (k0*x + k1*y) + k2, widened to float64.  Point k = (v-m)*(w_side-2m)+(u-m).
 *   flow [dev] batch x 2 x H x W float32; Kinv [dev] batch x 3 x 3 float32;
 *   pts_out [dev] batch x N x 4 float64, N = (h_side-2m)(w_side-2m). */
int sfm_flow_to_points(const float* flow, int batch, int H, int W, int h_side, int w_side,
                       int margin, const float* Kinv, double* pts_out, void* stream);

/* Sparse correspondences of SFMnet.pose_by_ransac (models/SFMnet.py:218-258),
 * for keypoints from any matcher (the reference uses cv2 SIFT/SURF + FLANN):
 *   mode 0: flow at np.round(kp1) (round half to even; caller validates the
 *           range — the reference's indexing raises), cfg default;
 *   mode 1: cfg.SAMPLE_SP — grid_sample (align_corners=True, zeros) of the
 *           coordinate grids at kp1;
 *   mode 2: cfg.SIFT_POSE — the matched keypoints kp1 / kp2 themselves;
 * then K^-1 (float32, 3 rows) and f64 widening.
 *   flow [dev] batch x 2 x H x W float32 (unused for mode 2), cropped to
 *   h_side x w_side; kp1, kp2 [dev] batch x kp_stride x 2 float32 pixel (x, y);
 *   n [host] batch int64 keypoints per pair; Kinv [dev] batch x 3 x 3 float32;
 *   pts_out [dev] batch x n_stride x 4 float64 (rows >= n[b] untouched). */
int sfm_keypoints_to_points(const float* flow, int batch, int H, int W, int h_side, int w_side,
                            const float* kp1, const float* kp2, int64_t kp_stride, const int64_t* n, int mode,
                            const float* Kinv, double* pts_out, int64_t n_stride, void* stream);

/* Scored candidate E's per pair of the last sfm_ransac5_packed call made with
 * this workspace (the last <= SFM_MAX_BATCH chunk), copied to the host
 * (synchronous).  Work accounting: the score kernel evaluates
 * counts[b] x max(num_test, num_ransac_test) correspondences for pair b. */
int sfm_ransac5_candidate_counts(const void* workspace, size_t workspace_bytes, int batch, int iters,
                                 int32_t* counts_host);

/* Evaluations the last RANSAC call with this workspace skipped by exact
 * bound pruning (tuning key score_prune; on when num_test == num_ransac_test
 * and hyp_score_out is NULL), copied to the host (synchronous).  The score
 * kernel performed sum(counts) x max(num_test, num_ransac_test) minus this
 * many evaluations.  Pruning never changes E, P, the inlier count or the
 * winner (ransac5.hip, PruneState). */
int sfm_ransac5_skipped_evaluations(const void* workspace, size_t workspace_bytes, int batch, int iters,
                                    unsigned long long* skipped_host);
/* Diagnostics of the last pruned k_score_mf2 call on the workspace
 * (sfm_last_scorer() "k_score_mf2+prune"): per pair, the candidates the
 * count bound kept (scored to their exact counts); every other candidate was
 * dropped after the pruning point; points_host (optional): per pair, the
 * pruning point in points (a multiple of the 1024-point span: clamp at the
 * pair's N).  Undefined after an unpruned call.  Synchronises. */
int sfm_ransac5_kept_candidates(const void* workspace, size_t workspace_bytes, int batch, int iters,
                                int32_t* kept_host, int32_t* points_host);

/* Pack reference-layout q, qp (n x 2 each) into pts (n x 4). */
int sfm_pack_points(const double* q, const double* qp, int64_t n, double* pts_out, void* stream);

/* ------------------------------------------------------------------------
 * Host-side E utilities (the reference runs these on CPU tensors too)
 * ------------------------------------------------------------------------ */
/* EssentialMatrixOptimise -> polish_E_robust_parametric (essential_matrix.cu:
 * 76-105, polish_E.cu:1470-1577).  All pointers [host]; q, qp n x 2. */
int sfm_essential_optimise(const double* q, const double* qp, int64_t n, const double* E_init,
                           double delta, double alpha, int max_reps, double* E_out);
/* Batched GPU form of the same IRLS.  The sums are
 * reassociated (parallel reduction), so E agrees with the host version to
 * rounding level, not bit for bit.
 *   pts [dev] batch x n_stride x 4 float64 (x, y, x', y'); n [host] batch;
 *   E_init, E_out [dev] batch x 9 float64. */
size_t sfm_essential_optimise_workspace_bytes(int batch, int64_t n_max);
int sfm_essential_optimise_batched(const double* pts, int64_t n_stride, const int64_t* n, int batch,
                                   const double* E_init, double delta, double alpha, int max_reps,
                                   double* E_out, void* workspace, size_t workspace_bytes, void* stream);
/* EssentialMatrixDecompose -> Edecomp(E, params) (essential_matrix.cu:29-43). */
int sfm_essential_decompose(const double* E, double* params5);
/* EssentialMatrixDecomposeUV -> Edecomp(E, U, V) (essential_matrix.cu:48-70). */
int sfm_essential_decompose_uv(const double* E, double* U, double* V);

/* ------------------------------------------------------------------------
 * Plane sweep
 * ------------------------------------------------------------------------ */
/* Scratch for the plane sweep: the target features re-laid out as channel
 * quads [B][ceil(C/4)][h*w][4] float32. */
size_t sfm_plane_sweep_workspace_bytes(int batch, int channels, int h, int w);

/* Cost volume of models/PSNet.py:144-157 for one target view:
 *   cost[b, c,   i] = ref[b, c]                     (c < C)
 *   cost[b, C+c, i] = inverse_warp(tgt, d_i)[b, c]
 * with d_i = (min_depth * nlabel) / (i + 1) in float32.
 *   ref, tgt [dev] batch x C x h x w float32
 *   pose     [dev] batch x 3 x 4 float32 (already RESCALE_DEPTH-scaled)
 *   K4, K4inv [dev] batch x 3 x 3 float32 (feature-resolution intrinsics)
 *   out_dtype 0: float32, 1: bfloat16 (round-to-nearest-even)
 *   cost     [dev] batch x 2C x nlabel x h x w */
int sfm_plane_sweep(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                    const float* pose, const float* K4, const float* K4inv,
                    int nlabel, float min_depth, int out_dtype, void* cost,
                    void* workspace, size_t workspace_bytes, void* stream);

/* General form.  ref == NULL: warped half only, out batch x C x nlabel x h x w.
 *   depth_mode 0: d_i = (min_depth * nlabel) / (i + 1)   (disp2depth, default)
 *   depth_mode 1: d_i = (i + 1) * min_depth               (cfg.PREDICT_BY_DEPTH,
 *                                                          PSNet.py:150-151) */
int sfm_plane_sweep_ex(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                       const float* pose, const float* K4, const float* K4inv,
                       int nlabel, float min_depth, int depth_mode, int out_dtype, void* cost,
                       void* workspace, size_t workspace_bytes, void* stream);

/* The sweep section of PSNet.forward from the pose stage's outputs, in one
 * call (models/PSNet.py:130-157): the reference's tensor preparation runs in a
 * one-thread-per-pair kernel instead of ~10 ATen launches, bit for bit:
 *   pose      [dev] batch x 3 x 4, pose_dtype 0: float32, 1: float64 (P.float())
 *   K, Kinv   [dev] batch x 3 x 3 float32, full resolution; K4 = K with rows
 *             0-1 / 4, K4inv = Kinv with [:2,:2] * 4 (PSNet.py:130-133)
 *   t_scale   > 0: translation column * t_scale in float32 (cfg.RESCALE_DEPTH);
 *             <= 0: unscaled
 * then as sfm_plane_sweep_ex (ref == NULL: warped half only). */
int sfm_plane_sweep_psnet(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                          const void* pose, int pose_dtype, const float* K, const float* Kinv, float t_scale,
                          int nlabel, float min_depth, int depth_mode, int out_dtype, void* cost,
                          void* workspace, size_t workspace_bytes, void* stream);

/* The two halves of sfm_plane_sweep_psnet's volume separately, so that the
 * pose-independent reference half (cost[:, :C, i] = ref, PSNet.py:155) can be
 * written on a second stream while RANSAC runs (round 4; the scorer is
 * compute-bound and leaves HBM idle):
 *   sfm_plane_sweep_ref_planes         rows 0..C-1 of every pair's
 *       [2C, nlabel, h, w] volume: a copy of ref per plane (bf16: RNE), in one
 *       wave per SIMD with 8 VGPRs, which fits beside the scorer's waves.
 *       workspace: sfm_plane_sweep_ref_planes_workspace_bytes (a padded copy
 *       of ref); shapes off its fast path use a generic kernel.
 *   sfm_plane_sweep_psnet_warped_half  sfm_plane_sweep_psnet without those rows
 *       (windows off the sweep's fast path still write them from ref: the
 *       same values).
 * Together they write exactly sfm_plane_sweep_psnet's volume. */
size_t sfm_plane_sweep_ref_planes_workspace_bytes(int batch, int channels, int h, int w);
/* Score fence: while enabled, every RANSAC call records a library-owned
 * event on its stream right before its scoring phase; sfm_score_fence_wait
 * makes `stream` wait for the last one recorded on that stream's device (so
 * the reference half can run beside the compute-bound scorer rather than the
 * latency-bound solve).  One event per device, created on the device of the
 * stream (not the caller's current device).  enable(1) / enable(0) are
 * reference-counted: recording stays on until every enable(1) has been
 * matched by an enable(0) (TwoViewHotPath enables it for its lifetime).
 * Every RANSAC call on a device records the same fence, so two hot paths
 * sharing a device wait on whichever scoring phase was enqueued last. */
int sfm_score_fence_enable(int on);
int sfm_score_fence_wait(void* stream);

/* Score gate (round 5; scoped to a waiting stream in round 6).  arm = 1:
 * record a library-owned event on `stream` and arm it for `waiter`: the next
 * RANSAC call (sfm_ransac5 / _packed / _flow) issued on the stream `waiter`
 * (on stream's device) makes `waiter` wait for the event right before its
 * scoring phase, and disarms the gate (one-shot).  RANSAC calls on any other
 * stream neither wait for nor consume it, so a second hot path or a plain
 * computeP on the same device is unaffected.  Re-arming for the same waiter
 * replaces the previous gate; arm = 0 disarms the waiter's gate.  At most 32
 * gates are armed at once (SFM_ERR_ARG beyond).  A pipelined caller arms it on
 * the side stream right after the previous step's sweep, for its own main
 * stream, so that sweep overlaps this step's correspondence build and
 * five-point solve but not the scorer
 * (sfm_amd.pipeline.TwoViewHotPath.step_pipelined).  No reference
 * counterpart: the reference's steps are serial (essential_matrix.cu:190-280
 * then PSNet.py:130-158). */
int sfm_score_gate(void* stream, void* waiter, int arm);
int sfm_plane_sweep_ref_planes(const float* ref, int batch, int channels, int h, int w, int nlabel, int out_dtype,
                               void* cost, void* workspace, size_t workspace_bytes, void* stream);
int sfm_plane_sweep_psnet_warped_half(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                                      const void* pose, int pose_dtype, const float* K, const float* Kinv,
                                      float t_scale, int nlabel, float min_depth, int depth_mode, int out_dtype,
                                      void* cost, void* workspace, size_t workspace_bytes, void* stream);

/* Warped half only (cost[b, c, i] = inverse_warp(tgt, d_i)), batch x C x nlabel x h x w. */
int sfm_plane_sweep_warped(const float* tgt, int batch, int channels, int h, int w,
                           const float* pose, const float* K4, const float* K4inv,
                           int nlabel, float min_depth, int out_dtype, void* out,
                           void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------
 * Depth stage after the sweep
 * ------------------------------------------------------------------------ */
/* Scratch for sfm_plane_sweep_correlation: channel quads of ref and tgt. */
size_t sfm_correlation_workspace_bytes(int batch, int channels, int h, int w);

/* Correlation cost of REG2D.py:103-109 without the warped volume:
 *   cost[b, i] = mean_c(ref[b, c] * inverse_warp(tgt, d_i)[b, c])
 *   ref, tgt [dev] batch x C x h x w float32; pose/K4/K4inv as sfm_plane_sweep;
 *   depth_mode as sfm_plane_sweep_ex; cost [dev] batch x nlabel x h x w float32. */
int sfm_plane_sweep_correlation(const float* ref, const float* tgt, int batch, int channels, int h, int w,
                                const float* pose, const float* K4, const float* K4inv, int nlabel,
                                float min_depth, int depth_mode, float* cost,
                                void* workspace, size_t workspace_bytes, void* stream);

/* Soft-argmin depth head of PSNet.py:191-213 (submodule.py:57-93):
 * F.interpolate(cost, [L, H, W], 'trilinear', align_corners=False) -> softmax
 * over planes -> depth_mode 0: depth = min_depth*L / (sum p_i (i+1) + 1e-16)
 *                depth_mode 1: depth = min_depth * sum p_i (i+1) depth_step
 *                              (cfg.PREDICT_BY_DEPTH; depth_step = int(MIN_DEPTH))
 *   cost [dev] batch x nlabel x h x w float32; depth [dev] batch x H x W float32. */
int sfm_depth_head(const float* cost, int batch, int nlabel, int h, int w, int H, int W, int depth_mode,
                   float min_depth, float depth_step, float* depth, void* stream);

/* K^-1 of a batch of 3x3 matrices, as models/SFMnet.py:104 forms it
 * (intrinsic_inv_gpu = torch.inverse(intrinsic_gpu)): bit for bit what
 * torch.linalg.inv_ex returns on ROCm (rocsolver getrf + getrs order), in one
 * launch.  K, Kinv [dev] batch x 3 x 3 float32 row-major.  Singular K gives
 * inf / NaN entries (torch raises). */
int sfm_kinv3x3(const float* K, int batch, float* Kinv, void* stream);

/* models/inverse_warp.py:121-153 for an arbitrary depth map:
 *   feat [dev] B x C x h x w; depth [dev] B x h x w; pose [dev] B x 3 x 4;
 *   K, Kinv [dev] B x 3 x 3; out [dev] B x C x h x w (float32). */
int sfm_inverse_warp(const float* feat, int batch, int channels, int h, int w,
                     const float* depth, const float* pose, const float* K, const float* Kinv,
                     float* out, void* stream);

/* Flow2Depth, models/flow2depth.py:7-41 (dead code in the reference):
 *   KR = K.R [dev] B x 3 x 3, KT = K.T [dev] B x 3, Kinv [dev] B x 3 x 3
 *   (float32, numpy's inverse of K as the reference takes it);
 *   out [dev] B x H x W float32 = channel 2 of the [B, H*W, 3] result viewed
 *   as [B, 3, H, W], exactly as the reference returns it. */
int sfm_flow2depth(const float* KR, const float* KT, const float* Kinv, int batch, int H, int W, float* out,
                   void* stream);

/* 3-D cost regularisation layer of PSNet (models/PSNet.py:79-102, applied at
 * PSNet.py:159-165; convbn_3d = Conv3d(3, stride 1, pad 1, no bias) +
 * BatchNorm3d, models/submodule.py:17-20), on the matrix cores in bf16 with
 * fp32 accumulation:
 *   out = [relu](conv3x3x3(in) * scale[co] + bias[co]) [+ residual]
 *   in [dev] batch x depth x h x w x cin bf16 (channels-last), cin 32 or 64;
 *   weights [dev] 27 x 32 x cin bf16, tap = (kd*3 + kh)*3 + kw, cout
 *     zero-padded to 32 when cout == 1;
 *   scale, bias [dev] 32 float32 (BatchNorm folded; 1 / 0 for a plain conv);
 *   residual [dev] like out or NULL (cout 32 only), added after the ReLU;
 *   out [dev] batch x depth x h x w x 32 bf16 (cout 32), or
 *       batch x depth x h x w float32 (cout 1: the classify output). */
int sfm_conv3_bf16(const void* in, int batch, int cin, int depth, int h, int w, const void* weights,
                   const float* scale, const float* bias, const void* residual, int relu, int cout, void* out,
                   void* stream);

/* [batch][channels][plane] float32 (in_dtype 0) or bfloat16 (1) ->
 * [batch][plane][channels] bfloat16 (channels a multiple of 8): the
 * sweep's cost volume [B, 2C, L, h, w] into sfm_conv3_bf16's layout. */
int sfm_to_channels_last_bf16(const void* in, int in_dtype, int batch, int channels, int64_t plane, void* out,
                              void* stream);

/* The same layer with float16 activations and weights (11-bit mantissa,
 * fp32 accumulation on v_mfma_f32_32x32x16_f16): the precision the
 * reference's Conv3d layers run at under cfg.MIXED_PREC autocast
 * (models/SFMnet.py:164, cfgs/kitti.yml:10).  Arguments and layouts as
 * sfm_conv3_bf16, every 16-bit operand IEEE half. */
int sfm_conv3_f16(const void* in, int batch, int cin, int depth, int h, int w, const void* weights,
                  const float* scale, const float* bias, const void* residual, int relu, int cout, void* out,
                  void* stream);

/* [batch][channels][plane] float32 (in_dtype 0) or bfloat16 (1) ->
 * [batch][plane][channels] float16 (round to nearest even), sfm_conv3_f16's
 * layout. */
int sfm_to_channels_last_f16(const void* in, int in_dtype, int batch, int channels, int64_t plane, void* out,
                             void* stream);

/* The same layer at the reference's precision (conv_precision "fp32"):
 * float32 operands on v_mfma_f32_32x32x2_f32 (an exact fmaf chain: products
 * and sums round as float32 arithmetic; only the summation order differs from
 * PSNet's own Conv3d, models/PSNet.py:79-102).
 *   in [dev] batch x depth x h x w x cin float32 (channels-last), cin 32 or 64;
 *   weights [dev] 27 x 32 x cin float32 (layout as sfm_conv3_bf16);
 *   scale, bias [dev] 32 float32; residual [dev] like out or NULL;
 *   out [dev] batch x depth x h x w x 32 float32 (cout 32), or
 *       batch x depth x h x w float32 (cout 1).  All 16-byte aligned. */
int sfm_conv3_f32(const float* in, int batch, int cin, int depth, int h, int w, const float* weights,
                  const float* scale, const float* bias, const float* residual, int relu, int cout, float* out,
                  void* stream);

/* sfm_conv3_f32's layer with fp32 products formed on the f16 matrix cores
 * (conv_precision "fp32x3", round 5): both operands split in two f16 terms
 * (x = x_hi + x_lo; the weights first scaled by 2^wexp so their lo terms stay
 * normal, the scale folded back in the epilogue) and
 * w x ~ w_hi x_hi + w_hi x_lo + w_lo x_hi, three v_mfma_f32_32x32x16_f16 per
 * k = 16 into fp32 accumulators (~2^-21 relative per product).  Same layouts
 * and arguments as sfm_conv3_f32, plus wexp in [-24, 24] (the caller picks it
 * so that 2^wexp max|w| < 2^15).  Replaces the same Conv3d layers
 * (models/PSNet.py:79-102, applied at 159-165).
 * The split is valid while every input activation is within the f16 range
 * (|x| <= 65504; the reference's fp32 Conv3d has no such limit).  range_flag
 * [dev] 4 bytes or NULL: when given, the call zeroes it, the kernel sets it to
 * 1 if any input activation exceeds 65504 (or is infinite), and a second,
 * stream-ordered launch of the sfm_conv3_f32 layer overwrites out in that case
 * (its blocks exit at once otherwise) -- the layer's result is then exactly
 * sfm_conv3_f32's.  NULL: no check (the caller guarantees the range).  Below
 * 2^-14 the f16 terms are subnormal: such activations keep an absolute error
 * <= 2^-25 per product term, not a relative one. */
int sfm_conv3_f32x3(const float* in, int batch, int cin, int depth, int h, int w, const float* weights, int wexp,
                    const float* scale, const float* bias, const float* residual, int relu, int cout, float* out,
                    int* range_flag, void* stream);

/* [batch][channels][plane] float32 (in_dtype 0) or bfloat16 (1) ->
 * [batch][plane][channels] float32 (channels a multiple of 4): the sweep's
 * cost volume into sfm_conv3_f32's layout. */
int sfm_to_channels_last_f32(const void* in, int in_dtype, int batch, int channels, int64_t plane, float* out,
                             void* stream);

/* Tuning knobs (process-wide; every key, its accepted values and default):
 *
 *   launch shape only -- outputs are bit-identical for every value:
 *     "solve_lanes"           1..16   lanes per wave in k_solve_front (16)
 *     "solve_coop"            0, 1    k_solve_front's equations and reduction and
 *                                     k_solve_back on DPP quads, 4 lanes per
 *                                     hypothesis (1); 0: one lane each
 *     "roots_lanes"           1..32   lanes per wave in k_roots (32)
 *     "sweep_lane_pixels"     0..2    pixel-to-lane mapping of the per-row sweep (0)
 *     "sweep_items_per_block" 1,2,4,8 work items per block of the per-row sweep (4)
 *     "sweep_nj"              1,2,4   pixels per lane of k_sweep_tile (1; bf16 uses 2)
 *     "sweep_buffer"          0, 1    buffer-addressed interior path of k_sweep_tile (1)
 *     "sweep_share"           0, 1    k_sweep_tile interior path: right-hand bilinear taps
 *                                     from the next lane where the offsets match (0)
 *     "sweep_store_nt"        0,1,2   k_sweep_tile's volume stores non-temporal (sc0 nt)
 *                                     so they do not evict the re-read operands
 *                                     (2, default: bf16 volumes, and fp32 volumes
 *                                     whose channel slab L*h*w*4 is <= 6 MiB --
 *                                     measured per shape, e.g. on for the indoor
 *                                     120x160 L=64 volume, off for KITTI 94x311)
 *     "sweep_store_wt"        -1..3   cache policy of k_sweep_tile's 16-byte stores:
 *                                     0 by sweep_store_nt, 1 sc1 (write-through:
 *                                     the line is not kept in the XCD's L2), 2 sc0
 *                                     sc1, 3 nt sc1; -1 (default): fp32 volumes 3,
 *                                     bf16 volumes 0; same bits
 *     "sweep_store_px"        -1,0,1, 16-byte lane stores of k_sweep_tile (8 bf16 / 4
 *                             2,4,8   fp32 consecutive pixels through a per-wave LDS
 *                                     stage) with that many pixels per lane for the
 *                                     taps; 0: plain 4-byte lane stores; -1 (default):
 *                                     bf16 2, fp32 1; same bits
 *     "sweep_run"             1..1024 planes per block of k_sweep_band (16)
 *     "sweep_band_rows"       2..64   target rows k_sweep_band stages in LDS (16,
 *                                     clipped to 80 KB per block)
 *     "score_blocks_per_cu"   1..64   persistent k_score32 blocks per CU (32)
 *     "score_mf_blocks_per_cu" 1..8   persistent k_score_mf blocks per CU (1)
 *     "score_prune"           0, 1    exact bound pruning in k_score32 (1; winner,
 *                                     count, E, P unchanged -- losing hypotheses'
 *                                     scores become lower bounds, so it is off
 *                                     whenever per-hypothesis scores are requested)
 *     "score_interleave"      0, 1    pair-interleaved k_score32 items (0)
 *     "score_fp32"            0, 1    float32 pre-decision level of k_score32 (1; exact by proof)
 *     "score_mf"              0..2    split-f16 matrix-core scorers (2: span-major
 *                                     k_score_mf2, 1: k_score_mf, 0: VALU scorers;
 *                                     2 by default; exact by proof, same counts)
 *     "score_mf_chunk"        1..4096 k_score_mf2's smallest claimed unit range, in
 *                                     (span, 32-candidate tile) units (64)
 *     "score_mf_chunk2"       0..4096 the same for the pruned sequence's last launch (0: as
 *                                     score_mf_chunk)
 *     "score_mf_prune"        0, 500..990  count-bound pruning in k_score_mf2 (880):
 *                                     every candidate scored on the first N per
 *                                     mille of each pair's 1024-point spans, then
 *                                     up to the pair's pruning point 1 - (inlier
 *                                     ratio estimated from them) + margin
 *                                     (k_mf2_split), then only candidates whose
 *                                     bound can still reach the leader's exact
 *                                     count (k_mf2_lead / _keep); 0 = one launch.
 *                                     Winner, count, E, P unchanged; only with
 *                                     num_test == num_ransac_test, no per-
 *                                     hypothesis scores, >= 32 spans per pair
 *     "score_mf_prune_margin" 0..200  that margin, per mille (10)
 *     "score_mf_prune_upper"  0, 1    1 (default, round 6): every candidate on
 *                                     every point with the one-sided test (counts
 *                                     of the points not certainly outliers: upper
 *                                     bounds), the leader counted exactly, and only
 *                                     the candidates whose upper count reaches it
 *                                     counted exactly (float64, or the two-sided
 *                                     matrix-core pass past 256 per pair); 0: the
 *                                     round-5 two-sided passes with the pruning
 *                                     point above.  Winner, count, E, P unchanged
 *     "score_mf_exact_max"    0..256  with score_mf_prune_upper: pairs with at most
 *                                     this many kept candidates count them in
 *                                     float64 (k_mf2_exact), the others on the
 *                                     matrix cores (256; same counts either way)
 *     "roots_split"           0, 1, 2 k_roots_split: falsi nodes shared by the wave's
 *                                     64 lanes (1, default), or by the four waves of
 *                                     a block (2, measured 2-6 % slower), speculated
 *                                     fallback bisection; same bits as k_roots (0)
 *     "conv_rolling"          0, 1    rolling-plane Conv3d for cin 32 (1; same bits)
 *
 *   results MAY change (sweep outputs by FMA rounding only):
 *     "sweep_flat"            0..3    2 (default): k_sweep_tile, 1: k_sweep_flat,
 *                                     3: k_sweep_band (plane runs, target band in
 *                                     LDS; measured slower); 1-3 are bit-identical
 *                                     to each other; they sum the
 *                                     four bilinear taps with FMA, which differs
 *                                     from 0, the per-row kernel in the
 *                                     reference's mul/add order, by <= 7.2e-7
 *                                     absolute on N(0,1) features
 *     "sweep_group"           4, 8    channels per sweep window (8); the channel
 *                                     group changes nothing but the launch shape
 *     "score_precision"       64, 32, 16  64 (default): the reference's float64
 *                                     ComputeError decision, exact; 32 / 16:
 *                                     ComputeError<float> / <half> semantics
 *                                     (approximate inlier sets, BASELINE C5)
 *     "score_lowp_template"   0, 1    32 / 16 only: 0 (default) E and every
 *                                     operation held in T; 1 the literal
 *                                     ComputeError<T> with the reference's
 *                                     double Ematrix (double products, sums
 *                                     rounded to T; kernel_functions.cu:231-264,
 *                                     common.h:26) */
int sfm_tune_set(const char* key, int value);
/* The current value of a tuning key. */
int sfm_tune_get(const char* key, int* value);
/* The name of tuning key `index` (0, 1, ...), NULL past the last one: lets a
 * caller snapshot and restore every knob (tests/conftest.py does, around
 * each GPU test). */
const char* sfm_tune_key(int index);
/* The score kernel the most recent RANSAC / score call of this process
 * dispatched ("k_score_mf2", "k_score_mf", "k_score32", ...; "" before any),
 * followed by "+prune" when k_score_mf2 ran with count-bound pruning (two
 * launches and k_mf2_lead / k_mf2_keep between them).  A dispatch check for tests. */
const char* sfm_last_scorer(void);

/* ------------------------------------------------------------------------
 * Per-kernel timing (HIP events recorded around every launch on the
 * launching stream while enabled).
 * ------------------------------------------------------------------------ */
int sfm_profile_enable(int on);
/* Restrict the recording to the comma-separated kernel names in `names`
 * (NULL or "" = every profiled kernel).  Each recorded launch adds two event
 * records to its stream (~3.5 us per step per kernel on MI355X between
 * dependent launches), so bench.py records only the roofline kernels inside
 * its timed region. */
int sfm_profile_select(const char* names);
int sfm_profile_reset(void);
/* Synchronises the recorded events; total milliseconds and launch count of
 * kernel `name` ("ransac_solve", "ransac_chain", "ransac_score",
 * "ransac_select", "flow_to_points", "plane_sweep", "sweep_tgt_quads", ...). */
int sfm_profile_read(const char* name, double* total_ms, int* launches);

#ifdef __cplusplus
}
#endif

#endif /* SFM_HIP_H */
