"""The measured hot path: dense flow -> RANSAC five-point pose -> plane sweep.

``TwoViewHotPath`` runs, for a batch of image pairs already resident on the
GPU, exactly the work SFMnet.forward does between the flow estimator and the
3-D cost-regularisation CNN (models/SFMnet.py:103-166 with the dense-flow
branch of pose_by_ransac 176-274, and PSNet.py:130-158):

  1. correspondences from the flow (margin 10, K^-1)      sfm_flow_to_points
     (fused=True: read on the fly by the RANSAC kernels,   sfm_ransac5_flow)
  2. RANSAC five-point E / P per pair (H = 512 x iters)    sfm_ransac5_packed
  3. P -> pose, optional RESCALE_DEPTH translation scaling
  4. cost volume [B, 2C, L, h, w] at quarter resolution    sfm_plane_sweep

All buffers (points, RANSAC workspace, cost volume) are allocated once and
reused, so a step launches kernels only (hipGraph-capturable).
"""
import ctypes

import torch

from . import _lib, ransac, sweep


def kinv3x3(K):
    """K^-1 of [B,3,3] (or [3,3]) CUDA intrinsics, float32: torch.inverse's
    bits on ROCm in one launch (C ABI sfm_kinv3x3)."""
    if not K.is_cuda:
        raise RuntimeError("K must be a CUDA tensor")
    Kf = K.float().contiguous()
    if Kf.shape[-2:] != (3, 3):
        raise RuntimeError(f"K must be [..., 3, 3], got {tuple(K.shape)}")
    out = torch.empty_like(Kf)
    n = Kf.numel() // 9
    with torch.cuda.device(Kf.device):
        _lib.check(_lib.load().sfm_kinv3x3(_lib.ptr(Kf), n, _lib.ptr(out), _lib.stream_ptr(Kf.device)),
                   "sfm_kinv3x3")
    return out


class TwoViewHotPath:
    def __init__(self, batch, image_hw, feat_hw, channels=32, nlabel=128, iters=8, threshold=1e-4,
                 min_depth=1.0, rescale_depth=False, norm_target=0.6, cost_dtype=torch.float32, margin=10,
                 device="cuda", seed=ransac.DEFAULT_SEED, fused=False, keypoints=None, overlap_ref=False,
                 gate_scorer=True):
        self.batch = int(batch)
        # step_pipelined: the next step's scorer waits for this step's sweep
        # (sfm_score_gate), so the side-stream sweep overlaps the solve only
        self.gate_scorer = bool(gate_scorer)
        self.H, self.W = image_hw
        self.h, self.w = feat_hw
        self.C = int(channels)
        self.L = int(nlabel)
        self.iters = int(iters)
        self.thr = float(threshold)
        self.min_depth = float(min_depth)
        self.rescale = float(norm_target) if rescale_depth else None
        self.margin = int(margin)
        self.seed = int(seed)
        self.device = torch.device(device)
        self.n = (self.H - 2 * margin) * (self.W - 2 * margin)
        self.fused = bool(fused)
        B = self.batch
        # keypoints: (kp [B, n, 2] float32 on the device, counts) -> the sparse
        # branch of pose_by_ransac (SFMnet.py:250-254) instead of the dense one
        self.kp = keypoints
        if keypoints is not None:
            if self.fused:
                raise ValueError("the fused flow path is dense-only")
            self.kp_n = [int(v) for v in keypoints[1]]
            self.n = max(self.kp_n)
        # fused: RANSAC reads the flow directly (no correspondence buffer)
        self.pts = None if self.fused else torch.empty(B, self.n, 4, dtype=torch.float64, device=self.device)
        self.ws = ransac.workspace_for(B, self.iters, self.device)
        self.cost = torch.empty(B, 2 * self.C, self.L, self.h, self.w, dtype=cost_dtype, device=self.device)
        self.cost_dtype = cost_dtype
        self.sweep_ws = sweep.workspace_for(B, self.C, self.h, self.w, self.device)
        # overlap_ref: the volume's pose-independent reference half on a side
        # stream (see step_overlap): "score" (or True) beside the RANSAC scorer,
        # behind the score fence; "step" from the start of the step
        if overlap_ref not in (False, True, "score", "step"):
            raise ValueError("overlap_ref must be False, True, 'score' or 'step'")
        self.overlap_ref = {False: None, True: "score"}.get(overlap_ref, overlap_ref)
        if self.overlap_ref:
            self.ref_ws = sweep.ref_planes_workspace_for(B, self.C, self.h, self.w, self.device)
            self.ref_stream = torch.cuda.Stream(device=self.device)
            # per-device fence (created on the stream's device), reference-counted:
            # released in __del__
            _lib.check(_lib.load().sfm_score_fence_enable(1), "sfm_score_fence_enable")
            self._fence_on = True

    def __del__(self):
        if getattr(self, "_fence_on", False):
            self._fence_on = False
            try:
                _lib.load().sfm_score_fence_enable(0)
            except Exception:
                pass

    @staticmethod
    def k_inverse(K):
        """K^-1 as SFMnet.forward forms it (torch.inverse, models/SFMnet.py:104):
        one launch of sfm_kinv3x3, bit for bit torch.linalg.inv_ex's result on
        ROCm (tests/test_gpu_kinv.py), without a host sync."""
        return kinv3x3(K)

    def pose(self, flow, K, Kinv=None):
        if Kinv is None:
            Kinv = self.k_inverse(K)
        if self.fused:
            return ransac.ransac5_flow(flow, Kinv, self.iters, self.thr, self.H, self.W, self.margin, seed=self.seed,
                                       workspace=self.ws)
        n = None
        if self.kp is not None:
            ransac.gather_keypoints(flow, Kinv, self.kp[0], self.kp_n, "round", out=self.pts)
            n = self.kp_n
        else:
            ransac.flow_to_points(flow, Kinv, self.H, self.W, self.margin, out=self.pts)
        E, P, inl, win = ransac.ransac5_batched(self.pts, n, None, None, self.iters, self.thr, self.seed,
                                                True, workspace=self.ws)
        return E, P, inl, win

    def sweep(self, ref_fea, tgt_fea, P, K, Kinv=None):
        if Kinv is None:
            Kinv = self.k_inverse(K)
        # PSNet.py:130-133 + RESCALE_DEPTH inside the sweep call (same float32 bits
        # as quarter_intrinsics / P.float() * rescale, without ~10 ATen launches)
        return sweep.plane_sweep_cost_psnet(ref_fea, tgt_fea, P, K, Kinv, self.L, self.min_depth, self.rescale,
                                            self.cost_dtype, out=self.cost, workspace=self.sweep_ws)

    def step_pipelined(self, flow, K, ref_fea, tgt_fea):
        """``step`` with the sweep on a side stream: the pose stage runs on
        the caller's stream and does not wait for the previous step's sweep,
        so that HBM-bound sweep overlaps the next step's latency-bound
        five-point solve (1 wave/SIMD).  Same kernels, same results; the
        sweeps stay ordered on their stream, so the shared cost buffer is
        written in step order.  The caller synchronises (or waits on
        ``self.sweep_stream``) before reading the cost volume."""
        if getattr(self, "sweep_stream", None) is None:
            self.sweep_stream = torch.cuda.Stream(device=self.device)
        main = torch.cuda.current_stream(self.device)
        Kinv = self.k_inverse(K)
        E, P, inl, win = self.pose(flow, K, Kinv)
        side = self.sweep_stream
        side.wait_stream(main)
        for t in (Kinv, P, K, ref_fea, tgt_fea):
            t.record_stream(side)       # allocator: live until the side stream is done with them
        with torch.cuda.stream(side):
            cost = self.sweep(ref_fea, tgt_fea, P, K, Kinv)
        if self.gate_scorer:
            # the next step's scorer waits for this sweep (sfm_score_gate, an
            # event the library records on the side stream, armed for this
            # hot path's main stream only): the sweep overlaps that step's
            # solve, not its compute-bound scorer
            _lib.check(_lib.load().sfm_score_gate(ctypes.c_void_p(side.cuda_stream),
                                                  ctypes.c_void_p(main.cuda_stream), 1), "sfm_score_gate")
        return E, P, inl, cost

    def step_overlap(self, flow, K, ref_fea, tgt_fea):
        """``step`` with the cost volume's reference half (cost[:, :C, i] =
        ref, PSNet.py:155: no pose needed) written on a side stream that waits
        for the score fence, i.e. runs beside the compute-bound RANSAC scorer,
        which leaves HBM idle; the sweep after RANSAC then writes only the
        warped half.  The same volume bit for bit; the step returns after
        both halves (the caller's stream waits for the side stream)."""
        main = torch.cuda.current_stream(self.device)
        side = self.ref_stream
        side.wait_stream(main)                 # the previous step is done with the cost buffer
        Kinv = self.k_inverse(K)
        E, P, inl, win = self.pose(flow, K, Kinv)
        with torch.cuda.stream(side):
            if self.overlap_ref == "score":
                _lib.check(_lib.load().sfm_score_fence_wait(_lib.stream_ptr(self.device)), "sfm_score_fence_wait")
            sweep.plane_sweep_ref_half(ref_fea, self.L, self.cost, self.ref_ws)
        ref_fea.record_stream(side)
        cost = sweep.plane_sweep_cost_psnet(ref_fea, tgt_fea, P, K, Kinv, self.L, self.min_depth, self.rescale,
                                            self.cost_dtype, out=self.cost, workspace=self.sweep_ws, warped_half=True)
        main.wait_stream(side)
        return E, P, inl, cost

    def step(self, flow, K, ref_fea, tgt_fea):
        if self.overlap_ref:
            return self.step_overlap(flow, K, ref_fea, tgt_fea)
        Kinv = self.k_inverse(K)
        E, P, inl, win = self.pose(flow, K, Kinv)
        cost = self.sweep(ref_fea, tgt_fea, P, K, Kinv)
        return E, P, inl, cost
