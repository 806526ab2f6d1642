"""Depth stage after the plane sweep, over the C ABI.

* ``correlation_cost`` — REG2D.py:103-109's parameter-free cost
  (ref * inverse_warp(tgt, d_i)).mean(1) for every plane in one launch, without
  the [B, C, L, h, w] warped volume.
* ``depth_head``       — PSNet.py:191-213 soft-argmin head: trilinear upsample
  of a [B, L, h, w] (or [B, 1, L, h, w]) cost to the image size, softmax over
  planes, disparity / depth regression (submodule.py:57-93).
* ``CorrelationDepth`` — correlation cost + head: a parameter-free depth map
  from (ref_fea, tgt_fea, pose) at image resolution.
"""
import torch

from . import _lib
from .sweep import quarter_intrinsics


def _dev_f32(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    return t.contiguous().float()


def workspace_for(batch, channels, h, w, device):
    n = _lib.load().sfm_correlation_workspace_bytes(int(batch), int(channels), int(h), int(w))
    return torch.empty(int(n), dtype=torch.uint8, device=device)


def correlation_cost(ref_fea, tgt_fea, pose, intrinsics4, intrinsics_inv4, nlabel, min_depth=1.0,
                     predict_by_depth=False, out=None, workspace=None):
    """[B, L, h, w] float32 cost; pose [B,3,4] (already rescaled), feature-resolution intrinsics."""
    ref = _dev_f32(ref_fea, "ref_fea")
    tgt = _dev_f32(tgt_fea, "tgt_fea")
    B, C, h, w = tgt.shape
    if tuple(ref.shape) != (B, C, h, w):
        raise RuntimeError(f"ref_fea shape {tuple(ref.shape)} != tgt_fea shape {(B, C, h, w)}")
    pose = _dev_f32(pose.reshape(B, 3, 4), "pose")
    K4 = _dev_f32(intrinsics4.reshape(B, 3, 3), "intrinsics")
    Ki4 = _dev_f32(intrinsics_inv4.reshape(B, 3, 3), "intrinsics_inv")
    shape = (B, int(nlabel), h, w)
    if out is None:
        out = torch.empty(shape, dtype=torch.float32, device=tgt.device)
    elif tuple(out.shape) != shape or out.dtype != torch.float32 or not out.is_contiguous():
        raise RuntimeError(f"out must be a contiguous float32 tensor of shape {shape}")
    if workspace is None:
        workspace = workspace_for(B, C, h, w, tgt.device)
    with torch.cuda.device(tgt.device):
        rc = _lib.load().sfm_plane_sweep_correlation(
            _lib.ptr(ref), _lib.ptr(tgt), B, C, h, w, _lib.ptr(pose), _lib.ptr(K4), _lib.ptr(Ki4), int(nlabel),
            float(min_depth), 1 if predict_by_depth else 0, _lib.ptr(out), _lib.ptr(workspace), workspace.numel(),
            _lib.stream_ptr(tgt.device))
        _lib.check(rc, "sfm_plane_sweep_correlation")
    return out


def depth_head(cost, nlabel, min_depth=1.0, out_hw=None, predict_by_depth=False, out=None, scale=None):
    """Soft-argmin depth [B, 1, H, W] float32 from a cost [B, L, h, w] / [B, 1, L, h, w].
    ``scale`` (predict_by_depth only) replaces the final ``* min_depth``: PSNet's
    depth_init is depthregression's output without it (PSNet.py:200-202)."""
    c = _dev_f32(cost, "cost")
    if c.dim() == 5:
        if c.shape[1] != 1:
            raise RuntimeError("a 5-D cost must have one channel (the classify output)")
        c = c[:, 0]
    B, L, h, w = c.shape
    if L != int(nlabel):
        raise RuntimeError(f"cost has {L} planes, nlabel is {nlabel}")
    H, W = (h, w) if out_hw is None else (int(out_hw[0]), int(out_hw[1]))
    step = 0.0
    if predict_by_depth:
        step = float(int(min_depth))        # depthregression: depth_inter = int(cfg.MIN_DEPTH)
        if step <= 0:
            raise RuntimeError("PREDICT_BY_DEPTH needs MIN_DEPTH >= 1 (submodule.py:85-87)")
    if out is None:
        out = torch.empty(B, 1, H, W, dtype=torch.float32, device=c.device)
    with torch.cuda.device(c.device):
        mul = float(min_depth) if (scale is None or not predict_by_depth) else float(scale)
        rc = _lib.load().sfm_depth_head(_lib.ptr(c), B, L, h, w, H, W, 1 if predict_by_depth else 0,
                                        mul, step, _lib.ptr(out), _lib.stream_ptr(c.device))
        _lib.check(rc, "sfm_depth_head")
    return out


class CorrelationDepth(torch.nn.Module):
    """Parameter-free two-view depth: correlation cost over the planes of
    PSNet's sweep (quarter intrinsics, optional RESCALE_DEPTH) + the
    soft-argmin head at image resolution."""

    def __init__(self, nlabel, mindepth=1.0, rescale_depth=False, norm_target=0.8, predict_by_depth=False):
        super().__init__()
        self.nlabel = int(nlabel)
        self.mindepth = float(mindepth)
        self.rescale_depth = rescale_depth
        self.norm_target = norm_target
        self.predict_by_depth = predict_by_depth

    def forward(self, ref_fea, tgt_fea, pose, intrinsics, intrinsics_inv, out_hw):
        K4, Ki4 = quarter_intrinsics(intrinsics, intrinsics_inv)
        pose = pose.clone()
        if self.rescale_depth:
            pose[:, :, -1:] = pose[:, :, -1:] * self.norm_target
        cost = correlation_cost(ref_fea, tgt_fea, pose, K4, Ki4, self.nlabel, self.mindepth, self.predict_by_depth)
        return depth_head(cost, self.nlabel, self.mindepth, out_hw, self.predict_by_depth)


class SweepDepthEstimator(torch.nn.Module):
    """Drop-in ``depth_estimator`` for SFMnet with PSNet's call signature
    (PSNet.forward(ref, targets, pose, intrinsics, intrinsics_inv, ...),
    PSNet.py:128) and return value (depth_init, depth), parameter-free:
    features = ``feature_fn(image)`` at quarter resolution (default: 4x4 average
    pooling, matching PSNet's two stride-2 stages), the correlation cost over
    the sweep planes averaged over target views (PSNet.py:166-170), and the
    soft-argmin head at image resolution.  RESCALE_DEPTH scales pose[:, 0] in
    place, as PSNet.py:135-136 does."""

    def __init__(self, nlabel, mindepth=1.0, rescale_depth=False, norm_target=0.8, predict_by_depth=False,
                 feature_fn=None):
        super().__init__()
        self.nlabel = int(nlabel)
        self.mindepth = float(mindepth)
        self.rescale_depth = rescale_depth
        self.norm_target = norm_target
        self.predict_by_depth = predict_by_depth
        self.feature_fn = feature_fn or (lambda x: torch.nn.functional.avg_pool2d(x.float(), 4))

    def forward(self, ref, targets, pose, intrinsics, intrinsics_inv, pose_gt=None, depth_gt=None, E_mat=None):
        K4, Ki4 = quarter_intrinsics(intrinsics.float(), intrinsics_inv.float())
        if self.rescale_depth:
            pose[:, 0, :, -1:] = pose[:, 0, :, -1:] * self.norm_target
        ref_fea = self.feature_fn(ref)
        cost = None
        for j, target in enumerate(targets):
            c = correlation_cost(ref_fea, self.feature_fn(target), pose[:, j], K4, Ki4, self.nlabel, self.mindepth,
                                 self.predict_by_depth)
            cost = c if cost is None else cost + c
        cost = cost / len(targets)
        depth = depth_head(cost, self.nlabel, self.mindepth, (ref.shape[2], ref.shape[3]), self.predict_by_depth)
        return depth, depth


def flow2depth(R, T, initial_flow, K_mat):
    """Flow2Depth(R, T, initial_flow, K_mat) of models/flow2depth.py:7-41 ->
    [B, H, W] float32 on the flow's device.  The flow is read for its shape
    only, as in the reference.  K^-1 is numpy's inverse of K (float32, as
    the reference computes it on the host); K.R and K.T are torch matmuls.
    Unlike the reference (whose pixel loop only works for B = 1) any batch
    size is accepted, each pair with its own K."""
    import numpy as np
    B, _, H, W = initial_flow.shape
    dev = initial_flow.device
    if not initial_flow.is_cuda:
        raise RuntimeError("flow2depth needs a device flow tensor (HIP path, no CPU fallback)")
    Kd = K_mat.to(dev, torch.float32).reshape(B, 3, 3)
    KR = torch.matmul(Kd, R.to(dev, torch.float32).reshape(B, 3, 3)).contiguous()
    KT = torch.matmul(Kd, T.to(dev, torch.float32).reshape(B, 3, 1)).reshape(B, 3).contiguous()
    Ki = torch.from_numpy(np.linalg.inv(K_mat.detach().cpu().numpy().reshape(B, 3, 3))).to(dev, torch.float32)
    out = torch.empty(B, H, W, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.load().sfm_flow2depth(_lib.ptr(KR), _lib.ptr(KT), _lib.ptr(Ki.contiguous()), B, H, W,
                                        _lib.ptr(out), _lib.stream_ptr(dev))
        _lib.check(rc, "sfm_flow2depth")
    return out
