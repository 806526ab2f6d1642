"""ORACLE (test infrastructure only): torch-CPU fp32 restatement of the
plane-sweep stage.

* ``inverse_warp``      — models/inverse_warp.py:121-153 (+ pixel2cam 27-41,
  cam2pixel 44-75): back-project with K^-1, scale by depth, transform with
  K.[R|t], perspective divide with Z clamped at 1e-3, normalise to [-1,1],
  push out-of-range coordinates to 2, bilinear grid_sample with zero padding
  and align_corners=True.
* ``plane_sweep_cost``  — models/PSNet.py:130-158: K/4 (rows 0-1), K^-1 with
  [:2,:2]*4, optional RESCALE_DEPTH translation scaling, planes
  d_i = MIN_DEPTH*L / (i+1), cost[:, :C, i] = ref, cost[:, C:, i] = warped.
* ``flow2depth``        — models/flow2depth.py:7-41, including its
  reinterpretation of the [B, H*W, 3] result as [B, 3, H, W].
* ``depth_head``        — PSNet.py:194-216 + submodule.py:57-80 (softmax over
  planes, disparity regression, depth = MIN_DEPTH*L/disp) for a cost [B,L,H,W].
"""
import numpy as np
import torch
import torch.nn.functional as F


def _pixel_grid(h, w, dtype=torch.float32):
    ys = torch.arange(h, dtype=dtype).view(h, 1).expand(h, w)
    xs = torch.arange(w, dtype=dtype).view(1, w).expand(h, w)
    return torch.stack([xs, ys, torch.ones(h, w, dtype=dtype)], 0).reshape(1, 3, h * w)


def warp_grid(depth, pose, K, Kinv, h, w):
    """Sampling grid [B,h,w,2] in [-1,1] (out-of-range -> 2)."""
    b = depth.shape[0]
    pix = _pixel_grid(h, w).expand(b, 3, h * w).contiguous()
    cam = Kinv.bmm(pix) * depth.reshape(b, 1, h * w)
    proj = K.bmm(pose)
    pc = proj[:, :, :3].bmm(cam) + proj[:, :, 3:]
    X, Y = pc[:, 0], pc[:, 1]
    Z = pc[:, 2].clamp(min=1e-3)
    xn = 2 * (X / Z) / (w - 1) - 1
    yn = 2 * (Y / Z) / (h - 1) - 1
    xn = torch.where((xn > 1) | (xn < -1), torch.full_like(xn, 2.0), xn)
    yn = torch.where((yn > 1) | (yn < -1), torch.full_like(yn, 2.0), yn)
    return torch.stack([xn, yn], 2).reshape(b, h, w, 2)


def inverse_warp(feat, depth, pose, K, Kinv):
    b, c, h, w = feat.shape
    grid = warp_grid(depth, pose, K, Kinv, h, w)
    return F.grid_sample(feat, grid, mode="bilinear", padding_mode="zeros", align_corners=True)


def quarter_intrinsics(K, Kinv):
    K4 = K.clone()
    Ki4 = Kinv.clone()
    K4[:, :2, :] = K4[:, :2, :] / 4
    Ki4[:, :2, :2] = Ki4[:, :2, :2] * 4
    return K4, Ki4


def plane_sweep_cost(ref_fea, tgt_fea, pose, K, Kinv, nlabel, min_depth=1.0, rescale=None,
                     planes=None, predict_by_depth=False):
    """Cost volume [B, 2C, L, h, w] (fp32).  ``pose`` [B,3,4]; K, Kinv are the
    full-resolution intrinsics (quartered here as PSNet does).  ``rescale``:
    NORM_TARGET factor applied to the translation (RESCALE_DEPTH) or None.
    ``planes``: optional subset of plane indices (for bounded CPU baselines).
    ``predict_by_depth``: cfg.PREDICT_BY_DEPTH planes (PSNet.py:150-151)."""
    K4, Ki4 = quarter_intrinsics(K, Kinv)
    pose = pose.clone()
    if rescale is not None:
        pose[:, :, 3:] = pose[:, :, 3:] * rescale
    b, c, h, w = ref_fea.shape
    planes = list(range(nlabel)) if planes is None else list(planes)
    ones = torch.ones(b, h, w)
    disp2depth = ones * min_depth * nlabel
    cost = torch.zeros(b, 2 * c, len(planes), h, w)
    for s, i in enumerate(planes):
        if predict_by_depth:
            depth = ones * (i + 1) * min_depth                 # PSNet.py:151
        else:
            depth = torch.div(disp2depth, i + 1 + 1e-16)       # PSNet.py:153
        cost[:, :c, s] = ref_fea
        cost[:, c:, s] = inverse_warp(tgt_fea, depth, pose, K4, Ki4)
    return cost


def flow2depth(R, T, flow, K):
    """models/flow2depth.py:7-41 restated (B must be 1, as in the reference)."""
    B, _, H, W = flow.shape
    Ki = np.linalg.inv(K.numpy()).reshape(3, 3)
    jj, ii = np.meshgrid(np.arange(W), np.arange(H))
    pix = np.stack([jj, ii, np.ones_like(jj)], -1).reshape(H * W, 3).astype(np.float64)
    dirs = (pix @ Ki.T).astype(np.float32).reshape(H * W, 3, 1)
    first = torch.matmul(torch.matmul(K, R).view(B, 1, 3, 3), torch.from_numpy(dirs))
    second = torch.matmul(K, T.unsqueeze(-1)).view(B, 1, 3, 1).expand(-1, H * W, -1, -1)
    out = (first + second).reshape(B, -1, H, W)
    return out[:, -1, :, :]


def correlation_cost(ref_fea, tgt_fea, pose, K, Kinv, nlabel, min_depth=1.0, rescale=None,
                     predict_by_depth=False):
    """Parameter-free correlation cost of REG2D.py:103-109 (before its
    leaky_relu): cost[:, i] = (ref * inverse_warp(tgt, d_i)).mean(1) with
    quarter intrinsics; [B, L, h, w] fp32."""
    K4, Ki4 = quarter_intrinsics(K, Kinv)
    pose = pose.clone()
    if rescale is not None:
        pose[:, :, 3:] = pose[:, :, 3:] * rescale
    b, c, h, w = ref_fea.shape
    ones = torch.ones(b, h, w)
    disp2depth = ones * min_depth * nlabel
    cost = torch.zeros(b, nlabel, h, w)
    for i in range(nlabel):
        depth = ones * (i + 1) * min_depth if predict_by_depth else torch.div(disp2depth, i + 1 + 1e-16)
        cost[:, i] = (ref_fea * inverse_warp(tgt_fea, depth, pose, K4, Ki4)).mean(dim=1)
    return cost


def depth_head(cost, nlabel, min_depth=1.0, out_hw=None, predict_by_depth=False):
    """Soft-argmin head of PSNet.py:191-213 on a cost [B, L, h, w] (or
    [B, 1, L, h, w]): trilinear upsample to [L, H, W] (align_corners=False),
    softmax over planes, disparityregression / depthregression
    (submodule.py:57-93) -> depth [B, 1, H, W]."""
    if cost.dim() == 4:
        cost = cost.unsqueeze(1)
    B, _, L, h, w = cost.shape
    H, W = (h, w) if out_hw is None else out_hw
    up = F.interpolate(cost, [nlabel, H, W], mode="trilinear")
    prob = F.softmax(torch.squeeze(up, 1), dim=1)
    if predict_by_depth:
        step = int(min_depth)
        vals = torch.Tensor(np.reshape(np.array(range(1 * step, step * (nlabel + 1), step)), [1, nlabel, 1, 1]))
        pred = torch.sum(prob * vals.expand(B, -1, H, W), 1)
        return pred.unsqueeze(1) * min_depth
    disp = torch.Tensor(np.reshape(np.array(range(1, nlabel + 1)), [1, nlabel, 1, 1]))
    pred = torch.sum(prob * disp.expand(B, -1, H, W), 1)
    return min_depth * nlabel / (pred.unsqueeze(1) + 1e-16)