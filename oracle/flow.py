"""ORACLE (test infrastructure only): restatement of the dense-flow
correspondence build that feeds the RANSAC (models/SFMnet.py:176-263 with
flow2coord 298-318, dense branch 239-241, K^-1 bmm 259-263, .double() in
epipolar_utils.py:130).

Per pixel (u, v) inside the margin of the h_side x w_side crop:
    coord1 = (u, v, 1),  coord2 = (u + flow_u, v + flow_v, 1)      (fp32)
    q  = (K^-1 coord1)[:2],  qp = (K^-1 coord2)[:2]                  (fp32)
with each row evaluated as (k0*x + k1*y) + k2 in fp32 (the order the HIP
kernel uses; the reference's sgemm order may differ by 1 fp32 ulp), then
widened to fp64.  Row-major pixel order (v outer, u inner) gives index k.
"""
import numpy as np


def dense_correspondences(flow, Kinv, h_side=None, w_side=None, margin=10):
    """flow: [B,2,H,W] float32 ndarray; Kinv: [B,3,3] float32.
    Returns q, qp: [B, N, 2] float64 with N = (h-2m)(w-2m)."""
    flow = np.asarray(flow, dtype=np.float32)
    Kinv = np.asarray(Kinv, dtype=np.float32)
    B, _, H, W = flow.shape
    h = H if h_side is None else h_side
    w = W if w_side is None else w_side
    fl = flow[:, :, :h, :w]
    vs, us = np.meshgrid(np.arange(margin, h - margin, dtype=np.float32),
                         np.arange(margin, w - margin, dtype=np.float32), indexing="ij")
    u1 = np.broadcast_to(us, (B,) + us.shape)
    v1 = np.broadcast_to(vs, (B,) + vs.shape)
    u2 = (u1 + fl[:, 0, margin:h - margin, margin:w - margin]).astype(np.float32)
    v2 = (v1 + fl[:, 1, margin:h - margin, margin:w - margin]).astype(np.float32)

    def apply(u, v):
        k = Kinv[:, None, None, :, :]
        out = []
        for r in range(2):
            a = (k[..., r, 0] * u).astype(np.float32)
            b = (k[..., r, 1] * v).astype(np.float32)
            out.append(((a + b).astype(np.float32) + k[..., r, 2]).astype(np.float32))
        return np.stack(out, -1).reshape(B, -1, 2).astype(np.float64)

    return apply(u1, v1), apply(u2, v2)


def _apply_kinv(Kinv, c):
    """rows (k0*x + k1*y) + k2*z in fp32 (c: [n, 3] float32) -> [n, 2] float64."""
    out = []
    for r in range(2):
        a = (Kinv[r, 0] * c[:, 0]).astype(np.float32)
        b = (Kinv[r, 1] * c[:, 1]).astype(np.float32)
        z = (Kinv[r, 2] * c[:, 2]).astype(np.float32)
        out.append(((a + b).astype(np.float32) + z).astype(np.float32))
    return np.stack(out, -1).astype(np.float64)


def keypoint_correspondences(flow, Kinv, kp1, kp2=None, mode="round", h_side=None, w_side=None):
    """Sparse branch of SFMnet.pose_by_ransac (models/SFMnet.py:218-258) for one
    pair: flow [2,H,W] float32, Kinv [3,3] float32, kp [n,2] pixel (x, y).
    mode "round": coord[:, round(y), round(x)]; "sample_sp": F.grid_sample of the
    coordinate grids (align_corners=True); "sift_pose": the keypoints.
    Returns q, qp [n, 2] float64."""
    import torch
    import torch.nn.functional as F
    flow = np.asarray(flow, dtype=np.float32)
    Kinv = np.asarray(Kinv, dtype=np.float32)
    if mode == "sift_pose":
        c1 = np.c_[np.asarray(kp1, np.float32), np.ones(len(kp1), np.float32)]
        c2 = np.c_[np.asarray(kp2, np.float32), np.ones(len(kp2), np.float32)]
        return _apply_kinv(Kinv, c1), _apply_kinv(Kinv, c2)
    H, W = flow.shape[1:]
    h = H if h_side is None else h_side
    w = W if w_side is None else w_side
    fl = torch.from_numpy(flow[None, :, :h, :w].copy())
    c1 = torch.zeros_like(fl)
    c1[:, 0] += torch.arange(w).float()
    c1[:, 1] += torch.arange(h).float()[:, None]
    c2 = c1 + fl
    ones = torch.ones(1, 1, h, w)
    g1 = torch.cat((c1, ones), 1)
    g2 = torch.cat((c2, ones), 1)
    if mode == "round":
        p = np.int32(np.round(np.asarray(kp1, np.float64)))
        s1 = g1[0, :, p[:, 1], p[:, 0]].T.numpy()
        s2 = g2[0, :, p[:, 1], p[:, 0]].T.numpy()
    else:
        p = torch.from_numpy(np.asarray(kp1, np.float64)).float()
        p[:, 0] = 2.0 * p[:, 0] / max(w - 1, 1) - 1.0
        p[:, 1] = 2.0 * p[:, 1] / max(h - 1, 1) - 1.0
        s1 = F.grid_sample(g1, p[None, :, None, :], align_corners=True)[0, :, :, 0].T.numpy()
        s2 = F.grid_sample(g2, p[None, :, None, :], align_corners=True)[0, :, :, 0].T.numpy()
    return _apply_kinv(Kinv, s1.astype(np.float32)), _apply_kinv(Kinv, s2.astype(np.float32))
