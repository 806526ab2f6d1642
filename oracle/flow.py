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
