"""Seeded synthetic KITTI-shaped two-view inputs.

No dataset or checkpoint is reachable offline, so every workload is
generated: a smooth random depth field in [MIN_DEPTH, L*MIN_DEPTH], a mostly
forward relative pose (|t| 0.8-1.5 m, rotation <= 2 deg), the rigid flow it
induces through the KITTI intrinsics, N(0, sigma) pixel noise and a fraction
of uniformly random outlier flows; plane-sweep features are N(0,1).
"""
import math

import torch
import torch.nn.functional as F

KITTI_K = (721.5377, 721.5377, 609.5593, 172.854)   # fx, fy, cx, cy
KITTI_HW = (376, 1242)


def intrinsics(batch, fx=KITTI_K[0], fy=KITTI_K[1], cx=KITTI_K[2], cy=KITTI_K[3], device="cpu"):
    K = torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=torch.float32)
    return K.unsqueeze(0).repeat(batch, 1, 1).to(device)


def _rotation(axis, angle):
    a = axis / axis.norm()
    K = torch.tensor([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]], dtype=torch.float64)
    return torch.eye(3, dtype=torch.float64) + math.sin(angle) * K + (1 - math.cos(angle)) * (K @ K)


def relative_pose(batch, gen, max_rot_deg=2.0, t_range=(0.8, 1.5)):
    """[B,3,4] float32 poses X2 = R X1 + t (camera moving mostly forward)."""
    out = torch.zeros(batch, 3, 4, dtype=torch.float64)
    for b in range(batch):
        axis = torch.randn(3, generator=gen, dtype=torch.float64)
        ang = math.radians(max_rot_deg) * float(torch.rand(1, generator=gen, dtype=torch.float64))
        R = _rotation(axis, ang)
        d = torch.tensor([0.1, 0.05, 1.0], dtype=torch.float64) * torch.randn(3, generator=gen, dtype=torch.float64)
        d[2] = 1.0
        mag = t_range[0] + (t_range[1] - t_range[0]) * float(torch.rand(1, generator=gen, dtype=torch.float64))
        out[b, :, :3] = R
        out[b, :, 3] = -mag * d / d.norm()
    return out.float()


def depth_field(batch, h, w, gen, min_depth=1.0, max_depth=128.0, coarse=(6, 20)):
    """Smooth random depth in [min_depth, max_depth] (log-uniform coarse grid, bilinear up)."""
    lo, hi = math.log(min_depth), math.log(max_depth)
    g = lo + (hi - lo) * torch.rand(batch, 1, coarse[0], coarse[1], generator=gen)
    up = F.interpolate(g, size=(h, w), mode="bilinear", align_corners=True)
    return up[:, 0].exp().clamp(min_depth, max_depth)


def rigid_flow(depth, pose, K):
    """Flow [B,2,H,W] induced by depth [B,H,W] and pose [B,3,4] (float64 math)."""
    B, H, W = depth.shape
    K = K.double()
    Ki = torch.inverse(K)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float64), torch.arange(W, dtype=torch.float64),
                            indexing="ij")
    pix = torch.stack([xs, ys, torch.ones_like(xs)], 0).reshape(1, 3, -1)
    X = (Ki @ pix) * depth.double().reshape(B, 1, -1)
    X2 = pose[:, :, :3].double() @ X + pose[:, :, 3:].double()
    p2 = K @ X2
    z = p2[:, 2:].clamp(min=1e-6)
    uv = p2[:, :2] / z
    flow = (uv - pix[:, :2]).reshape(B, 2, H, W)
    behind = (X2[:, 2] <= 0.1).reshape(B, H, W)
    return flow, behind


INDOOR_K = (518.86, 519.47, 325.58, 253.74)   # 640x480 (NYU/ScanNet-like; DeMoN-style indoor pairs)
INDOOR_HW = (480, 640)


def kitti_pair_batch(batch, seed=0, hw=KITTI_HW, noise_px=0.5, outlier_frac=0.15, device="cpu", k=None):
    """Synthetic (flow [B,2,H,W] f32, K [B,3,3] f32, pose_gt [B,3,4] f32, depth [B,H,W] f32).
    ``k`` = (fx, fy, cx, cy) (default: KITTI)."""
    gen = torch.Generator().manual_seed(int(seed))
    H, W = hw
    K = intrinsics(batch) if k is None else intrinsics(batch, *k)
    pose = relative_pose(batch, gen)
    depth = depth_field(batch, H, W, gen)
    flow, behind = rigid_flow(depth, pose, K)
    flow = flow + noise_px * torch.randn(flow.shape, generator=gen, dtype=torch.float64)
    out = torch.rand(batch, H, W, generator=gen) < outlier_frac
    out = out | behind
    rnd = (torch.rand(batch, 2, H, W, generator=gen, dtype=torch.float64) - 0.5) * 100.0
    flow = torch.where(out.unsqueeze(1), rnd, flow)
    return (flow.float().to(device), K.to(device), pose.to(device), depth.float().to(device))


def features(batch, channels, h, w, seed=0, device="cpu"):
    """Plane-sweep features ~ N(0,1): (ref_fea, tgt_fea) [B,C,h,w] float32."""
    gen = torch.Generator().manual_seed(int(seed) + 7919)
    ref = torch.randn(batch, channels, h, w, generator=gen)
    tgt = torch.randn(batch, channels, h, w, generator=gen)
    return ref.to(device), tgt.to(device)


def feature_hw(hw=KITTI_HW):
    """Feature-map size after the two stride-2 convs of PSNet's feature CNN (submodule.py:112,120)."""
    h, w = hw
    return ((h + 1) // 2 + 1) // 2, ((w + 1) // 2 + 1) // 2   # 376x1242 -> 94x311


def keypoints(batch, n, hw=KITTI_HW, margin=10, seed=0, device="cpu"):
    """Sparse (SIFT-like) keypoints for the bench's sparse regime (SURVEY.md
    §8(d): N=2,048 random pixels per pair): [B, n, 2] float32 (x, y) pixel
    positions, already rounded to integers as SFMnet.py:250-253 does."""
    gen = torch.Generator().manual_seed(int(seed) + 104729)
    H, W = hw
    x = torch.randint(margin, W - margin, (batch, n), generator=gen)
    y = torch.randint(margin, H - margin, (batch, n), generator=gen)
    return torch.stack([x, y], -1).float().to(device)
