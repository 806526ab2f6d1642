"""Plane-sweep stage over the C ABI.

* ``plane_sweep_cost`` — replaces the per-plane loop of models/PSNet.py:144-157
  (cost[:, :C, i] = ref, cost[:, C:, i] = inverse_warp(tgt, d_i)) with one
  kernel launch.
* ``inverse_warp``     — drop-in for models/inverse_warp.py:121-153.
* ``PlaneSweep``       — the sweep section of PSNet.forward (PSNet.py:130-158):
  K/4 rows 0-1, K^-1[:2,:2]*4, optional RESCALE_DEPTH translation scaling (in
  place on the caller's pose tensor, as the reference does), one cost volume
  per target view.
"""
import torch

from . import _lib


def _dev_f32(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    return t.contiguous().float()


def _refuse_grad(**tensors):
    """The sweep kernels are forward-only: they return tensors with no autograd
    link.  The reference backpropagates through grid_sample into the target
    features (models/PSNet.py:155), so a grad-requiring input would silently
    lose its gradient here -- refuse it instead."""
    if not torch.is_grad_enabled():
        return
    for name, t in tensors.items():
        if t is not None and t.requires_grad:
            raise RuntimeError(f"{name} requires grad, but the HIP plane sweep is forward-only (no backward "
                               f"kernel); run it under torch.no_grad() or detach the input")


def check_sizes(t, name, expected):
    """models/inverse_warp.py:19-24"""
    ok = t.dim() == len(expected) and all(
        (not s.isdigit()) or t.size(i) == int(s) for i, s in enumerate(expected))
    assert ok, "wrong size for {}, expected {}, got  {}".format(name, "x".join(expected), list(t.size()))


def workspace_for(batch, channels, h, w, device):
    """Reusable plane-sweep scratch (channel-quad copy of the target features)."""
    n = _lib.load().sfm_plane_sweep_workspace_bytes(int(batch), int(channels), int(h), int(w))
    return torch.empty(int(n), dtype=torch.uint8, device=device)


def plane_sweep_cost(ref_fea, tgt_fea, pose, intrinsics4, intrinsics_inv4, nlabel, min_depth=1.0,
                     dtype=torch.float32, out=None, warped_only=False, workspace=None, predict_by_depth=False):
    """Cost volume [B, 2C, L, h, w] (or [B, C, L, h, w] with warped_only).
    ``pose`` [B,3,4] (already translation-rescaled), intrinsics at feature
    resolution.  ``dtype``: torch.float32 or torch.bfloat16.  Planes are
    d_i = MIN_DEPTH*L/(i+1), or (i+1)*MIN_DEPTH with ``predict_by_depth``
    (cfg.PREDICT_BY_DEPTH, PSNet.py:150-153)."""
    _refuse_grad(ref_fea=None if warped_only else ref_fea, tgt_fea=tgt_fea, pose=pose,
                 intrinsics4=intrinsics4, intrinsics_inv4=intrinsics_inv4)
    tgt = _dev_f32(tgt_fea, "tgt_fea")
    B, C, h, w = tgt.shape
    ref = None if warped_only else _dev_f32(ref_fea, "ref_fea")
    if ref is not None and tuple(ref.shape) != (B, C, h, w):
        raise RuntimeError(f"ref_fea shape {tuple(ref.shape)} != tgt_fea shape {(B, C, h, w)}")
    pose = _dev_f32(pose.reshape(B, 3, 4), "pose")
    K4 = _dev_f32(intrinsics4.reshape(B, 3, 3), "intrinsics")
    Ki4 = _dev_f32(intrinsics_inv4.reshape(B, 3, 3), "intrinsics_inv")
    if dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError("cost dtype must be float32 or bfloat16")
    cout = C if warped_only else 2 * C
    shape = (B, cout, int(nlabel), h, w)
    if out is None:
        out = torch.empty(shape, dtype=dtype, device=tgt.device)
    elif tuple(out.shape) != shape or out.dtype != dtype or not out.is_contiguous() or out.device != tgt.device:
        raise RuntimeError(f"out must be a contiguous {dtype} tensor of shape {shape} on {tgt.device}")
    code = 0 if dtype == torch.float32 else 1
    L = _lib.load()
    if workspace is None:
        workspace = workspace_for(B, C, h, w, tgt.device)
    with torch.cuda.device(tgt.device):
        rc = L.sfm_plane_sweep_ex(None if ref is None else _lib.ptr(ref), _lib.ptr(tgt), B, C, h, w, _lib.ptr(pose),
                                  _lib.ptr(K4), _lib.ptr(Ki4), int(nlabel), float(min_depth),
                                  1 if predict_by_depth else 0, code, _lib.ptr(out), _lib.ptr(workspace),
                                  workspace.numel(), _lib.stream_ptr(tgt.device))
        _lib.check(rc, "sfm_plane_sweep")
    return out


def ref_planes_workspace_for(B, C, h, w, device):
    n = _lib.load().sfm_plane_sweep_ref_planes_workspace_bytes(B, C, h, w)
    return torch.empty(n, dtype=torch.uint8, device=device)


def plane_sweep_ref_half(ref_fea, nlabel, out, workspace=None):
    """The pose-independent reference half of the cost volume, cost[:, :C, i] =
    ref for every plane (PSNet.py:155), into ``out`` [B, 2C, L, h, w]
    (sfm_plane_sweep_ref_planes; typically on a side stream beside RANSAC)."""
    ref = _dev_f32(ref_fea, "ref_fea")
    B, C, h, w = ref.shape
    if tuple(out.shape) != (B, 2 * C, int(nlabel), h, w) or not out.is_contiguous() or \
            out.dtype not in (torch.float32, torch.bfloat16) or out.device != ref.device:
        raise RuntimeError(f"out must be a contiguous float32/bfloat16 tensor of shape {(B, 2 * C, int(nlabel), h, w)}")
    if workspace is None:
        workspace = ref_planes_workspace_for(B, C, h, w, ref.device)
    with torch.cuda.device(ref.device):
        rc = _lib.load().sfm_plane_sweep_ref_planes(_lib.ptr(ref), B, C, h, w, int(nlabel),
                                                    0 if out.dtype == torch.float32 else 1, _lib.ptr(out),
                                                    _lib.ptr(workspace), workspace.numel(),
                                                    _lib.stream_ptr(ref.device))
        _lib.check(rc, "sfm_plane_sweep_ref_planes")
    return out


def plane_sweep_cost_psnet(ref_fea, tgt_fea, pose, intrinsics, intrinsics_inv, nlabel, min_depth=1.0,
                           rescale=None, dtype=torch.float32, out=None, workspace=None, predict_by_depth=False,
                           warped_half=False):
    """``plane_sweep_cost`` from the pose stage's outputs: ``pose`` [B,3,4]
    float32 or float64 (unscaled), full-resolution ``intrinsics`` /
    ``intrinsics_inv`` [B,3,3].  PSNet.forward's preparation (P.float(),
    RESCALE_DEPTH translation * ``rescale``, K/4 rows 0-1, K^-1[:2,:2]*4;
    PSNet.py:130-133) runs inside the call (sfm_plane_sweep_psnet), with the
    same float32 bits as ``quarter_intrinsics`` + ``plane_sweep_cost``.  Unlike
    PlaneSweep it does not rescale the caller's pose in place.  ``warped_half``:
    leave the reference rows to ``plane_sweep_ref_half``
    (sfm_plane_sweep_psnet_warped_half)."""
    _refuse_grad(ref_fea=ref_fea, tgt_fea=tgt_fea, pose=pose, intrinsics=intrinsics, intrinsics_inv=intrinsics_inv)
    tgt = _dev_f32(tgt_fea, "tgt_fea")
    B, C, h, w = tgt.shape
    ref = _dev_f32(ref_fea, "ref_fea")
    if tuple(ref.shape) != (B, C, h, w):
        raise RuntimeError(f"ref_fea shape {tuple(ref.shape)} != tgt_fea shape {(B, C, h, w)}")
    if not pose.is_cuda:
        raise RuntimeError("pose must be a CUDA tensor")
    P = pose.reshape(B, 3, 4).contiguous()
    if P.dtype not in (torch.float32, torch.float64):
        P = P.float()
    K = _dev_f32(intrinsics.reshape(B, 3, 3), "intrinsics")
    Ki = _dev_f32(intrinsics_inv.reshape(B, 3, 3), "intrinsics_inv")
    if dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError("cost dtype must be float32 or bfloat16")
    shape = (B, 2 * C, int(nlabel), h, w)
    if out is None:
        out = torch.empty(shape, dtype=dtype, device=tgt.device)
    elif tuple(out.shape) != shape or out.dtype != dtype or not out.is_contiguous() or out.device != tgt.device:
        raise RuntimeError(f"out must be a contiguous {dtype} tensor of shape {shape} on {tgt.device}")
    L = _lib.load()
    if workspace is None:
        workspace = workspace_for(B, C, h, w, tgt.device)
    fn = L.sfm_plane_sweep_psnet_warped_half if warped_half else L.sfm_plane_sweep_psnet
    with torch.cuda.device(tgt.device):
        rc = fn(_lib.ptr(ref), _lib.ptr(tgt), B, C, h, w, _lib.ptr(P),
                                     1 if P.dtype == torch.float64 else 0, _lib.ptr(K), _lib.ptr(Ki),
                                     float(rescale) if rescale is not None else 0.0, int(nlabel), float(min_depth),
                                     1 if predict_by_depth else 0, 0 if dtype == torch.float32 else 1,
                                     _lib.ptr(out), _lib.ptr(workspace), workspace.numel(),
                                     _lib.stream_ptr(tgt.device))
        _lib.check(rc, "sfm_plane_sweep_psnet_warped_half" if warped_half else "sfm_plane_sweep_psnet")
    return out


def inverse_warp(feat, depth, pose, intrinsics, intrinsics_inv, padding_mode="zeros"):
    """models/inverse_warp.py:121-153 (bilinear, zeros padding, align_corners=True)."""
    check_sizes(depth, "depth", "BHW")
    check_sizes(pose, "pose", "B34")
    check_sizes(intrinsics, "intrinsics", "B33")
    check_sizes(intrinsics_inv, "intrinsics", "B33")
    assert intrinsics_inv.size() == intrinsics.size()
    if padding_mode != "zeros":
        raise NotImplementedError("only padding_mode='zeros' is on the plane-sweep path")
    _refuse_grad(feat=feat, depth=depth, pose=pose, intrinsics=intrinsics, intrinsics_inv=intrinsics_inv)
    f = _dev_f32(feat, "feat")
    B, C, h, w = f.shape
    if tuple(depth.shape) != (B, h, w) or pose.size(0) != B or intrinsics.size(0) != B:
        raise RuntimeError(f"inverse_warp: depth {tuple(depth.shape)}, pose {tuple(pose.shape)} and intrinsics "
                           f"{tuple(intrinsics.shape)} must match feat {(B, C, h, w)}")
    # every converted operand is bound to a local until the launch is enqueued:
    # a temporary freed inside the call could be handed to the next copy
    d = _dev_f32(depth, "depth")
    pose32 = _dev_f32(pose, "pose")
    K32 = _dev_f32(intrinsics, "intrinsics")
    Ki32 = _dev_f32(intrinsics_inv, "intrinsics_inv")
    out = torch.empty_like(f)
    with torch.cuda.device(f.device):
        rc = _lib.load().sfm_inverse_warp(_lib.ptr(f), B, C, h, w, _lib.ptr(d), _lib.ptr(pose32), _lib.ptr(K32),
                                          _lib.ptr(Ki32), _lib.ptr(out), _lib.stream_ptr(f.device))
        _lib.check(rc, "sfm_inverse_warp")
    return out


def quarter_intrinsics(intrinsics, intrinsics_inv):
    """PSNet.py:130-133: K/4 on rows 0-1; K^-1 with [:2,:2]*4."""
    K4 = intrinsics.clone()
    Ki4 = intrinsics_inv.clone()
    K4[:, :2, :] = K4[:, :2, :] / 4
    Ki4[:, :2, :2] = Ki4[:, :2, :2] * 4
    return K4, Ki4


class PlaneSweep(torch.nn.Module):
    """Sweep section of PSNet.forward (models/PSNet.py:128-158) on given features."""

    def __init__(self, nlabel, mindepth=1.0, rescale_depth=False, norm_target=0.8, dtype=torch.float32,
                 predict_by_depth=False):
        super().__init__()
        self.predict_by_depth = predict_by_depth
        self.nlabel = int(nlabel)
        self.mindepth = float(mindepth)
        self.rescale_depth = rescale_depth
        self.norm_target = norm_target
        self.dtype = dtype

    def forward(self, ref_fea, tgt_feas, pose, intrinsics, intrinsics_inv):
        """ref_fea [B,C,h,w]; tgt_feas list of [B,C,h,w]; pose [B,T,3,4];
        returns a list of cost volumes [B,2C,L,h,w]."""
        K4, Ki4 = quarter_intrinsics(intrinsics, intrinsics_inv)
        if self.rescale_depth:
            pose[:, 0, :, -1:] = pose[:, 0, :, -1:] * self.norm_target
        return [plane_sweep_cost(ref_fea, t, pose[:, j], K4, Ki4, self.nlabel, self.mindepth, self.dtype,
                                 predict_by_depth=self.predict_by_depth)
                for j, t in enumerate(tgt_feas)]
