"""Torch-facing RANSAC five-point entry points over the C ABI.

Reference semantics: RANSAC_FiveP/essential_matrix/essential_matrix.cu:110-280
(host drivers) and kernel_functions.cu:53-226 (kernels); see include/sfm_hip.h
for the exact selection rules and the canonical handling of the reference's
indeterminate cases.
"""
import torch

from . import _lib

CHAINS = 512          # reference: 8 blocks x 64 threads (essential_matrix.cu:201-203)
DEFAULT_SEED = 1234   # essential_matrix.cu:15


def _check_dev_f64(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if t.dtype != torch.float64:
        raise RuntimeError(f"{name} must be a double tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def _flow_and_kinv(flow, intrinsic_inv):
    """Validated float32 flow [B,2,H,W] and per-pair K^-1 [B,3,3] (a shared
    [3,3] or [1,3,3] K^-1 is broadcast): the kernels read Ki at b*9."""
    if not flow.is_cuda:
        raise RuntimeError("flow must be a CUDA tensor")
    if flow.dim() != 4 or flow.shape[1] != 2:
        raise RuntimeError(f"flow must be [B,2,H,W], got {tuple(flow.shape)}")
    B = flow.shape[0]
    return flow.contiguous().float(), _kinv_batch(intrinsic_inv, B, flow.device)


def _kinv_batch(intrinsic_inv, B, device):
    Ki = intrinsic_inv
    if Ki.device != device:
        raise RuntimeError(f"intrinsic_inv must be on {device}, got {Ki.device}")
    if Ki.dim() == 2:
        Ki = Ki.unsqueeze(0)
    if Ki.dim() != 3 or tuple(Ki.shape[1:]) != (3, 3) or Ki.shape[0] not in (1, B):
        raise RuntimeError(f"intrinsic_inv must be [B,3,3], [1,3,3] or [3,3] with B={B}, got "
                           f"{tuple(intrinsic_inv.shape)}")
    return Ki.float().expand(B, 3, 3).contiguous()


def hypotheses(iters):
    return CHAINS * int(iters)


def _workspace(batch, n_max, iters, device):
    nbytes = _lib.load().sfm_ransac5_workspace_bytes(int(batch), int(n_max), int(iters))
    if nbytes == 0:
        raise RuntimeError("invalid RANSAC workspace request")
    return torch.empty(int(nbytes), dtype=torch.uint8, device=device)


def ransac5(q, qp, num_test_points, num_ransac_test_points, iters, threshold, seed=DEFAULT_SEED,
            cheirality=True):
    """One pair, reference layout: q, qp [N,2] float64 CUDA contiguous.
    Returns (E [3,3] f64, P [3,4] f64 or None, inliers int32[1], winner int32[1])
    — all on the device, nothing synchronises."""
    _check_dev_f64(q, "input1")
    _check_dev_f64(qp, "input2")
    if q.dim() != 2 or q.shape[1] != 2 or qp.shape != q.shape:
        raise RuntimeError("input1/input2 must both be [N, 2]")
    n = q.shape[0]
    dev = q.device
    with torch.cuda.device(dev):
        ws = _workspace(1, n, iters, dev)
        E = torch.empty(3, 3, dtype=torch.float64, device=dev)
        P = torch.empty(3, 4, dtype=torch.float64, device=dev) if cheirality else None
        inl = torch.empty(1, dtype=torch.int32, device=dev)
        win = torch.empty(1, dtype=torch.int32, device=dev)
        rc = _lib.load().sfm_ransac5(_lib.ptr(q), _lib.ptr(qp), n, int(num_test_points),
                                     int(num_ransac_test_points), int(iters), float(threshold), int(seed),
                                     1 if cheirality else 0, _lib.ptr(ws), ws.numel(), _lib.ptr(E), _lib.ptr(P),
                                     _lib.ptr(inl), _lib.ptr(win), _lib.stream_ptr(dev))
        _lib.check(rc, "sfm_ransac5")
    return E, P, inl, win


class score_precision:
    """Context manager selecting the inlier-scoring precision of the RANSAC
    calls inside it (tuning key "score_precision", process-wide): 64 (the
    default) reproduces the reference's float64 decisions exactly; 32 / 16
    evaluate ComputeError<float> / <half> (approximate inlier sets; BASELINE
    C5's fp32-vs-fp16 sweep).  Nests: leaving restores the precision that was
    in force on entry.  Not thread-safe across concurrent callers.

    The reference only ever instantiates its template (kernel_functions.cu:
    231-264) with T = double, so both reduced forms are parity-unpinned
    against the reference (see DESIGN.md "Reduced-precision scoring"):
      * 32 / 16: this build's variant, E, the products and the sums all held
        in T (E normalised by a power of two);
      * 33 / 17: the literal ComputeError<float> / <half> with the reference's
        double Ematrix (common.h:26): double products, sums rounded to T."""

    def __init__(self, bits):
        if int(bits) not in (64, 32, 16, 33, 17):
            raise ValueError("score precision must be 64, 32, 16 (held in T) or 33, 17 (template form)")
        self.bits = int(bits)
        self._saved = []

    def __enter__(self):
        self._saved.append((int(_lib.tune_get("score_precision")), int(_lib.tune_get("score_lowp_template"))))
        _lib.tune("score_precision", self.bits & ~1 if self.bits != 64 else 64)
        _lib.tune("score_lowp_template", self.bits & 1)
        return self

    def __exit__(self, *exc):
        p, t = self._saved.pop()
        _lib.tune("score_precision", p)
        _lib.tune("score_lowp_template", t)


def ransac5_batched(pts, n=None, num_test_points=None, num_ransac_test_points=None, iters=5, threshold=1e-4,
                    seed=DEFAULT_SEED, cheirality=True, return_scores=False, workspace=None, precision=64):
    """Batched pairs on packed correspondences pts [B, Nstride, 4] float64
    (x, y, x', y').  ``n``: points per pair (default: all Nstride).  Returns
    (E [B,3,3], P [B,3,4] or None, inliers [B] int32, winner [B] int32[, scores [B,H]]).
    ``precision``: inlier-scoring precision (see ``score_precision``)."""
    if int(precision) != 64:
        with score_precision(precision):
            return ransac5_batched(pts, n, num_test_points, num_ransac_test_points, iters, threshold, seed,
                                   cheirality, return_scores, workspace)
    _check_dev_f64(pts, "pts")
    if pts.dim() != 3 or pts.shape[2] != 4:
        raise RuntimeError("pts must be [B, N, 4]")
    B, ns, _ = pts.shape
    n = [ns] * B if n is None else [int(v) for v in n]
    if len(n) != B:
        raise RuntimeError("len(n) must equal the batch size")
    dev = pts.device
    H = hypotheses(iters)
    with torch.cuda.device(dev):
        if workspace is None:
            workspace = _workspace(B, 0, iters, dev)
        E = torch.empty(B, 3, 3, dtype=torch.float64, device=dev)
        P = torch.empty(B, 3, 4, dtype=torch.float64, device=dev) if cheirality else None
        inl = torch.empty(B, dtype=torch.int32, device=dev)
        win = torch.empty(B, dtype=torch.int32, device=dev)
        scores = torch.empty(B, H, dtype=torch.int32, device=dev) if return_scores else None
        rc = _lib.load().sfm_ransac5_packed(
            _lib.ptr(pts), ns, _lib.i64_array(n), B, int(num_test_points or 0), int(num_ransac_test_points or 0),
            int(iters), float(threshold), int(seed), 1 if cheirality else 0, _lib.ptr(workspace),
            workspace.numel(), _lib.ptr(E), _lib.ptr(P), _lib.ptr(inl), _lib.ptr(win), _lib.ptr(scores),
            _lib.stream_ptr(dev))
        _lib.check(rc, "sfm_ransac5_packed")
    out = (E, P, inl, win)
    return out + (scores,) if return_scores else out


def score_essentials(pts, E, threshold, n=None):
    """Exact inlier counts of given essential matrices (the reference's
    ComputeError test, e <= thr) through the RANSAC's own scorer: pts [B, N, 4]
    float64, E [B, C, 3, 3] (or [B, C, 9]) float64 -> counts [B, C] int32."""
    _check_dev_f64(pts, "pts")
    B, ns, _ = pts.shape
    n = [ns] * B if n is None else [int(v) for v in n]
    E = E.reshape(B, -1, 9).to(pts.device, torch.float64).contiguous()
    C = E.shape[1]
    L = _lib.load()
    counts = torch.empty(B, C, dtype=torch.int32, device=pts.device)
    with torch.cuda.device(pts.device):
        ws = torch.empty(int(L.sfm_score_essentials_workspace_bytes(B, C)), dtype=torch.uint8, device=pts.device)
        _lib.check(L.sfm_score_essentials(_lib.ptr(pts), ns, _lib.i64_array(n), B, _lib.ptr(E), C, float(threshold),
                                          _lib.ptr(counts), _lib.ptr(ws), ws.numel(), _lib.stream_ptr(pts.device)),
                   "sfm_score_essentials")
    return counts


def workspace_for(batch, iters, device):
    """Pre-allocate a reusable workspace for ransac5_batched (graph capture)."""
    return _workspace(batch, 0, iters, device)


def pack_points(q, qp):
    """q, qp [N,2] float64 CUDA -> pts [1, N, 4]."""
    _check_dev_f64(q, "input1")
    _check_dev_f64(qp, "input2")
    n = q.shape[0]
    out = torch.empty(1, n, 4, dtype=torch.float64, device=q.device)
    with torch.cuda.device(q.device):
        _lib.check(_lib.load().sfm_pack_points(_lib.ptr(q), _lib.ptr(qp), n, _lib.ptr(out),
                                               _lib.stream_ptr(q.device)), "sfm_pack_points")
    return out


def inlier_mask(pts, E, threshold, n=None):
    """Exact inlier mask [B, Nstride] (bool) of E [B,3,3] over packed points."""
    _check_dev_f64(pts, "pts")
    B, ns, _ = pts.shape
    n = [ns] * B if n is None else [int(v) for v in n]
    E = E.reshape(B, 9).contiguous().to(torch.float64)
    mask = torch.empty(B, ns, dtype=torch.uint8, device=pts.device)
    with torch.cuda.device(pts.device):
        _lib.check(_lib.load().sfm_ransac5_inlier_mask(_lib.ptr(pts), ns, _lib.i64_array(n), B, _lib.ptr(E),
                                                       float(threshold), _lib.ptr(mask),
                                                       _lib.stream_ptr(pts.device)), "sfm_ransac5_inlier_mask")
    return mask.bool()


def flow_to_points(flow, intrinsic_inv, h_side=None, w_side=None, margin=10, out=None):
    """Dense correspondences of SFMnet.pose_by_ransac (models/SFMnet.py:179-263):
    flow [B,2,H,W] float32, intrinsic_inv [B,3,3] float32 (CUDA) -> pts [B,N,4]
    float64 with N = (h_side-2m)(w_side-2m)."""
    flow, Ki = _flow_and_kinv(flow, intrinsic_inv)
    B, _, H, W = flow.shape
    h = H if h_side is None else int(h_side)
    w = W if w_side is None else int(w_side)
    if not (2 * margin < h <= H and 2 * margin < w <= W):
        raise RuntimeError(f"h_side/w_side ({h}, {w}) must lie in (2*margin, flow size {(H, W)}]")
    N = (h - 2 * margin) * (w - 2 * margin)
    if out is None:
        out = torch.empty(B, N, 4, dtype=torch.float64, device=flow.device)
    with torch.cuda.device(flow.device):
        _lib.check(_lib.load().sfm_flow_to_points(_lib.ptr(flow), B, H, W, h, w, int(margin), _lib.ptr(Ki),
                                                  _lib.ptr(out), _lib.stream_ptr(flow.device)),
                   "sfm_flow_to_points")
    return out


def candidate_counts(workspace, batch, iters):
    """Per-pair number of candidate E's scored by the last ransac5_batched call
    that used ``workspace`` (synchronises)."""
    import ctypes
    out = (ctypes.c_int32 * int(batch))()
    _lib.check(_lib.load().sfm_ransac5_candidate_counts(_lib.ptr(workspace), workspace.numel(), int(batch),
                                                        int(iters), out), "sfm_ransac5_candidate_counts")
    return [int(v) for v in out]


def skipped_evaluations(workspace, batch, iters):
    """Evaluations the last RANSAC call that used ``workspace`` skipped by exact
    bound pruning (0 when it was off; synchronises)."""
    import ctypes
    out = ctypes.c_uint64(0)
    _lib.check(_lib.load().sfm_ransac5_skipped_evaluations(_lib.ptr(workspace), workspace.numel(), int(batch),
                                                           int(iters), ctypes.byref(out)),
               "sfm_ransac5_skipped_evaluations")
    return int(out.value)


def kept_candidates(workspace, batch, iters, with_points=False):
    """Per pair, the candidates the last pruned k_score_mf2 call kept (scored
    to their exact counts) and, with_points, its pruning point (points scored
    before it, a multiple of 1024: clamp at N); synchronises.  Undefined after
    an unpruned call."""
    out = torch.zeros(batch, dtype=torch.int32)
    pts = torch.zeros(batch, dtype=torch.int32)
    _lib.check(_lib.load().sfm_ransac5_kept_candidates(_lib.ptr(workspace), workspace.numel(), int(batch), int(iters),
                                                       _lib.ptr(out), _lib.ptr(pts)), "sfm_ransac5_kept_candidates")
    return (out, pts) if with_points else out


KEYPOINT_MODES = {"round": 0, "sample_sp": 1, "sift_pose": 2}


def keypoints_to_points(flow, intrinsic_inv, kp1, kp2=None, mode="round", h_side=None, w_side=None, out=None):
    """Sparse correspondences of SFMnet.pose_by_ransac (models/SFMnet.py:218-258)
    for per-pair keypoint lists (any matcher; the reference uses cv2 SIFT/SURF).

    kp1 / kp2: lists (one per pair) of [n_b, 2] pixel (x, y) arrays of the
    reference / target image.  mode: "round" (default: flow at np.round(kp1)),
    "sample_sp" (cfg.SAMPLE_SP bilinear), "sift_pose" (cfg.SIFT_POSE: kp1, kp2
    directly).  Returns (pts [B, n_max, 4] float64, n list)."""
    import numpy as np
    m = KEYPOINT_MODES[mode]
    if not intrinsic_inv.is_cuda:
        raise RuntimeError("intrinsic_inv must be a CUDA tensor")
    dev = intrinsic_inv.device
    B = len(kp1)
    Ki = _kinv_batch(intrinsic_inv, B, dev)
    if len(kp1) != B or (m == 2 and (kp2 is None or len(kp2) != B)):
        raise RuntimeError("one keypoint array per pair is required")
    if m != 2:
        if not flow.is_cuda:
            raise RuntimeError("flow must be a CUDA tensor")
        if flow.dim() != 4 or flow.shape[1] != 2 or flow.shape[0] != B:
            raise RuntimeError(f"flow must be [B,2,H,W] with B={B}, got {tuple(flow.shape)}")
        flow = flow.contiguous().float()
        _, _, H, W = flow.shape
    else:
        H = int(h_side or 1); W = int(w_side or 1)
    h = H if h_side is None else int(h_side)
    w = W if w_side is None else int(w_side)
    n = [int(np.asarray(k).reshape(-1, 2).shape[0]) for k in kp1]
    nmax = max(max(n), 1)
    a1 = np.zeros((B, nmax, 2), np.float32)
    a2 = np.zeros((B, nmax, 2), np.float32)
    for b in range(B):
        k = np.asarray(kp1[b], dtype=np.float64).reshape(-1, 2)
        if m == 0:
            # np.int32(np.round(pts)) then coord[:, y, x]: torch indexing wraps
            # negative indices and raises past the end (SFMnet.py:250-253)
            r = np.int32(np.round(k))
            for j, size in ((0, w), (1, h)):
                if np.any(r[:, j] >= size) or np.any(r[:, j] < -size):
                    raise IndexError(f"keypoint index out of range for size {size}")
                r[:, j] = np.where(r[:, j] < 0, r[:, j] + size, r[:, j])
            k = r
        a1[b, :n[b]] = k
        if m == 2:
            a2[b, :n[b]] = np.asarray(kp2[b], dtype=np.float32).reshape(-1, 2)
    t1 = torch.from_numpy(a1).to(dev)
    t2 = torch.from_numpy(a2).to(dev) if m == 2 else None
    out = gather_keypoints(flow if m != 2 else None, Ki, t1, n, mode, kp2=t2, h_side=h, w_side=w, hw=(H, W),
                           out=out)
    return out, n


def gather_keypoints(flow, intrinsic_inv, kp1, n, mode="round", kp2=None, h_side=None, w_side=None, hw=None,
                     out=None):
    """Device-resident form of ``keypoints_to_points``: kp1 (and kp2 for
    "sift_pose") are [B, n_max, 2] float32 CUDA tensors already prepared as
    that function does (rounded and wrapped for "round"); ``n`` the per-pair
    counts.  One launch, no host copies (the bench's sparse step)."""
    m = KEYPOINT_MODES[mode]
    B, nmax, _ = kp1.shape
    dev = kp1.device
    Ki = _kinv_batch(intrinsic_inv, B, dev)
    if m != 2:
        if flow is None or flow.dim() != 4 or flow.shape[:2] != (B, 2):
            raise RuntimeError("flow [B,2,H,W] is required for this keypoint mode")
        flow = flow.contiguous().float()
        H, W = flow.shape[2:]
    else:
        if kp2 is None or tuple(kp2.shape) != tuple(kp1.shape):
            raise RuntimeError("SIFT_POSE needs target keypoints of the same shape as kp1")
        H, W = hw if hw is not None else (int(h_side or 1), int(w_side or 1))
    h = H if h_side is None else int(h_side)
    w = W if w_side is None else int(w_side)
    if len(n) != B:
        raise RuntimeError("one keypoint count per pair is required")
    if out is None:
        out = torch.zeros(B, max(nmax, 1), 4, dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.load().sfm_keypoints_to_points(
            None if m == 2 else _lib.ptr(flow), B, H, W, h, w, _lib.ptr(kp1.contiguous()),
            None if kp2 is None else _lib.ptr(kp2.contiguous()), nmax, _lib.i64_array(n), m, _lib.ptr(Ki),
            _lib.ptr(out), out.shape[1], _lib.stream_ptr(dev)), "sfm_keypoints_to_points")
    return out


def optimise_batched(pts, E_init, delta=0.001, alpha=0.0, max_reps=200, n=None, workspace=None):
    """GPU IRLS refinement of E for a batch of pairs (the loop of
    EssentialMatrixOptimise, polish_E.cu:1470-1577): pts [B, N, 4] float64,
    E_init [B, 3, 3] float64 (CUDA) -> E [B, 3, 3].  Agrees with the host
    `essential_matrix.optimise` to rounding level (reassociated sums)."""
    _check_dev_f64(pts, "pts")
    B, ns, _ = pts.shape
    n = [ns] * B if n is None else [int(v) for v in n]
    E0 = E_init.reshape(B, 9).to(pts.device, torch.float64).contiguous()
    out = torch.empty(B, 3, 3, dtype=torch.float64, device=pts.device)
    L = _lib.load()
    with torch.cuda.device(pts.device):
        if workspace is None:
            nb = L.sfm_essential_optimise_workspace_bytes(B, ns)
            workspace = torch.empty(int(nb), dtype=torch.uint8, device=pts.device)
        rc = L.sfm_essential_optimise_batched(_lib.ptr(pts), ns, _lib.i64_array(n), B, _lib.ptr(E0), float(delta),
                                              float(alpha), int(max_reps), _lib.ptr(out), _lib.ptr(workspace),
                                              workspace.numel(), _lib.stream_ptr(pts.device))
        _lib.check(rc, "sfm_essential_optimise_batched")
    return out


def ransac5_flow(flow, intrinsic_inv, iters=5, threshold=1e-4, h_side=None, w_side=None, margin=10,
                 num_test_points=None, num_ransac_test_points=None, seed=DEFAULT_SEED, cheirality=True,
                 return_scores=False, workspace=None):
    """Fused dense path (SFMnet.py:179-274 without the correspondence buffer):
    RANSAC straight from flow [B,2,H,W] float32 and K^-1 [B,3,3] (CUDA).
    Bit-identical to ransac5_batched(flow_to_points(flow, K^-1), ...)."""
    flow, Ki = _flow_and_kinv(flow, intrinsic_inv)
    B, _, H, W = flow.shape
    h = H if h_side is None else int(h_side)
    w = W if w_side is None else int(w_side)
    if not (2 * margin < h <= H and 2 * margin < w <= W):
        raise RuntimeError(f"h_side/w_side ({h}, {w}) must lie in (2*margin, flow size {(H, W)}]")
    dev = flow.device
    Hh = hypotheses(iters)
    with torch.cuda.device(dev):
        if workspace is None:
            workspace = _workspace(B, 0, iters, dev)
        E = torch.empty(B, 3, 3, dtype=torch.float64, device=dev)
        P = torch.empty(B, 3, 4, dtype=torch.float64, device=dev) if cheirality else None
        inl = torch.empty(B, dtype=torch.int32, device=dev)
        win = torch.empty(B, dtype=torch.int32, device=dev)
        scores = torch.empty(B, Hh, dtype=torch.int32, device=dev) if return_scores else None
        rc = _lib.load().sfm_ransac5_flow(
            _lib.ptr(flow), B, H, W, h, w, int(margin), _lib.ptr(Ki), int(num_test_points or 0),
            int(num_ransac_test_points or 0), int(iters), float(threshold), int(seed), 1 if cheirality else 0,
            _lib.ptr(workspace), workspace.numel(), _lib.ptr(E), _lib.ptr(P), _lib.ptr(inl), _lib.ptr(win),
            _lib.ptr(scores), _lib.stream_ptr(dev))
        _lib.check(rc, "sfm_ransac5_flow")
    out = (E, P, inl, win)
    return out + (scores,) if return_scores else out
