"""BASELINE.json's other configurations as parity cases (the bench line is
configs[1]):

  C1  b=1, nlabel=16, GT pose: the golden cost volume (test_gpu_sweep.py)
  C3  b=32 pairs per launch, bf16 cost volume (8 GPUs in the bench)
  C4  640x480 indoor pairs, nlabel=64, 2048 hypotheses
  C5  LO-RANSAC: 8192 hypotheses + local E refinement (optimise), and the
      reduced-precision inlier-set parity (float32 pre-decision vs float64)
"""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R
from oracle import sweep as S

pytestmark = pytest.mark.gpu


def _pts(flow, K, cuda, **kw):
    from sfm_amd import ransac
    return ransac.flow_to_points(flow.to(cuda), torch.inverse(K).to(cuda), **kw)


def test_c4_indoor_640x480(cuda):
    """640x480 dense flow (N = 285,200), H = 2048 (ransac_iter 4): winner,
    inlier count, E, P and every hypothesis score equal the oracle's; the
    nlabel=64 sweep at 120x160 matches the oracle within 1e-4."""
    from sfm_amd import ransac, synth
    from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics
    flow, K, pose, _ = synth.kitti_pair_batch(1, seed=21, hw=synth.INDOOR_HW, k=synth.INDOOR_K)
    pts = _pts(flow, K, cuda)
    assert pts.shape[1] == 285200
    E, P, inl, win, scores = ransac.ransac5_batched(pts, iters=4, threshold=1e-4, return_scores=True)
    p = pts[0].cpu().numpy()
    ref = R.ransac5(p[:, :2], p[:, 2:], iters=4, thr=1e-4, nthreads=16)
    assert int(win[0]) == ref["winner"] and int(inl[0]) == ref["inliers"]
    assert np.array_equal(scores[0].cpu().numpy(), ref["hyp_score"])
    assert np.array_equal(E[0].cpu().numpy(), ref["E"]) and np.array_equal(P[0].cpu().numpy(), ref["P"])
    # sweep at the indoor feature size with the recovered pose
    h, w = synth.feature_hw(synth.INDOOR_HW)
    assert (h, w) == (120, 160)
    ref_f, tgt_f = synth.features(1, 32, h, w, seed=4)
    Kf, Kif = K.float(), torch.inverse(K.float())
    K4, Ki4 = quarter_intrinsics(Kf, Kif)
    pose_f = P.float().cpu()
    cost = plane_sweep_cost(ref_f.to(cuda), tgt_f.to(cuda), pose_f.to(cuda), K4.to(cuda), Ki4.to(cuda), 64, 1.0)
    planes = [0, 7, 31, 63]
    want = S.plane_sweep_cost(ref_f, tgt_f, pose_f, Kf, Kif, 64, 1.0, planes=planes)
    got = cost[:, :, planes].cpu()
    assert torch.equal(got[:, :32], want[:, :32])
    err = (got - want).abs() - 1e-4 * torch.clamp(want.abs(), min=1.0)   # test_gpu_sweep.py's bar
    assert float(err.max()) <= 0, float((got - want).abs().max())


def test_c5_lo_ransac_8192_and_refinement(cuda):
    """H = 8192 (ransac_iter 16) on a 160x240 dense crop, then the host IRLS
    refinement of the winner (essential_matrix.optimise): bit-exact against
    the oracle; the inlier sets with and without the float32 pre-decision are
    identical (the reduced-precision parity sweep of configs[4])."""
    import essential_matrix
    from sfm_amd import _lib, ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=22, hw=(160, 240))
    pts = _pts(flow, K, cuda)
    outs = []
    for flag in (1, 0):
        _lib.tune("score_fp32", flag)
        try:
            outs.append(ransac.ransac5_batched(pts, iters=16, threshold=1e-4, return_scores=True))
        finally:
            _lib.tune("score_fp32", 1)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    E, P, inl, win, scores = outs[0]
    p = pts[0].cpu().numpy()
    ref = R.ransac5(p[:, :2], p[:, 2:], iters=16, thr=1e-4, nthreads=16)
    assert int(win[0]) == ref["winner"] and np.array_equal(scores[0].cpu().numpy(), ref["hyp_score"])
    assert np.array_equal(E[0].cpu().numpy(), ref["E"])
    m32 = ransac.inlier_mask(pts, E, 1e-4)[0].cpu().numpy()
    assert int(m32.sum()) == int(inl[0])
    q = torch.from_numpy(np.ascontiguousarray(p[:, :2])); qp = torch.from_numpy(np.ascontiguousarray(p[:, 2:]))
    E_opt = essential_matrix.optimise(q, qp, E[0].cpu(), 1e-3, 0.0, 200)
    assert np.array_equal(E_opt.numpy(), R.optimise(p[:, :2], p[:, 2:], ref["E"], 1e-3, 0.0, 200))


def test_c5_full_size_kitti_h8192_pruned_vs_oracle(cuda):
    """C5 at full size: one KITTI pair (N = 435,032), H = 8192 (ransac_iter
    16) through the default launch -- k_score_mf2 with count-bound pruning,
    dispatch asserted -- against the oracle: winner, inlier count, E and P
    (kernel_functions.cu:141-226, essential_matrix.cu:248-265)."""
    from sfm_amd import _lib, ransac, synth
    assert _lib.tune_get("score_mf") == 2 and _lib.tune_get("score_mf_prune") > 0
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=2024)
    pts = _pts(flow, K, cuda)
    assert pts.shape[1] == 435032
    E, P, inl, win = ransac.ransac5_batched(pts, None, None, None, 16, 1e-4)
    assert _lib.last_scorer() == "k_score_mf2+prune"
    p = pts[0].cpu().numpy()
    ref = R.ransac5(np.ascontiguousarray(p[:, :2]), np.ascontiguousarray(p[:, 2:]), iters=16, thr=1e-4,
                    nthreads=16)
    assert int(win[0]) == ref["winner"] and int(inl[0]) == ref["inliers"], (int(inl[0]), ref["inliers"])
    assert np.array_equal(E[0].cpu().numpy(), ref["E"])
    assert np.array_equal(P[0].cpu().numpy(), ref["P"])


def test_c3_batch32_and_bf16(cuda):
    """32 pairs in one batched launch, each equal to the oracle; bf16 cost
    volume at batch 32 is the RNE rounding of the fp32 one."""
    from sfm_amd import ransac, synth
    from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics
    B = 32
    flow, K, pose, _ = synth.kitti_pair_batch(B, seed=23, hw=(64, 96))
    pts = _pts(flow, K, cuda)
    E, P, inl, win = ransac.ransac5_batched(pts, iters=1, threshold=1e-4)
    for b in range(0, B, 7):
        p = pts[b].cpu().numpy()
        ref = R.ransac5(p[:, :2], p[:, 2:], iters=1, thr=1e-4, nthreads=16)
        assert int(win[b]) == ref["winner"] and np.array_equal(E[b].cpu().numpy(), ref["E"]), b
    ref_f, tgt_f = synth.features(B, 32, 16, 24, seed=5)
    K4, Ki4 = quarter_intrinsics(K.float(), torch.inverse(K.float()))
    args = (ref_f.to(cuda), tgt_f.to(cuda), pose.to(cuda), K4.to(cuda), Ki4.to(cuda), 128, 1.0)
    f32 = plane_sweep_cost(*args)
    b16 = plane_sweep_cost(*args, dtype=torch.bfloat16)
    assert torch.equal(b16.cpu(), f32.to(torch.bfloat16).cpu())


@pytest.mark.parametrize("delta,alpha,reps", [(1e-3, 0.0, 200), (2e-3, 1.0, 30), (1e-3, 0.5, 0)])
def test_gpu_irls_matches_host(cuda, delta, alpha, reps):
    """GPU IRLS (sfm_essential_optimise_batched) vs the host restatement of
    polish_E_robust_parametric: 1e-4 relative on E (reassociated sums)."""
    from sfm_amd import ransac, synth
    B = 3
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=31, hw=(120, 200))
    pts = _pts(flow, K, cuda)
    E, _, _, _ = ransac.ransac5_batched(pts, iters=1, threshold=1e-4)
    got = ransac.optimise_batched(pts, E, delta, alpha, reps).cpu().numpy()
    for b in range(B):
        p = pts[b].cpu().numpy()
        want = R.optimise(p[:, :2], p[:, 2:], E[b].cpu().numpy(), delta, alpha, reps)
        rel = np.abs(got[b] - want).max() / np.abs(want).max()
        assert rel <= 1e-4, (b, rel)
