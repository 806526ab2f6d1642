"""The bench's own step against the oracle: TwoViewHotPath.step at the C2
shape (KITTI 376x1242 dense flow, N = 435,032, H = 4096, nlabel = 128, fp32
volume), two pairs, through the default dispatch (k_score_mf2 with
count-bound pruning, asserted).  Winner, inlier count, E and P of every pair
equal the oracle's on the step's own correspondences (reference:
kernel_functions.cu:141-264, essential_matrix.cu:190-280)."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R

pytestmark = pytest.mark.gpu


def test_bench_step_c2_shape_vs_oracle(cuda):
    from sfm_amd import _lib, synth
    from sfm_amd.pipeline import TwoViewHotPath
    B, C, L, iters, thr = 2, 32, 128, 8, 1e-4
    hw = synth.KITTI_HW
    fhw = synth.feature_hw(hw)
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, hw=hw, device=cuda)
    ref_fea, tgt_fea = synth.features(B, C, fhw[0], fhw[1], seed=0, device=cuda)
    hp = TwoViewHotPath(B, hw, fhw, C, L, iters, thr, 1.0, rescale_depth=True, norm_target=0.6,
                        cost_dtype=torch.float32, device=cuda)
    assert hp.n == 435032
    E, P, inl, cost = hp.step(flow, K, ref_fea, tgt_fea)
    torch.cuda.synchronize()
    assert _lib.last_scorer() == "k_score_mf2+prune"
    assert cost.shape == (B, 2 * C, L, fhw[0], fhw[1]) and bool(torch.isfinite(cost).all())
    _, _, _, win = hp.pose(flow, K)                        # the same call again: the winners
    for b in range(B):
        p = hp.pts[b].cpu().numpy()
        ref = R.ransac5(np.ascontiguousarray(p[:, :2]), np.ascontiguousarray(p[:, 2:]), iters=iters, thr=thr,
                        nthreads=16)
        assert int(win[b]) == ref["winner"] and int(inl[b]) == ref["inliers"], (b, int(inl[b]), ref["inliers"])
        assert np.array_equal(E[b].cpu().numpy(), ref["E"])
        assert np.array_equal(P[b].cpu().numpy(), ref["P"])
