"""The bench's own step against the oracle: TwoViewHotPath.step at the C2
shape (KITTI 376x1242 dense flow, N = 435,032, H = 4096, nlabel = 128, fp32
volume), two pairs, through the default dispatch (dense flow read by the
RANSAC kernels, k_score_mf2 with count-bound pruning, asserted).  Winner, inlier count, E and P of every pair
equal the oracle's on the step's own correspondences (reference:
kernel_functions.cu:141-264, essential_matrix.cu:190-280), and the step's
cost volume (sfm_plane_sweep_psnet: quarter intrinsics and RESCALE_DEPTH
inside the call, full slab size, the bench's store policy) equals the
oracle's PSNet sweep on a plane subset with the step's own P rescaled by
NORM_TARGET = 0.6 (PSNet.py:130-157)."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R
from oracle import sweep as S

pytestmark = pytest.mark.gpu


def test_bench_step_c2_shape_vs_oracle(cuda):
    from sfm_amd import _lib, synth
    from sfm_amd.pipeline import TwoViewHotPath
    B, C, L, iters, thr = 2, 32, 128, 8, 1e-4
    hw = synth.KITTI_HW
    fhw = synth.feature_hw(hw)
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, hw=hw, device=cuda)
    ref_fea, tgt_fea = synth.features(B, C, fhw[0], fhw[1], seed=0, device=cuda)
    # the bench's configuration: dense flow read by the RANSAC kernels (fused)
    hp = TwoViewHotPath(B, hw, fhw, C, L, iters, thr, 1.0, rescale_depth=True, norm_target=0.6,
                        cost_dtype=torch.float32, device=cuda, fused=True)
    assert hp.n == 435032
    E, P, inl, cost = hp.step(flow, K, ref_fea, tgt_fea)
    torch.cuda.synchronize()
    assert _lib.last_scorer() == "k_score_mf2+prune"
    assert cost.shape == (B, 2 * C, L, fhw[0], fhw[1]) and bool(torch.isfinite(cost).all())
    # the volume the step wrote, against the oracle's sweep with the step's P
    # (float64 -> float32, translation x 0.6 as PSNet.py:135-136) and the
    # step's K^-1 (kinv3x3, bit-equal to torch.inverse on the device); bar:
    # test_gpu_sweep.py's _close_rel (1e-4 relative + 2e-6 absolute)
    planes = [0, 31, 64, 127]
    Kinv = hp.k_inverse(K)
    want = S.plane_sweep_cost(ref_fea.cpu(), tgt_fea.cpu(), P.float().cpu(), K.cpu(), Kinv.cpu(), L, 1.0,
                              rescale=0.6, planes=planes)
    got = cost[:, :, planes].float().cpu()
    assert torch.equal(got[:, :C], want[:, :C])
    err = (got[:, C:] - want[:, C:]).abs() - (1e-4 * want[:, C:].abs() + 2e-6)
    assert float(err.max()) <= 0.0, float((got[:, C:] - want[:, C:]).abs().max())
    assert float(want[:, C:].abs().sum()) > 0.0       # the step's poses project into the image
    _, _, _, win = hp.pose(flow, K)                        # the same call again: the winners
    # the step's correspondences as the fused kernels read them (bit-identical
    # to the materialised ones: test_gpu_ransac.py::test_fused_flow_path_equals_packed)
    from sfm_amd import ransac
    pts = ransac.flow_to_points(flow, Kinv)
    for b in range(B):
        p = pts[b].cpu().numpy()
        ref = R.ransac5(np.ascontiguousarray(p[:, :2]), np.ascontiguousarray(p[:, 2:]), iters=iters, thr=thr,
                        nthreads=16)
        assert int(win[b]) == ref["winner"] and int(inl[b]) == ref["inliers"], (b, int(inl[b]), ref["inliers"])
        assert np.array_equal(E[b].cpu().numpy(), ref["E"])
        assert np.array_equal(P[b].cpu().numpy(), ref["P"])
