"""Correspondence build on the GPU vs the reference's own output: corr.npz
holds the float64 q / qp that the reference's SFMnet.pose_by_ransac handed to
essential_matrix.computeP (oracle/gen_golden.py:gen_corr).  Bit-exact in the
dense branch (with and without the h_side/w_side crop) and the rounded-keypoint
and SIFT_POSE branches; SAMPLE_SP within fp32 ulps (grid_sample's CPU and CUDA
unnormalisation orders differ); then the drop-in epipolar glue through the real
extension."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_dense_correspondences_bit_exact_vs_reference(golden, cuda):
    from sfm_amd import ransac
    g = golden("corr.npz")
    inp = g["input"]
    flow = torch.from_numpy(inp["flow"]).to(cuda)
    Ki = torch.from_numpy(inp["Kinv"]).to(cuda)
    for name, side in (("dense", (None, None)), ("dense_side", tuple(int(v) for v in inp["side"]))):
        pts = ransac.flow_to_points(flow, Ki, *side).cpu().numpy()
        assert np.array_equal(pts[..., :2], g[name]["q"]), name
        assert np.array_equal(pts[..., 2:], g[name]["qp"]), name
    fused = ransac.ransac5_flow(flow, Ki, iters=1, threshold=1e-3)     # same points, read on the fly
    packed = ransac.ransac5_batched(ransac.flow_to_points(flow, Ki), None, None, None, 1, 1e-3)
    assert all(torch.equal(a, b) for a, b in zip(fused, packed))


@pytest.mark.parametrize("mode", ["round", "sample_sp", "sift_pose"])
def test_keypoint_correspondences_bit_exact_vs_reference(golden, cuda, mode):
    from sfm_amd import ransac
    g = golden("corr.npz")
    inp = g["input"]
    flow = torch.from_numpy(inp["flow"]).to(cuda)
    Ki = torch.from_numpy(inp["Kinv"]).to(cuda)
    kp1 = list(inp["kp1"]); kp2 = list(inp["kp2"])
    H, W = flow.shape[2:]
    pts, n = ransac.keypoints_to_points(flow, Ki, kp1, kp2, mode=mode, h_side=H, w_side=W)
    pts = pts.cpu().numpy()
    assert n == [kp1[0].shape[0]] * 2
    want = np.concatenate([g[mode]["q"], g[mode]["qp"]], -1)
    if mode == "sample_sp":
        # the fixture is torch-CPU's vectorised grid_sample, which unnormalises
        # as (x+1)*((W-1)/2); the kernel follows the CUDA grid_sampler of the
        # reference's GPU deployment, ((x+1)/2)*(W-1): a few fp32 ulps of the
        # pixel coordinate apart
        assert np.allclose(pts, want, rtol=2e-6, atol=1e-7), np.abs(pts - want).max()
    else:
        assert np.array_equal(pts, want)


def test_compute_P_matrix_ransac_through_extension(golden, cuda):
    """epipolar_utils.compute_P_matrix_ransac over the real extension: E is the
    golden float64 E cast to float32, P the golden P, F = K^-T E K^-1."""
    import epipolar_utils as EU
    g = golden("ransac.npz")["dense_tr_equal"]
    n, nt, nr, it, thr, cheir, seed = g["params"]
    c1 = torch.from_numpy(g["q"]).float().to(cuda)
    c2 = torch.from_numpy(g["qp"]).float().to(cuda)
    # the glue casts float32 correspondences to float64, so the golden case is
    # re-run on the same float32-rounded points through the packed entry point
    from sfm_amd import ransac
    pts = torch.cat([c1.double(), c2.double()], 1).unsqueeze(0)
    Ew, Pw, iw, _ = ransac.ransac5_batched(pts, None, int(nt), int(nr), int(it), float(thr))
    Ki = torch.eye(3, device=cuda) * 0.5
    Ki[2, 2] = 1.0
    E, P, F, inl = EU.compute_P_matrix_ransac(c1, c2, Ki, 0.001, 0.0, 200, int(nt), int(nr), int(it), float(thr))
    assert E.dtype == torch.float32 and torch.equal(E, Ew[0].float())
    assert torch.equal(P, Pw[0]) and inl == int(iw[0])
    assert torch.equal(F, Ki.t().mm(E).mm(Ki))


def test_reference_shaped_1xNx2_input_is_refused(golden, cuda):
    """The reference's compute_E_matrix passes [1, N, 2] (epipolar_utils.py:71-73)
    and its extension silently reads N = 1; this build raises instead."""
    import essential_matrix
    g = golden("ransac.npz")["dense_tr_equal"]
    q = torch.from_numpy(g["q"]).unsqueeze(0).contiguous().to(cuda)
    with pytest.raises(RuntimeError, match=r"\[N, 2\]"):
        essential_matrix.initialise(q, q, 10, 10, 1, 1e-3)
