"""SFMnet mirror (models/SFMnet.py) with injected flow / depth estimators and
matcher: the pose branch through libsfm_hip vs the oracle pipeline (oracle
correspondences -> oracle RANSAC per pair), bit-exact on E and P; the
keypoint gather modes vs oracle/flow.py; the reference's return tuples."""
import numpy as np
import pytest
import torch

from oracle import flow as OF
from oracle import ransac5 as ORR

pytestmark = pytest.mark.gpu

HW = (96, 160)


def _batch(B, seed):
    from sfm_amd import synth
    flow, K, pose, _ = synth.kitti_pair_batch(B, seed=seed, hw=HW)
    K = synth.intrinsics(B, 180.0, 180.0, 80.0, 48.0)
    return flow, K, pose


class _Flow(torch.nn.Module):
    def __init__(self, flow):
        super().__init__()
        self.flow = flow

    def forward(self, x):
        return self.flow.to(x.device), torch.ones_like(self.flow[:, :1]).to(x.device)


class _Depth(torch.nn.Module):
    def forward(self, ref, targets, P_mat, K, Kinv, pose_gt=None, depth_gt=None, E_mat=None):
        self.seen = (P_mat.clone(), None if E_mat is None else E_mat.clone())
        d = torch.ones(ref.shape[0], 1, ref.shape[2], ref.shape[3], device=ref.device)
        return d, 2 * d


def _model(flow, matcher=None, **over):
    from models.SFMnet import SFMnet
    from sfm_amd.config import defaults
    c = defaults()
    c.update(ransac_iter=2, **over)
    return SFMnet(64, 1.0, flow_estimator=_Flow(flow), depth_estimator=_Depth(), matcher=matcher, cfg=c).eval()


def _oracle_pose(q, qp, iters, thr):
    r = ORR.ransac5(q, qp, iters=iters, thr=thr)
    return r["E"].astype(np.float32), r["P"].astype(np.float32)


def test_dense_pose_matches_oracle(cuda):
    B = 3
    flow, K, pose = _batch(B, seed=11)
    m = _model(flow)
    img = torch.zeros(B, 3, *HW, device=cuda)
    flow_2D, P_mat, depth, times = m(img, img, K, pose_gt=pose.to(cuda))
    assert P_mat.shape == (B, 1, 3, 4) and P_mat.dtype == torch.float32
    assert depth.shape == (B, 1, *HW) and float(depth[0, 0, 0, 0]) == 2.0
    Ki = torch.inverse(K.float())
    q, qp = OF.dense_correspondences(flow.numpy(), Ki.numpy())
    for b in range(B):
        E, P = _oracle_pose(q[b], qp[b], 2, 1e-4)
        assert np.array_equal(P_mat[b, 0].cpu().numpy(), P), b
        assert np.array_equal(m.depth_estimator.seen[1][b].cpu().numpy(), E), b


def test_record_pose_and_gt_pose(cuda):
    B = 2
    flow, K, pose = _batch(B, seed=12)
    m = _model(flow, RECORD_POSE=True)
    img = torch.zeros(B, 3, *HW, device=cuda)
    P_mat, f = m(img, img, K)
    assert P_mat.shape == (B, 1, 3, 4) and torch.equal(f.cpu(), flow)
    m = _model(flow, GT_POSE_NORMALIZED=True)
    flow_2D, P_mat, depth, _ = m(img, img, K, pose_gt=pose.to(cuda), use_gt_pose=True)
    t = pose[:, :, 3]
    assert torch.allclose(P_mat[:, 0, :, 3].cpu(), t / t.norm(dim=1, keepdim=True))
    assert float(flow_2D.abs().sum()) == 0.0


@pytest.mark.parametrize("mode", ["round", "sample_sp", "sift_pose"])
def test_keypoint_points_match_oracle(cuda, mode):
    from sfm_amd import ransac
    B = 2
    flow, K, _ = _batch(B, seed=13)
    Ki = torch.inverse(K.float())
    rng = np.random.default_rng(5)
    kp1 = [rng.uniform(0, [HW[1] - 1, HW[0] - 1], (n, 2)) for n in (57, 33)]
    kp1[0][:4] = [[0.5, 1.5], [2.5, 0.0], [HW[1] - 1.0, HW[0] - 1.0], [10.5, 20.5]]   # ties, corners
    kp2 = [k + rng.normal(0, 2, k.shape) for k in kp1]
    pts, n = ransac.keypoints_to_points(flow.to(cuda), Ki.to(cuda), kp1, kp2 if mode == "sift_pose" else None, mode)
    assert n == [57, 33]
    for b in range(B):
        q, qp = OF.keypoint_correspondences(flow[b].numpy(), Ki[b].numpy(), kp1[b], kp2[b], mode)
        got = pts[b, :n[b]].cpu().numpy()
        want = np.c_[q, qp]
        if mode == "sample_sp":
            # CUDA-order unnormalisation ((x+1)/2)(W-1) vs torch-CPU's (x+1)((W-1)/2)
            assert np.allclose(got, want, rtol=2e-6, atol=1e-7), np.abs(got - want).max()
        else:
            assert np.array_equal(got, want)


def test_sparse_and_dense_pairs_in_one_batch(cuda):
    B = 3
    flow, K, _ = _batch(B, seed=14)
    Ki = torch.inverse(K.float())
    rng = np.random.default_rng(9)
    kps = {0: rng.uniform(0, [HW[1] - 1, HW[0] - 1], (400, 2)), 1: rng.uniform(0, 50, (5, 2)),
           2: rng.uniform(0, [HW[1] - 1, HW[0] - 1], (250, 2))}
    calls = []

    def matcher(r, t):
        i = len(calls)
        calls.append(r.shape)
        return kps[i], kps[i] + 1.0

    m = _model(flow, matcher=matcher)
    img = torch.zeros(B, 3, *HW, device=cuda)
    _, P_mat, _, _ = m(img, img, K)
    assert len(calls) == B and calls[0] == (HW[0], HW[1], 3)
    qd, qpd = OF.dense_correspondences(flow.numpy(), Ki.numpy())
    for b in range(B):
        if b == 1:          # 5 < min_matches: dense fallback (SFMnet.py:239-241)
            q, qp = qd[b], qpd[b]
        else:
            q, qp = OF.keypoint_correspondences(flow[b].numpy(), Ki[b].numpy(), kps[b], mode="round")
        _, P = _oracle_pose(q, qp, 2, 1e-4)
        assert np.array_equal(P_mat[b, 0].cpu().numpy(), P), b


def test_keypoint_index_errors(cuda):
    from sfm_amd import ransac
    flow, K, _ = _batch(1, seed=15)
    Ki = torch.inverse(K.float()).to(cuda)
    with pytest.raises(IndexError):
        ransac.keypoints_to_points(flow.to(cuda), Ki, [np.array([[HW[1] - 0.4, 3.0]])])
    # negative rounding wraps like torch indexing
    pts, _ = ransac.keypoints_to_points(flow.to(cuda), Ki, [np.array([[-0.6, 3.0]])])
    q, qp = OF.keypoint_correspondences(flow[0].numpy(), Ki[0].cpu().numpy(), np.array([[HW[1] - 1.0, 3.0]]))
    assert np.array_equal(pts[0].cpu().numpy(), np.c_[q, qp])


def test_end_to_end_with_sweep_depth(cuda):
    """SFMnet with only a flow estimator injected: RANSAC pose + correlation
    sweep + soft-argmin head, checked against the oracle chain."""
    from models.SFMnet import SFMnet
    from sfm_amd.config import defaults
    from sfm_amd.depth import SweepDepthEstimator
    from oracle import sweep as S
    B = 2
    flow, K, _ = _batch(B, seed=16)
    c = defaults()
    c.update(ransac_iter=2, RESCALE_DEPTH=True, NORM_TARGET=0.6)
    g = torch.Generator().manual_seed(3)
    ref = torch.randn(B, 3, *HW, generator=g)
    tgt = torch.randn(B, 3, *HW, generator=g)
    m = SFMnet(32, 1.0, flow_estimator=_Flow(flow), cfg=c,
               depth_estimator=SweepDepthEstimator(32, 1.0, rescale_depth=True, norm_target=0.6)).eval()
    flow_2D, P_mat, depth, _ = m(ref.to(cuda), tgt.to(cuda), K)
    assert depth.shape == (B, 1, *HW)
    # oracle chain on the poses the model used (P_mat was rescaled in place, as PSNet does)
    P = P_mat[:, 0].cpu()
    Ki = torch.inverse(K.float())
    f = lambda x: torch.nn.functional.avg_pool2d(x, 4)
    cost = S.correlation_cost(f(ref), f(tgt), P, K, Ki, 32, 1.0)
    want = S.depth_head(cost, 32, 1.0, HW)
    rel = ((depth.cpu() - want).abs() / want.abs()).max()
    assert float(rel) <= 1e-4, float(rel)


def _psnet_inputs(cuda, B=1, H=128, W=192):
    from sfm_amd import synth
    g = torch.Generator().manual_seed(3)
    ref = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).to(cuda)
    tgt = (torch.rand(B, 3, H, W, generator=g) * 2 - 1).to(cuda)
    K = synth.intrinsics(B, 100.0, 98.0, 95.5, 63.5).to(cuda)
    a = torch.tensor([[0, -0.02, 0.01], [0.02, 0, -0.015], [-0.01, 0.015, 0.0]])
    pose = torch.cat([torch.matrix_exp(a), torch.tensor([[0.2], [-0.05], [-1.2]])], 1)
    return ref, tgt, K, pose.reshape(1, 3, 4).repeat(B, 1, 1).to(cuda)


def test_default_sfmnet_runs_as_main_builds_it(cuda):
    """SFMnet(nlabel) with no injected estimators (main.py:198): GT pose, the
    PSNet-layout depth estimator (feature CNN, HIP sweep + regularisation +
    head, context networks), eval return tuple; a predicted pose without a
    flow estimator is a named error."""
    from models.SFMnet import SFMnet
    from sfm_amd.config import kitti
    c = kitti()
    c.update(MIXED_PREC=False)
    torch.manual_seed(0)
    m = SFMnet(16, 1.0, cfg=c).to(cuda).eval()
    ref, tgt, K, pose = _psnet_inputs(cuda)
    with torch.no_grad():
        flow, P_mat, depth, _ = m(ref, tgt, K, pose_gt=pose, use_gt_pose=True)
    assert P_mat.shape == (1, 1, 3, 4) and flow.shape == (1, 2, 128, 192)
    assert depth.shape == (1, 1, 128, 192) and bool(torch.isfinite(depth).all())
    with pytest.raises(RuntimeError, match="flow_estimator="):
        m(ref, tgt, K, pose_gt=pose)


def test_psnet_without_context_is_the_hot_path_chain(cuda):
    """PSNet with PSNET_CONTEXT off: both outputs equal psnet_depth (sweep ->
    CostRegularization -> head) on the module's own features, bit for bit."""
    from sfm_amd.config import defaults
    from sfm_amd.psnet import PSNet
    from sfm_amd.regularize import psnet_depth
    c = defaults()
    c.update(PSNET_CONTEXT=False, RESCALE_DEPTH=True, NORM_TARGET=0.6)
    torch.manual_seed(1)
    net = PSNet(16, 1.0, cfg=c).to(cuda).eval()
    ref, tgt, K, pose = _psnet_inputs(cuda)
    Kinv = torch.inverse(K)
    P = pose.unsqueeze(1).clone()
    fea = []             # the features this forward computed (MIOpen may pick another algorithm on a re-run)
    net.feature_extraction.register_forward_hook(lambda m, i, o: fea.append(o.detach().clone()))
    with torch.no_grad():
        d_init, d = net(ref, [tgt], P, K, Kinv)
        assert torch.allclose(P[:, 0, :, 3], pose[:, :, 3] * 0.6)           # RESCALE_DEPTH in place
        want = psnet_depth(fea[0].float(), fea[1].float(), P[:, 0], K, Kinv, net.regularize, 16, 1.0,
                           out_hw=(128, 192))
    assert torch.equal(d_init, d)
    assert torch.equal(d, want)


def test_psnet_predict_by_depth_init_is_unscaled(cuda):
    """PREDICT_BY_DEPTH at MIN_DEPTH = 2: the reference returns depthregression's
    output as depth_init and scales only depth by mindepth (PSNet.py:200-202 vs
    209-210); with PSNET_CONTEXT off both come from the same cost, so
    depth == 2 * depth_init exactly."""
    from sfm_amd.config import defaults
    from sfm_amd.psnet import PSNet
    c = defaults()
    c.update(PSNET_CONTEXT=False, PREDICT_BY_DEPTH=True, MIN_DEPTH=2.0)
    torch.manual_seed(2)
    net = PSNet(16, cfg=c).to(cuda).eval()
    ref, tgt, K, pose = _psnet_inputs(cuda)
    with torch.no_grad():
        d_init, d = net(ref, [tgt], pose.unsqueeze(1).clone(), K, torch.inverse(K))
    assert net.mindepth == 2.0
    assert torch.equal(d_init * 2.0, d)


def test_psnet_ind_context_feeds_dep_convs(cuda):
    """IND_CONTEXT with PSNET_CONTEXT: the reference reassigns refimg_fea =
    context_net(ref) (PSNet.py:177-178), so PSNET_DEP_CONTEXT upsamples the
    context features, not feature_extraction's (PSNet.py:219)."""
    import torch.nn.functional as F
    from sfm_amd.config import defaults
    from sfm_amd.psnet import PSNet
    c = defaults()
    c.update(PSNET_CONTEXT=True, IND_CONTEXT=True, PSNET_DEP_CONTEXT=True)
    torch.manual_seed(3)
    net = PSNet(16, 1.0, cfg=c).to(cuda).eval()
    ref, tgt, K, pose = _psnet_inputs(cuda)
    rec = {}
    net.context_net.register_forward_hook(lambda m, i, o: rec.__setitem__("ctx", o.detach().clone()))
    net.dep_convs.register_forward_pre_hook(lambda m, i: rec.__setitem__("dep_in", i[0].detach().clone()))
    with torch.no_grad():
        net(ref, [tgt], pose.unsqueeze(1).clone(), K, torch.inverse(K))
        up = F.interpolate(rec["ctx"].float(), list(ref.shape[2:]), mode="bilinear", align_corners=True)
    assert rec["dep_in"].shape[1] == 36
    assert torch.equal(rec["dep_in"][:, 1:33], up)
