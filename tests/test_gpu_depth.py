"""HIP depth stage (correlation cost + soft-argmin head) vs the oracle
restatements of REG2D.py:103-109 and PSNet.py:191-213.  Floating-point bar
(north_star): 1e-4 relative on the depth map."""
import pytest
import torch

from oracle import sweep as S

pytestmark = pytest.mark.gpu


def _scene(B, C, h, w, seed):
    from sfm_amd import synth
    ref, tgt = synth.features(B, C, h, w, seed=seed)
    K = synth.intrinsics(B, 4.0 * w, 4.0 * w, 2.0 * w, 2.0 * h)
    pose = synth.relative_pose(B, torch.Generator().manual_seed(seed))
    return ref, tgt, K, torch.inverse(K), pose


@pytest.mark.parametrize("B,C,L,h,w,by_depth", [(2, 32, 16, 12, 20, False), (1, 6, 9, 10, 31, True),
                                                 (1, 32, 128, 24, 78, False)])
def test_correlation_cost(cuda, B, C, L, h, w, by_depth):
    from sfm_amd.depth import correlation_cost
    from sfm_amd.sweep import quarter_intrinsics
    ref, tgt, K, Ki, pose = _scene(B, C, h, w, seed=L)
    K4, Ki4 = quarter_intrinsics(K, Ki)
    got = correlation_cost(ref.to(cuda), tgt.to(cuda), pose.to(cuda), K4.to(cuda), Ki4.to(cuda), L, 0.8,
                           predict_by_depth=by_depth).cpu()
    want = S.correlation_cost(ref, tgt, pose, K, Ki, L, 0.8, predict_by_depth=by_depth)
    assert float(want.abs().max()) > 0.05
    err = (got - want).abs() - (1e-4 * want.abs() + 2e-5)
    assert float(err.max()) <= 0, float((got - want).abs().max())


@pytest.mark.parametrize("B,L,h,w,H,W,by_depth", [(2, 16, 12, 20, 48, 80, False), (1, 128, 24, 78, 96, 312, False),
                                                   (1, 10, 7, 9, 7, 9, True), (2, 12, 5, 6, 17, 23, False)])
def test_depth_head(cuda, B, L, h, w, H, W, by_depth):
    from sfm_amd.depth import depth_head
    g = torch.Generator().manual_seed(L + h)
    cost = torch.randn(B, L, h, w, generator=g) * 3.0
    got = depth_head(cost.to(cuda), L, 1.0, (H, W), predict_by_depth=by_depth).cpu()
    want = S.depth_head(cost, L, 1.0, (H, W), predict_by_depth=by_depth)
    assert got.shape == want.shape == (B, 1, H, W)
    rel = ((got - want).abs() / want.abs()).max()
    assert float(rel) <= 1e-4, float(rel)


def test_correlation_depth_module(cuda):
    from sfm_amd.depth import CorrelationDepth
    B, C, L, h, w = 2, 8, 24, 16, 40
    ref, tgt, K, Ki, pose = _scene(B, C, h, w, seed=3)
    m = CorrelationDepth(L, 1.0, rescale_depth=True, norm_target=0.6)
    got = m(ref.to(cuda), tgt.to(cuda), pose.to(cuda), K.to(cuda), Ki.to(cuda), (4 * h, 4 * w)).cpu()
    cost = S.correlation_cost(ref, tgt, pose, K, Ki, L, 1.0, rescale=0.6)
    want = S.depth_head(cost, L, 1.0, (4 * h, 4 * w))
    rel = ((got - want).abs() / want.abs()).max()
    assert float(rel) <= 1e-4, float(rel)


def test_flow2depth_golden(cuda, golden):
    # models/flow2depth.py run by the reference itself (tests/golden/warp.npz)
    from sfm_amd.depth import flow2depth
    g = golden("warp.npz")["flow2depth"]
    flow = torch.zeros(*g["shape"].tolist(), device=cuda)
    got = flow2depth(torch.from_numpy(g["R"]), torch.from_numpy(g["T"]), flow, torch.from_numpy(g["K"])).cpu()
    want = torch.from_numpy(g["out"])
    assert got.shape == want.shape
    err = (got - want).abs() - (1e-5 * want.abs() + 1e-5)
    assert float(err.max()) <= 0, float((got - want).abs().max())


@pytest.mark.parametrize("H,W", [(37, 53), (376, 1242)])
def test_flow2depth_vs_oracle(cuda, H, W):
    from sfm_amd import synth
    from sfm_amd.depth import flow2depth
    pose = synth.relative_pose(1, torch.Generator().manual_seed(H)).float()
    K = synth.intrinsics(1)
    R, T = pose[:, :, :3], pose[:, :, 3]
    got = flow2depth(R, T, torch.zeros(1, 2, H, W, device=cuda), K).cpu()
    want = S.flow2depth(R, T, torch.zeros(1, 2, H, W), K)
    # fp32 sums of O(1e3) terms in another order; near-cancelling outputs keep
    # the operands' absolute rounding (a few ulp of max|out|)
    err = (got - want).abs() - (1e-5 * want.abs() + 1e-6 * float(want.abs().max()))
    assert float(err.max()) <= 0, float((got - want).abs().max())
