"""Drop-in hygiene of the Python entry points: operands that
need conversion (float64 pose / K, non-contiguous views) stay alive through
the launch, grad-requiring inputs are refused (the sweep is forward-only),
and a shared K^-1 is broadcast instead of read out of bounds."""
import numpy as np
import pytest
import torch

from oracle import flow as OF
from oracle import sweep as S

pytestmark = pytest.mark.gpu


def _warp_case(seed=3, B=2, C=4, h=12, w=20):
    g = torch.Generator().manual_seed(seed)
    feat = torch.randn(B, C, h, w, generator=g)
    depth = 2.0 + 10.0 * torch.rand(B, h, w, generator=g)
    K = torch.tensor([[18.0, 0, 10.0], [0, 18.0, 6.0], [0, 0, 1]]).expand(B, 3, 3).contiguous()
    pose = torch.cat([torch.eye(3).expand(B, 3, 3), torch.tensor([0.3, -0.1, 0.5]).expand(B, 3).unsqueeze(2)], 2)
    pose = pose + 0.01 * torch.randn(B, 3, 4, generator=g)
    return feat, depth, pose, K, torch.inverse(K)


def test_inverse_warp_float64_and_strided_operands(cuda):
    from sfm_amd.sweep import inverse_warp
    feat, depth, pose, K, Ki = _warp_case()
    want = S.inverse_warp(feat, depth, pose, K, Ki)
    # float64 pose / K / K^-1 and a transposed (non-contiguous) K^-1 view: each
    # needs a converted copy, which must outlive the launch
    Ki_t = Ki.double().transpose(1, 2).contiguous().transpose(1, 2)
    assert not Ki_t.is_contiguous()
    for _ in range(3):      # re-run: a recycled freed block would show up as garbage
        got = inverse_warp(feat.to(cuda), depth.to(cuda), pose.double().to(cuda), K.double().to(cuda),
                           Ki_t.to(cuda)).cpu()
        assert float((got - want).abs().max()) < 1e-4


def test_sweep_refuses_grad(cuda):
    from sfm_amd.sweep import inverse_warp, plane_sweep_cost, quarter_intrinsics
    feat, depth, pose, K, Ki = _warp_case()
    f = feat.to(cuda).requires_grad_(True)
    with pytest.raises(RuntimeError, match="forward-only"):
        inverse_warp(f, depth.to(cuda), pose.to(cuda), K.to(cuda), Ki.to(cuda))
    K4, Ki4 = quarter_intrinsics(K, Ki)
    with pytest.raises(RuntimeError, match="forward-only"):
        plane_sweep_cost(feat.to(cuda), f, pose.to(cuda), K4.to(cuda), Ki4.to(cuda), 4)
    with torch.no_grad():   # fine without autograd
        inverse_warp(f, depth.to(cuda), pose.to(cuda), K.to(cuda), Ki.to(cuda))
        plane_sweep_cost(feat.to(cuda), f, pose.to(cuda), K4.to(cuda), Ki4.to(cuda), 4)


def test_shared_kinv_is_broadcast(cuda):
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(3, seed=2, hw=(60, 90))
    Ki = torch.inverse(K[0])
    q, qp = OF.dense_correspondences(flow.numpy(), Ki.expand(3, 3, 3).numpy())
    want = torch.from_numpy(np.concatenate([q, qp], -1))
    for k in (Ki, Ki.unsqueeze(0)):
        got = ransac.flow_to_points(flow.to(cuda), k.to(cuda)).cpu()
        assert torch.equal(got, want)
    with pytest.raises(RuntimeError, match="intrinsic_inv"):
        ransac.flow_to_points(flow.to(cuda), Ki.expand(2, 3, 3).to(cuda))
    with pytest.raises(RuntimeError, match=r"\[B,2,H,W\]"):
        ransac.flow_to_points(flow[:, :1].to(cuda), Ki.to(cuda))
