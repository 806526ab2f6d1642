"""sfm_kinv3x3 (csrc/kinv.hip) against torch.linalg.inv_ex / torch.inverse on
the device, every bit compared (signed zeros included): SFMnet.forward's
intrinsic_inv_gpu = torch.inverse(intrinsic_gpu) (models/SFMnet.py:104) in
one launch.  Intrinsic matrices with and without row pivoting (|cx| > fx),
KITTI's and the bench's, and general 3x3 matrices."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.contiguous().view(torch.int32)


def _intrinsics(n, g):
    fx = 100 + 1900 * torch.rand(n, generator=g)
    fy = fx * (0.8 + 0.4 * torch.rand(n, generator=g))
    cx = 2500 * torch.rand(n, generator=g)        # |cx| > fx for part of them: pivoting
    cy = 1500 * torch.rand(n, generator=g)
    K = torch.zeros(n, 3, 3)
    K[:, 0, 0], K[:, 0, 2], K[:, 1, 1], K[:, 1, 2], K[:, 2, 2] = fx, cx, fy, cy, 1.0
    return K


@pytest.mark.parametrize("kind", ["intrinsics", "general", "bench"])
def test_kinv_bit_identical_to_torch(cuda, kind):
    from sfm_amd import synth
    from sfm_amd.pipeline import kinv3x3
    g = torch.Generator().manual_seed(11)
    if kind == "intrinsics":
        A = _intrinsics(20000, g)
    elif kind == "general":
        A = torch.randn(20000, 3, 3, generator=g) * torch.exp(torch.randn(20000, 1, 1, generator=g))
    else:
        A = torch.cat([synth.kitti_pair_batch(8, seed=1000)[1], synth.intrinsics(4)]).float()
    A = A.float().to(cuda)
    got = kinv3x3(A)
    want = torch.linalg.inv_ex(A)[0]
    assert torch.equal(_bits(got), _bits(want)), int((_bits(got) != _bits(want)).any(-1).any(-1).sum())
    assert torch.equal(_bits(kinv3x3(A[0])), _bits(torch.inverse(A[0])))


def test_kinv_pipeline_step_unchanged(cuda):
    """TwoViewHotPath.k_inverse is sfm_kinv3x3: the same bits as the
    torch.inverse the reference calls, so the correspondences are too."""
    from sfm_amd import ransac, synth
    from sfm_amd.pipeline import TwoViewHotPath
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=3, device=cuda)
    Ki = TwoViewHotPath.k_inverse(K)
    assert torch.equal(_bits(Ki), _bits(torch.inverse(K.float())))
    a = ransac.flow_to_points(flow, Ki)
    b = ransac.flow_to_points(flow, torch.inverse(K.float()))
    assert torch.equal(a, b)
