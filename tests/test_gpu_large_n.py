"""Correspondence counts past 2^24 (the undecided queues' point field is
span-relative): one pair of N = 2^24 + 8192 correspondences whose
last 8192 sit at the decision boundary of E_0 (test_gpu_score_edge.py's
construction), so undecided evaluations are queued at point indices >= 2^24.
Counts through the matrix-core scorer (score_mf 2) and the float32 VALU
scorer (score_mf 0) equal the exact float64 oracle's."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as ORR

pytestmark = pytest.mark.gpu


def test_counts_beyond_2_pow_24(cuda):
    from sfm_amd import _lib, ransac
    from tests.test_gpu_score_edge import _essential, _offsets
    rng = np.random.default_rng(5)
    thr = 1e-4
    Es = [_essential(rng) for _ in range(4)]
    tail = 8192
    N = (1 << 24) + tail
    g = torch.Generator(device=cuda).manual_seed(3)
    pts = (torch.rand(1, N, 4, generator=g, device=cuda, dtype=torch.float64) - 0.5) * 1.2
    q = rng.uniform(-0.6, 0.6, (tail // 2, 2))
    base, nrm, lo, hi = _offsets(Es[0], q, thr)
    edge = np.r_[np.c_[q, base + lo[:, None] * nrm], np.c_[q, base + hi[:, None] * nrm]]
    pts[0, N - tail:] = torch.from_numpy(edge).to(cuda)
    Et = torch.from_numpy(np.stack(Es)[None]).to(cuda)
    host = pts[0].cpu().numpy()
    qh = np.ascontiguousarray(host[:, :2])
    qph = np.ascontiguousarray(host[:, 2:])
    want = [int(ORR.inlier_mask(E, qh, qph, thr).sum()) for E in Es]
    try:
        for mf in (2, 0):
            _lib.tune("score_mf", mf)
            got = ransac.score_essentials(pts, Et, thr).cpu().numpy()[0]
            assert list(got) == want, (mf, list(got), want)
    finally:
        _lib.tune("score_mf", 2)
    assert want[0] >= tail // 2                 # the inside half of the boundary points counts
