"""The split-f16 matrix-core scorer (k_score_mf, csrc/score_mf.h; the default)
against the float32-VALU scorer k_score32 (score_mf=0) and the oracle: every
per-hypothesis score identical (the decisions are exact by bound, undecided
evaluations go to float64), on dense KITTI pairs, thresholds across the valid
range [2^-15, 1), points beyond the f16 monomial range (M > 15.9), the
num_test / num_ransac_test prefixes, and a ragged batch."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R

pytestmark = pytest.mark.gpu


def _scores(pts, n=None, iters=2, thr=1e-4, nt=None, nr=None, mf=1):
    from sfm_amd import _lib, ransac
    _lib.tune("score_mf", mf)
    try:
        out = ransac.ransac5_batched(pts, n, nt, nr, iters, thr, return_scores=True)
    finally:
        _lib.tune("score_mf", 1)
    return [t.cpu() for t in out]


def _equal(a, b):
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("thr", [1e-4, 3.1e-5, 1e-3, 0.02, 0.3, 2.0 ** -15])
def test_mf_equals_fp32_scorer(cuda, thr):
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=int(thr * 1e6) % 1000, hw=(160, 400))
    pts = ransac.flow_to_points(flow.to(cuda), torch.inverse(K).to(cuda))
    _equal(_scores(pts, thr=thr, mf=1), _scores(pts, thr=thr, mf=0))


def test_mf_full_size_vs_oracle(cuda):
    """One full KITTI pair (N = 435,032) at H = 4096: every hypothesis score."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=77)
    pts = ransac.flow_to_points(flow.to(cuda), torch.inverse(K).to(cuda))
    E, P, inl, win, scores = _scores(pts, iters=8)
    p = pts[0].cpu().numpy()
    ref = R.ransac5(p[:, :2], p[:, 2:], iters=8, thr=1e-4, nthreads=16)
    assert int(win[0]) == ref["winner"] and int(inl[0]) == ref["inliers"]
    assert np.array_equal(scores[0].numpy(), ref["hyp_score"])
    assert np.array_equal(E[0].numpy(), ref["E"]) and np.array_equal(P[0].numpy(), ref["P"])


def test_mf_large_coordinates_and_prefixes(cuda):
    """Points far outside the image (M up to 40: past the f16 monomial range,
    scored in float64), num_test < num_ransac_test, and a ragged batch."""
    from oracle.gen_golden import geometric_scene
    rng = np.random.default_rng(4)
    rows = []
    ns = [3000, 2500]
    for n in ns:
        q, qp = geometric_scene(rng, n, out_frac=0.2, noise=0.002)
        qp[:40] = rng.uniform(-40, 40, (40, 2))          # M > 15.9
        q[40:60] *= 12.0                                  # M in (8, 12): inside the range
        rows.append(np.c_[q, qp])
    pts = np.zeros((2, max(ns), 4))
    for i, r in enumerate(rows):
        pts[i, :len(r)] = r
    pts = torch.from_numpy(pts).to(cuda)
    for nt, nr in ((None, None), (1500, 2400)):
        got = _scores(pts, ns, iters=2, thr=1e-3, nt=nt, nr=nr)
        _equal(got, _scores(pts, ns, iters=2, thr=1e-3, nt=nt, nr=nr, mf=0))
        for b, n in enumerate(ns):
            r = R.ransac5(rows[b][:, :2], rows[b][:, 2:], nt or n, nr or n, iters=2, thr=1e-3)
            assert np.array_equal(got[4][b].numpy(), r["hyp_score"])
            assert int(got[3][b]) == r["winner"] and int(got[2][b]) == r["inliers"]
