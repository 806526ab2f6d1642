"""The split-f16 matrix-core scorers -- k_score_mf2 (score_mf=2, the default
and the benched kernel, csrc/score_mf2.h) and k_score_mf (score_mf=1, the
item-major kernel, which also serves num_test != num_ransac_test) -- against
the float32-VALU scorer k_score32 (score_mf=0) and the oracle: every
per-hypothesis score identical (the decisions are exact by bound, undecided
evaluations go to float64), on dense KITTI pairs, thresholds across the valid
range [2^-15, 1), points beyond the f16 monomial range (M > 15.9), the
num_test / num_ransac_test prefixes, and a ragged batch.  Every call asserts
the kernel it dispatched (sfm_last_scorer)."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R

pytestmark = pytest.mark.gpu


_KERNEL = {2: "k_score_mf2", 1: "k_score_mf", 0: "k_score32"}


def _scores(pts, n=None, iters=2, thr=1e-4, nt=None, nr=None, mf=2):
    from sfm_amd import _lib, ransac
    old = _lib.tune_get("score_mf")
    _lib.tune("score_mf", mf)
    try:
        out = ransac.ransac5_batched(pts, n, nt, nr, iters, thr, return_scores=True)
    finally:
        _lib.tune("score_mf", old)
    # k_score_mf2 runs only when num_test == num_ransac_test (k_score_mf otherwise)
    want = _KERNEL[mf] if (mf != 2 or nt == nr) else "k_score_mf"
    assert _lib.last_scorer() == want, (_lib.last_scorer(), want)
    return [t.cpu() for t in out]


def _equal(a, b):
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize("mf", [2, 1])
@pytest.mark.parametrize("thr", [1e-4, 3.1e-5, 1e-3, 0.02, 0.3, 2.0 ** -15])
def test_mf_equals_fp32_scorer_and_oracle(cuda, thr, mf):
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=int(thr * 1e6) % 1000, hw=(160, 400))
    pts = ransac.flow_to_points(flow.to(cuda), torch.inverse(K).to(cuda))
    got = _scores(pts, thr=thr, mf=mf)
    _equal(got, _scores(pts, thr=thr, mf=0))
    for b in range(2):
        p = pts[b].cpu().numpy()
        ref = R.ransac5(np.ascontiguousarray(p[:, :2]), np.ascontiguousarray(p[:, 2:]), iters=2, thr=thr,
                        nthreads=16)
        assert np.array_equal(got[4][b].numpy(), ref["hyp_score"])
        assert int(got[3][b]) == ref["winner"] and int(got[2][b]) == ref["inliers"]


@pytest.mark.parametrize("mf", [2, 1])
def test_mf_full_size_vs_oracle(cuda, mf):
    """One full KITTI pair (N = 435,032) at H = 4096: every hypothesis score."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=77)
    pts = ransac.flow_to_points(flow.to(cuda), torch.inverse(K).to(cuda))
    E, P, inl, win, scores = _scores(pts, iters=8, mf=mf)
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
        got = _scores(pts, ns, iters=2, thr=1e-3, nt=nt, nr=nr, mf=2)
        _equal(got, _scores(pts, ns, iters=2, thr=1e-3, nt=nt, nr=nr, mf=0))
        for b, n in enumerate(ns):
            r = R.ransac5(rows[b][:, :2], rows[b][:, 2:], nt or n, nr or n, iters=2, thr=1e-3)
            assert np.array_equal(got[4][b].numpy(), r["hyp_score"])
            assert int(got[3][b]) == r["winner"] and int(got[2][b]) == r["inliers"]
