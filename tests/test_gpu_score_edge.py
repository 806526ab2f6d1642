"""Decisions at the edges of the inlier test, through the RANSAC's own scorer
(sfm_score_essentials -> k_mf_cands + k_score_mf2: split-f16 matrix-core
decisions exact by bound, undecided -> float64 re-test).

For each essential matrix E the correspondences are built on purpose around
the decision e(x, x') = |x'^T E x| / sqrt(Ex0^2 + Ex1^2 + xE0^2 + xE1^2) = thr
(ComputeError, kernel_functions.cu:232-264): x' is moved off the epipolar line
of x along its normal until the reference-order float64 error is
  * exactly on the threshold: the two adjacent doubles of the offset between
    which e crosses thr (one an inlier by e <= thr, the other not), and
  * at e / thr = 1 -+ 1e-12, 1e-9, 1e-6, 1e-3 and 1 -+ 1 %, 2 %, 3 %, 4 %, 6 %:
    the edges of the split-f16 decision band (about +-3 % wide), where the
    certified matrix-core decisions and the float64 fallback take over from
    each other.
Each class of points is its own pair of the batch, so a count equals the
oracle's (the exact float64 reference order, oracle/ransac5_oracle.cpp) only
if every single decision does (the classes are one-sided).  Thresholds span
the matrix-core range 2^-15 .. 0.3, plus 1e-6 below it (the float32 VALU
scorer k_score32)."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as ORR

pytestmark = pytest.mark.gpu


def _score(data, Et, thr, dev):
    """Counts through sfm_score_essentials on the benched scorer, pinned:
    k_score_mf2 in the matrix-core threshold range [2^-15, 1), k_score32 below."""
    from sfm_amd import _lib, ransac
    _lib.tune("score_mf", 2)          # restored by conftest's tuning snapshot
    got = ransac.score_essentials(torch.from_numpy(data).to(dev), torch.from_numpy(Et).to(dev), thr).cpu().numpy()
    assert _lib.last_scorer() == ("k_score_mf2" if 2.0 ** -15 <= thr < 1.0 else "k_score32"), _lib.last_scorer()
    return got


def _err(E, q, qp):
    """The reference's error in its own operation order (float64, numpy)."""
    x = np.c_[q, np.ones(len(q))]
    xp = np.c_[qp, np.ones(len(qp))]
    Ex = np.zeros((len(q), 3))
    xE = np.zeros((len(q), 3))
    for k in range(3):
        s = np.zeros(len(q))
        for l in range(3):
            s = s + E[k, l] * x[:, l]
        Ex[:, k] = s
        s = np.zeros(len(q))
        for l in range(3):
            s = s + xp[:, l] * E[l, k]
        xE[:, k] = s
    a = np.zeros(len(q))
    for k in range(3):
        a = a + xp[:, k] * Ex[:, k]
    d = np.sqrt(Ex[:, 0] * Ex[:, 0] + Ex[:, 1] * Ex[:, 1] + xE[:, 0] * xE[:, 0] + xE[:, 1] * xE[:, 1])
    return np.abs(a / d)


def _essential(rng):
    a = rng.normal(size=3) * 0.05
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    R = np.eye(3) + np.sin(np.linalg.norm(a)) / max(np.linalg.norm(a), 1e-12) * K
    t = np.r_[rng.normal(size=2) * 0.3, 1.0]
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    return tx @ R * rng.uniform(0.3, 3.0)


def _offsets(E, q, target):
    """Per point the offset s along the epipolar line's normal with e = target
    (bisection in float64); returns (s_lo, s_hi) adjacent-ish doubles around it."""
    l = (E @ np.c_[q, np.ones(len(q))].T).T
    nrm = l[:, :2] / np.linalg.norm(l[:, :2], axis=1, keepdims=True)
    foot = q - 0.0  # any base point; project onto the line l' . (x', 1) = 0
    base = foot - ((l[:, :2] * foot).sum(1) + l[:, 2])[:, None] * l[:, :2] / (l[:, :2] ** 2).sum(1, keepdims=True)
    lo = np.zeros(len(q))
    hi = np.full(len(q), 0.05)
    f = lambda s: _err(E, q, base + s[:, None] * nrm)
    for _ in range(40):                         # widen until every point's bracket holds the crossing
        up = f(hi) <= target
        if not up.any():
            break
        hi = np.where(up, 2 * hi, hi)
    # far from the line the error saturates (a and x'^T E both grow with the
    # offset): at large thresholds some points never cross; they take a
    # crossing point's offset instead (the set stays one-sided per class)
    ok = f(hi) > target
    assert ok.sum() >= len(q) // 4
    src = np.flatnonzero(ok)
    fill = src[np.arange(len(q)) % len(src)]
    q[:] = np.where(ok[:, None], q, q[fill])
    base = np.where(ok[:, None], base, base[fill])
    nrm = np.where(ok[:, None], nrm, nrm[fill])
    hi = np.where(ok, hi, hi[fill])
    for _ in range(200):
        mid = 0.5 * (lo + hi)
        up = f(mid) > target
        hi = np.where(up, mid, hi)
        lo = np.where(up, lo, mid)
    return base, nrm, lo, hi


@pytest.mark.parametrize("thr", [1e-6, 2.0 ** -15, 1e-4, 1e-3, 0.3])
def test_decisions_at_the_threshold_and_band_edges(cuda, thr):
    from sfm_amd import ransac
    rng = np.random.default_rng(int(thr * 1e6) + 3)
    n_e, n_p = 6, 300
    Es = [_essential(rng) for _ in range(n_e)]
    classes = []            # (name, per-E (q, qp))
    rels = [1e-12, 1e-9, 1e-6, 1e-3, 1e-2, 2e-2, 3e-2, 4e-2, 6e-2]
    per_e = []
    for E in Es:
        q = rng.uniform(-0.6, 0.6, (n_p, 2))
        _offsets(E, q, thr * (1 + rels[-1]))   # the largest target first: fixes q (smaller targets all cross)
        base, nrm, lo, hi = _offsets(E, q, thr)
        pts = {"edge_in": base + lo[:, None] * nrm, "edge_out": base + hi[:, None] * nrm}
        for r in rels:
            for sgn, tag in ((-1, "in"), (1, "out")):
                b2, n2, l2, h2 = _offsets(E, q, thr * (1 + sgn * r))
                pts[f"{tag}_{r:g}"] = b2 + l2[:, None] * n2
        per_e.append((q, pts))
    names = list(per_e[0][1].keys())
    # one pair per class; all E's of the test are the candidates of every pair
    B = len(names)
    data = np.zeros((B, n_p, 4))
    for bi, nm in enumerate(names):
        # each class uses E_j's own points for point block j: build the pair from E_0's points only
        q, pts = per_e[0]
        data[bi, :, :2] = q
        data[bi, :, 2:] = pts[nm]
    Et = np.stack([np.stack(Es)] * B)
    got = _score(data, Et, thr, cuda)
    for bi, nm in enumerate(names):
        q = np.ascontiguousarray(data[bi, :, :2])
        qp = np.ascontiguousarray(data[bi, :, 2:])
        for ci, E in enumerate(Es):
            want = int(ORR.inlier_mask(E, q, qp, thr).sum())
            assert got[bi, ci] == want, (nm, ci, int(got[bi, ci]), want)
    # the constructed classes really sit where intended (for E_0, their own E)
    q, pts = per_e[0]
    e_in = _err(Es[0], q, pts["edge_in"])
    e_out = _err(Es[0], q, pts["edge_out"])
    assert (e_in <= thr).all() and (e_out > thr).all()
    assert got[names.index("edge_in"), 0] == n_p and got[names.index("edge_out"), 0] == 0


def test_every_e_on_its_own_band_edge(cuda):
    """Each candidate scored on points built at ITS OWN threshold crossing
    (both sides), thr = 1e-4 (SFMnet's default), many E's at once."""
    from sfm_amd import ransac
    rng = np.random.default_rng(11)
    thr = 1e-4
    n_e, n_p = 24, 128
    Es = [_essential(rng) for _ in range(n_e)]
    data = np.zeros((n_e, 2 * n_p, 4))
    for i, E in enumerate(Es):
        q = rng.uniform(-0.8, 0.8, (n_p, 2))
        base, nrm, lo, hi = _offsets(E, q, thr)
        data[i, :n_p, :2] = q
        data[i, :n_p, 2:] = base + lo[:, None] * nrm
        data[i, n_p:, :2] = q
        data[i, n_p:, 2:] = base + hi[:, None] * nrm
    Et = np.stack([np.stack(Es)] * n_e)
    got = _score(data, Et, thr, cuda)
    for i in range(n_e):
        q = np.ascontiguousarray(data[i, :, :2])
        qp = np.ascontiguousarray(data[i, :, 2:])
        for j, E in enumerate(Es):
            assert got[i, j] == int(ORR.inlier_mask(E, q, qp, thr).sum()), (i, j)
        assert got[i, i] == n_p            # exactly the inside half
