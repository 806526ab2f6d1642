"""Exact count-bound pruning, in both scorers that have it:

  * k_score_mf2 (the default and benched scorer; tuning key score_mf_prune):
    every candidate scored on the first 880 per mille of each pair's spans,
    then up to the pair's pruning point (k_mf2_split: 1 - estimated inlier
    ratio + margin), k_mf2_lead / k_mf2_keep keep the candidates whose bound
    can still reach the leader's exact count, a last launch scores those on
    the rest;
  * k_score32 (the float32 VALU scorer, score_mf=0; tuning key score_prune,
    PruneState).

The winner, its inlier count, E and P must be identical with pruning on and
off, and (through the unpruned path's bit-exact parity) equal to the
oracle's.  Pruning is active only without per-hypothesis scores and with
num_test == num_ransac_test (SFMnet's call).  Every call asserts the kernel
it dispatched."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R

pytestmark = pytest.mark.gpu


def _both(pts, n=None, iters=2, thr=1e-4, nt=None, nr=None, scorer="mf2"):
    """{0: unpruned, 1: pruned (k_score_mf2: the round-6 one-sided passes,
    score_mf_prune_upper = 1, the default), 2 (k_score_mf2 only): pruned with
    the round-5 two-sided passes} -> (E, P, inliers, winner, skipped
    evaluations, kept candidates (k_score_mf2 pruned: summed over the pairs;
    else None), candidates)."""
    from sfm_amd import _lib, ransac
    B = pts.shape[0]
    ws = ransac.workspace_for(B, iters, pts.device)
    out, kernels = {}, {}
    snap = _lib.tune_snapshot()
    try:
        _lib.tune("score_mf", 2 if scorer == "mf2" else 0)
        for prune in ((0, 1, 2) if scorer == "mf2" else (0, 1)):
            if scorer == "mf2":
                _lib.tune("score_mf_prune", 880 if prune else 0)
                _lib.tune("score_mf_prune_upper", 0 if prune == 2 else 1)
            else:
                _lib.tune("score_prune", prune)
            E, P, inl, win = ransac.ransac5_batched(pts, n, nt, nr, iters, thr, workspace=ws)
            torch.cuda.synchronize()
            kernels[prune] = _lib.last_scorer()
            kept = (int(ransac.kept_candidates(ws, B, iters).sum()) if scorer == "mf2" and prune else None)
            out[prune] = (E.cpu(), P.cpu(), inl.cpu(), win.cpu(), ransac.skipped_evaluations(ws, B, iters), kept,
                          int(sum(ransac.candidate_counts(ws, B, iters))))
    finally:
        _lib.tune_restore(snap)
    return out, kernels


def _same(out):
    a = out[0]
    for k in out:
        for x, y in zip(a[:4], out[k][:4]):
            assert torch.equal(x, y), k
    assert a[4] == 0


@pytest.mark.parametrize("scorer", ["mf2", "k32"])
def test_pruning_full_size_kitti(cuda, scorer):
    """The bench workload shape: 2 KITTI pairs, N = 435,032, H = 4096."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=1000, device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    out, kernels = _both(pts, iters=8, scorer=scorer)
    if scorer == "mf2":
        assert kernels == {0: "k_score_mf2", 1: "k_score_mf2+prune", 2: "k_score_mf2+prune"}
    else:
        assert kernels == {0: "k_score32", 1: "k_score32+prune"}
    _same(out)
    if scorer == "mf2":                                   # pruning engaged on real data:
        assert out[1][5] < 0.5 * out[1][6]                #   the one-sided form kept under half the candidates,
        assert out[2][4] > 0                              #   the two-sided form skipped evaluations
    else:
        assert out[1][4] > 0
    assert int(out[1][2].min()) > 10000


def test_mf2_pruning_full_size_vs_oracle(cuda):
    """One full KITTI pair through the default (pruned) launch against the
    oracle, with the share of skipped evaluations reported."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=1000, device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    out, kernels = _both(pts, iters=8)
    assert kernels[1] == "k_score_mf2+prune"
    _same(out)
    p = pts[0].cpu().numpy()
    ref = R.ransac5(p[:, :2], p[:, 2:], iters=8, thr=1e-4, nthreads=16)
    E, P, inl, win, _, kept, ncand = out[1]
    assert int(win[0]) == ref["winner"] and int(inl[0]) == ref["inliers"]
    assert np.array_equal(E[0].numpy(), ref["E"]) and np.array_equal(P[0].numpy(), ref["P"])
    total = int(ref["hyp_ncand"].clip(min=1).sum()) * p.shape[0]
    skipped = out[2][4]                                   # the round-5 two-sided form
    print(f"two-sided form: skipped {skipped} of {total} evaluations ({100.0 * skipped / total:.1f} %); "
          f"one-sided form: kept {kept} of {ncand} candidates")
    assert skipped > 0.03 * total
    assert kept < 0.5 * ncand


@pytest.mark.parametrize("upper", [1, 0])
@pytest.mark.parametrize("pm,margin", [(500, 25), (800, 0), (990, 25), (850, 200), (600, 100)])
def test_mf2_pruning_split_points(cuda, pm, margin, upper):
    """Other first-launch shares and margins (the keys' ranges, including a
    pruning point past 990: no pruning): the same results."""
    from sfm_amd import _lib, ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=5, hw=(200, 400), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    ref = ransac.ransac5_batched(pts, None, None, None, 2, 1e-3, return_scores=True)
    _lib.tune("score_mf_prune", pm)
    _lib.tune("score_mf_prune_margin", margin)
    _lib.tune("score_mf_prune_upper", upper)
    got = ransac.ransac5_batched(pts, None, None, None, 2, 1e-3)
    assert _lib.last_scorer() == "k_score_mf2+prune"
    for x, y in zip(got, ref[:4]):
        assert torch.equal(x, y)


@pytest.mark.parametrize("seed", [3, 11])
@pytest.mark.parametrize("scorer", ["mf2", "k32"])
def test_pruning_matches_oracle_winner(cuda, seed, scorer):
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=seed, hw=(200, 320), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    out, kernels = _both(pts, iters=2, scorer=scorer)
    assert kernels[1].endswith("+prune")
    _same(out)
    p = pts[0].cpu().numpy()
    ref = R.ransac5(np.ascontiguousarray(p[:, :2]), np.ascontiguousarray(p[:, 2:]), iters=2, thr=1e-4, nthreads=16)
    E, P, inl, win = out[1][:4]
    assert int(win[0]) == ref["winner"] and int(inl[0]) == ref["inliers"]
    assert np.array_equal(E[0].numpy(), ref["E"])
    assert np.array_equal(P[0].numpy(), ref["P"])


@pytest.mark.parametrize("scorer", ["mf2", "k32"])
def test_pruning_ragged_batch(cuda, scorer):
    """Pairs with different point counts (per-pair split points and bounds)."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(3, seed=21, hw=(240, 400), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    N = pts.shape[1]
    out, kernels = _both(pts, n=[N, N // 2, 2 * N // 3], iters=2, scorer=scorer)
    assert kernels[1].endswith("+prune")
    _same(out)


def test_mf2_pruning_off_for_short_pairs(cuda):
    """Pairs under 32 spans (e.g. 2,048 keypoints) run one launch."""
    from sfm_amd import _lib, ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=5, hw=(100, 160), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    ransac.ransac5_batched(pts, None, None, None, 2, 1e-4)
    assert _lib.last_scorer() == "k_score_mf2"


@pytest.mark.parametrize("scorer", ["mf2", "k32"])
def test_pruning_off_when_prefixes_differ(cuda, scorer):
    """num_test != num_ransac_test: the preselection count differs from the
    score, so the bound does not apply and nothing is skipped."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=5, hw=(200, 320), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    N = pts.shape[1]
    out, kernels = _both(pts, iters=2, nt=N // 2, nr=N, scorer=scorer)
    assert not kernels[1].endswith("+prune")
    _same(out)
    assert out[1][4] == 0


def test_mf2_pruning_adapts_to_the_indoor_inlier_ratio(cuda):
    """C4's indoor pairs hold ~10.5 % inliers: no candidate can be dropped
    before 1 - 0.105 of the points, so a fixed pruning point at 0.88 dropped
    nothing (round-5 first build); k_mf2_split moves it to ~0.92 and the
    pruned launch skips evaluations there too, with the same results."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=1000, hw=synth.INDOOR_HW, device=cuda, k=synth.INDOOR_K)
    pts = ransac.flow_to_points(flow, torch.inverse(K), synth.INDOOR_HW[0], synth.INDOOR_HW[1])
    out, kernels = _both(pts, iters=4)
    assert kernels[1] == "k_score_mf2+prune"
    _same(out)
    N = pts.shape[1]
    assert 0.05 < int(out[1][2].max()) / N < 0.12                 # the regime the test is about
    assert out[2][4] > 0 and out[1][5] < 0.5 * out[1][6]


@pytest.mark.parametrize("exact_max", [256, 4, 0])
def test_mf2_one_sided_exact_count_paths(cuda, exact_max):
    """The one-sided pruning counts the kept candidates exactly in float64
    (k_mf2_exact, pairs with at most score_mf_exact_max kept) or on the matrix
    cores (the two-sided k_score_mf2 through the index map, the other pairs):
    either way winner, count, E and P equal the unpruned run's, on KITTI-size
    pairs (2 pairs, full size) where both paths can occur in one batch."""
    from sfm_amd import _lib, ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=77, device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    ref = ransac.ransac5_batched(pts, None, None, None, 4, 1e-4, return_scores=True)
    assert _lib.last_scorer() == "k_score_mf2"
    ws = ransac.workspace_for(2, 4, pts.device)
    _lib.tune("score_mf_prune_upper", 1)
    _lib.tune("score_mf_exact_max", exact_max)
    got = ransac.ransac5_batched(pts, None, None, None, 4, 1e-4, workspace=ws)
    assert _lib.last_scorer() == "k_score_mf2+prune"
    for x, y in zip(got, ref[:4]):
        assert torch.equal(x, y)
    kept = ransac.kept_candidates(ws, 2, 4)
    assert int(kept.min()) >= 1 and int(kept.sum()) < 0.1 * sum(ransac.candidate_counts(ws, 2, 4))


@pytest.mark.parametrize("exact_max", [256, 0])
@pytest.mark.parametrize("noise_px,outlier_frac", [(0.0, 0.0), (0.0, 0.5), (0.5, 1.0)])
def test_mf2_pruning_ties_and_extremes(cuda, noise_px, outlier_frac, exact_max):
    """Noise-free pairs: many hypotheses count every point (or every true
    inlier) and tie at the top, so the one-sided pass must keep all of them
    and the winner is decided by the first-max rule alone (hundreds kept:
    past score_mf_exact_max, the two-sided matrix-core count through the
    index map).  All-outlier pairs: every count small, the pruning point near
    the end.  Pruned (both forms) == unpruned in every case."""
    from sfm_amd import _lib, ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=9, hw=(200, 320), noise_px=noise_px,
                                           outlier_frac=outlier_frac, device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    N = pts.shape[1]
    ref = ransac.ransac5_batched(pts, None, None, None, 2, 1e-4, return_scores=True)
    _lib.tune("score_mf_exact_max", exact_max)
    out, kernels = _both(pts, iters=2)
    assert kernels[1] == "k_score_mf2+prune" and kernels[2] == "k_score_mf2+prune"
    _same(out)
    for x, y in zip(out[1][:4], ref[:4]):
        assert torch.equal(x, y.cpu())
    inl, scores = ref[2].cpu(), ref[4].cpu()
    ties = (scores == inl[:, None]).sum(dim=1)
    if outlier_frac == 0.0:                       # the regime: (nearly) every point an inlier, many-way ties
        assert int(inl.min()) > 0.99 * N and int(ties.min()) > 10
    elif outlier_frac == 0.5:
        assert 0.4 * N < int(inl.min()) and int(inl.max()) < 0.7 * N
    else:
        assert int(inl.max()) < 0.5 * N
    if outlier_frac < 1.0:
        assert int(out[1][5]) >= int(ties.sum())  # every tied hypothesis' candidate was kept
