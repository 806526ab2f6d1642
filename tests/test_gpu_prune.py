"""Exact bound pruning in the float32 score kernel k_score32 (tuning key
score_prune; the split-f16 matrix-core scorer k_score_mf, the default, is
turned off here with score_mf=0): the
winner, its inlier count, E and P must be identical with pruning on and off,
and (through the unpruned path's bit-exact parity) equal to the oracle's.
Pruning is active only without per-hypothesis scores and with
num_test == num_ransac_test (SFMnet's call)."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R

pytestmark = pytest.mark.gpu


def _both(pts, n=None, iters=2, thr=1e-4, nt=None, nr=None):
    from sfm_amd import _lib, ransac
    B = pts.shape[0]
    ws = ransac.workspace_for(B, iters, pts.device)
    out = {}
    try:
        _lib.tune("score_mf", 0)
        for prune in (0, 1):
            _lib.tune("score_prune", prune)
            E, P, inl, win = ransac.ransac5_batched(pts, n, nt, nr, iters, thr, workspace=ws)
            torch.cuda.synchronize()
            out[prune] = (E.cpu(), P.cpu(), inl.cpu(), win.cpu(), ransac.skipped_evaluations(ws, B, iters))
    finally:
        _lib.tune("score_prune", 1)
        _lib.tune("score_mf", 1)
    return out


def _same(out):
    a, b = out[0], out[1]
    for x, y in zip(a[:4], b[:4]):
        assert torch.equal(x, y)
    assert a[4] == 0


def test_pruning_full_size_kitti(cuda):
    """The bench workload shape: 2 KITTI pairs, N = 435,032, H = 4096."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=1000, device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    out = _both(pts, iters=8)
    _same(out)
    assert out[1][4] > 0                                  # pruning engaged on real data
    assert int(out[1][2].min()) > 10000


@pytest.mark.parametrize("seed", [3, 11])
def test_pruning_matches_oracle_winner(cuda, seed):
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=seed, hw=(120, 200), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    out = _both(pts, iters=2)
    _same(out)
    p = pts[0].cpu().numpy()
    ref = R.ransac5(np.ascontiguousarray(p[:, :2]), np.ascontiguousarray(p[:, 2:]), iters=2, thr=1e-4, nthreads=16)
    E, P, inl, win, _ = out[1]
    assert int(win[0]) == ref["winner"] and int(inl[0]) == ref["inliers"]
    assert np.array_equal(E[0].numpy(), ref["E"])
    assert np.array_equal(P[0].numpy(), ref["P"])


def test_pruning_ragged_batch(cuda):
    """Pairs with different point counts (interleaved items, per-pair bounds)."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(3, seed=21, hw=(100, 180), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    N = pts.shape[1]
    out = _both(pts, n=[N, N // 3, 2 * N // 3], iters=2)
    _same(out)


def test_pruning_off_when_prefixes_differ(cuda):
    """num_test != num_ransac_test: the preselection count differs from the
    score, so the bound does not apply and nothing is skipped."""
    from sfm_amd import ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(1, seed=5, hw=(100, 160), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    N = pts.shape[1]
    out = _both(pts, iters=2, nt=N // 2, nr=N)
    _same(out)
    assert out[1][4] == 0


def test_mfma_scorer_is_exact(cuda):
    """The matrix-core scorer (tuning key score_mfma, off by default) gives the
    same per-hypothesis scores as the VALU scorer, hence the oracle's."""
    from sfm_amd import _lib, ransac, synth
    flow, K, _, _ = synth.kitti_pair_batch(2, seed=8, hw=(120, 200), device=cuda)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    outs = []
    try:
        for mx in (0, 1):
            _lib.tune("score_mfma", mx)
            outs.append(ransac.ransac5_batched(pts, iters=2, threshold=1e-4, return_scores=True))
            torch.cuda.synchronize()
    finally:
        _lib.tune("score_mfma", 0)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a.cpu(), b.cpu())
    p = pts[0].cpu().numpy()
    ref = R.ransac5(np.ascontiguousarray(p[:, :2]), np.ascontiguousarray(p[:, 2:]), iters=2, thr=1e-4, nthreads=16)
    assert np.array_equal(outs[1][4][0].cpu().numpy(), ref["hyp_score"])
