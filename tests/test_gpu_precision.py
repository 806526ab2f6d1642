"""Reduced-precision inlier scoring (tuning key score_precision; BASELINE.json
configs[4], C5: LO-RANSAC 8192 hypotheses + local E refinement, fp32 vs fp16
inlier-set parity sweep).

* 32 / 16 evaluate ComputeError<float> / <half> with E held in T
  (ransac5.hip:inlier_lowp): bit-exact against the oracle's restatement
  (ransac5_oracle.cpp:is_inlier_lp), itself checked against numpy
  float16/float32 arithmetic on the CPU.
* 33 / 17 are the literal template form (double Ematrix, double products,
  sums rounded to T; ransac5.hip:inlier_lowp_tpl vs is_inlier_lp_tpl).
* C5 at full size: one KITTI pair (N = 435,032), H = 8192, each precision's
  winner refined by the GPU IRLS (optimise); the agreement table of
  DESIGN.md §C5 is asserted here against its documented bounds."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R

pytestmark = pytest.mark.gpu


def _scene(seed, n=3000):
    from oracle.gen_golden import geometric_scene
    return geometric_scene(np.random.default_rng(seed), n, out_frac=0.2, noise=0.002)


@pytest.mark.parametrize("prec", [32, 16, 33, 17])
@pytest.mark.parametrize("thr", [1e-3, 1e-2])
def test_lowp_scoring_bit_exact_vs_oracle(cuda, prec, thr):
    """32 / 16: E and every operation held in T; 33 / 17: the literal
    ComputeError<T> with the reference's double Ematrix (is_inlier_lp_tpl)."""
    from sfm_amd import ransac
    q, qp = _scene(int(prec + 1e4 * thr))
    pts = torch.from_numpy(np.c_[q, qp]).unsqueeze(0).to(cuda)
    E, P, inl, win, scores = ransac.ransac5_batched(pts, iters=2, threshold=thr, return_scores=True, precision=prec)
    ref = R.ransac5(q, qp, iters=2, thr=thr, prec=prec)
    assert int(win[0]) == ref["winner"] and int(inl[0]) == ref["inliers"]
    assert np.array_equal(scores[0].cpu().numpy(), ref["hyp_score"])
    assert np.array_equal(E[0].cpu().numpy(), ref["E"]) and np.array_equal(P[0].cpu().numpy(), ref["P"])
    # the default is restored: the next call is the exact float64 path
    E64, _, inl64, win64 = ransac.ransac5_batched(pts, iters=2, threshold=thr)
    ref64 = R.ransac5(q, qp, iters=2, thr=thr)
    assert int(win64[0]) == ref64["winner"] and int(inl64[0]) == ref64["inliers"]


def _unit(E):
    E = E / np.linalg.norm(E)
    k = np.argmax(np.abs(E))
    return E * np.sign(E.flat[k])


def test_c5_precision_sweep(cuda):
    """C5: fp64 (exact) vs fp32 vs fp16 scoring (both low-precision forms) on 4 full-size KITTI pairs,
    H = 8192 (ransac_iter 16), thresholds 1e-4 (the default) and 1e-3, each
    winner refined by optimise (GPU IRLS, polish_E.cu:1470-1577).  Reported
    per (pair, threshold, precision): the winner, its count under its own
    scoring, |symmetric difference| of its inlier set vs fp64's (both sets
    under the exact fp64 test), relative E error before / after refinement."""
    from sfm_amd import _lib, ransac, synth
    B = 4
    flow, K, pose, _ = synth.kitti_pair_batch(B, seed=31)
    pts = ransac.flow_to_points(flow.to(cuda), torch.inverse(K).to(cuda))
    N = pts.shape[1]
    rows = []
    for thr in (1e-4, 1e-3):
        res = {}
        for prec in (64, 32, 16, 33, 17):
            _lib.profile_reset(); _lib.profile_enable(True)
            E, P, inl, win = ransac.ransac5_batched(pts, iters=16, threshold=thr, precision=prec)
            torch.cuda.synchronize()
            _lib.profile_enable(False)
            ms, _ = _lib.profile_read("ransac_score")
            Eo = ransac.optimise_batched(pts, E, 0.001, 0.0, 200)
            mask = ransac.inlier_mask(pts, E, thr).cpu().numpy()
            res[prec] = dict(win=win.cpu().numpy(), inl=inl.cpu().numpy(), E=E.cpu().numpy(), Eo=Eo.cpu().numpy(),
                             mask=mask, ms=ms)
        for prec in (64, 32, 16, 33, 17):
            r = res[prec]
            for b in range(B):
                sd = int(np.count_nonzero(r["mask"][b] ^ res[64]["mask"][b]))
                eE = float(np.linalg.norm(_unit(r["E"][b]) - _unit(res[64]["E"][b])))
                eO = float(np.linalg.norm(_unit(r["Eo"][b]) - _unit(res[64]["Eo"][b])))
                same = int(r["win"][b]) == int(res[64]["win"][b])
                rows.append(dict(thr=thr, prec=prec, b=b, same=same, inl=int(r["inl"][b]),
                                 inl64=int(res[64]["inl"][b]), sd=sd, eE=eE, eO=eO))
                print(f"C5 thr={thr:g} prec={prec} pair {b}: winner {int(r['win'][b])} "
                      f"({'=' if same else '!='} fp64) count {int(r['inl'][b])} vs {int(res[64]['inl'][b])} "
                      f"symdiff {sd} ({sd / N:.1e} of N) |dE| {eE:.2e} |dE_opt| {eO:.2e}")
            print(f"C5 thr={thr:g} prec={prec}: score kernel {r['ms']:.2f} ms for {B} pairs")
    # fp32: ComputeError<float> moves counts by a handful of points; the
    # winning hypothesis and the refined pose agree with fp64
    r32 = [r for r in rows if r["prec"] == 32]
    assert all(r["same"] for r in r32)
    assert all(abs(r["inl"] - r["inl64"]) <= 1e-3 * r["inl64"] for r in r32)
    assert all(r["eO"] <= 1e-9 for r in r32)
    # fp16 (half ulp at 1 is 4.9e-4, above the 1e-4 threshold): counts drop by
    # up to 3.3 % and at 1e-3 the winner can move to a near-equivalent
    # hypothesis, but the refined pose matches fp64's (measured <= 2.4e-7)
    r16 = [r for r in rows if r["prec"] == 16]
    assert all(r["eO"] <= 1e-5 for r in r16)
    assert all(abs(r["inl"] - r["inl64"]) <= 5e-2 * r["inl64"] for r in r16)
    # the literal template forms (33 / 17: double E and products, sums rounded
    # to T) are reported beside them; parity unpinned against the reference,
    # bounds recorded in DESIGN.md from this table
    for r in rows:
        if r["prec"] in (33, 17):
            assert np.isfinite(r["eE"]) and np.isfinite(r["eO"])
