"""The oracle (CPU restatement) against the golden vectors generated from the
reference's own code (oracle/gen_golden.py).  Pins the oracle before it is
used as the checker of the HIP path."""
import numpy as np
import pytest
import torch

from oracle import ransac5 as R
from oracle import sweep as S


def test_solve5_bit_exact(golden):
    g = golden("solve5.npz")
    for i in range(len(g["q5"])):
        r = R.solve5(g["q5"][i], g["qp5"][i], cheir=True)
        assert r["nroots"] == g["nroots"][i]
        assert r["nP"] == g["nP"][i]
        nr = max(r["nroots"], 0)
        assert np.array_equal(r["E_roots"][:nr].view(np.uint64), g["E_roots"][i][:nr].view(np.uint64)), i
        k = r["nP"]
        assert np.array_equal(r["E"][:k].view(np.uint64), g["E"][i][:k].view(np.uint64)), i
        assert np.array_equal(r["P"][:k].view(np.uint64), g["P"][i][:k].view(np.uint64)), i
        if k == 0 and nr > 0:   # slot 0 keeps root 0's E when nothing passes cheirality
            assert np.array_equal(r["E"][0], g["E"][i][0])


def test_solve5_no_cheirality(golden):
    g = golden("solve5.npz")
    for i in range(0, len(g["q5"]), 7):
        r = R.solve5(g["q5"][i], g["qp5"][i], cheir=False)
        assert r["nroots"] == g["nroots_nc"][i]
        nr = max(r["nroots"], 0)
        assert np.array_equal(r["E"][:nr], g["E_nc"][i][:nr])


def test_solve5_finds_true_essential(golden):
    """Known-answer: on exact geometric tuples one root reproduces the
    epipolar constraint to ~1e-12 (essential_matrix_main.cu:227-233 style)."""
    g = golden("solve5.npz")
    for i in range(600, 800):
        r = R.solve5(g["q5"][i], g["qp5"][i], cheir=False)
        assert r["nroots"] >= 1
        q = np.c_[g["q5"][i], np.ones(5)]
        qp = np.c_[g["qp5"][i], np.ones(5)]
        for E in r["E"][: r["nroots"]]:
            E = E.reshape(3, 3)
            res = np.abs(np.einsum("ni,ij,nj->n", qp, E, q)).max() / np.abs(E).max()
            assert res < 1e-8


@pytest.mark.parametrize("case", ["dense_tr_equal", "harness_style", "no_cheirality", "tight_threshold",
                                  "test_gt_ransac", "tiny_n"])
def test_ransac_matches_reference(golden, case):
    g = golden("ransac.npz")[case]
    n, nt, nr, it, thr, cheir, seed = g["params"]
    r = R.ransac5(g["q"], g["qp"], int(nt), int(nr), int(it), float(thr), seed=int(seed), cheir=bool(cheir))
    assert r["winner"] == int(g["winner"])
    assert r["inliers"] == int(g["inliers"])
    assert np.array_equal(r["E"], g["E"])
    assert np.array_equal(r["P"], g["P"])
    assert np.array_equal(r["hyp_score"], g["hyp_score"])
    assert np.array_equal(r["hyp_ncand"], g["hyp_ncand"])
    m = R.inlier_mask(r["E"], g["q"], g["qp"], float(thr))
    assert np.array_equal(m, g["mask"])
    assert int(m[: int(nr)].sum()) == r["inliers"]


def test_sampler_golden(golden):
    g = golden("sampler.npz")
    for a, s in enumerate(g["seeds"]):
        for b, h in enumerate(g["hs"]):
            for d in range(5):
                assert R.philox_u32(int(s), int(h), d) == g["u32"][a, b, d]
                for c, n in enumerate(g["ns"]):
                    assert R.sample_index(int(s), int(h), d, int(n)) == g["idx"][a, b, d, c]


def test_sampler_range_and_spread():
    n = 435032
    idx = np.array([R.sample_index(1234, h, d, n) for h in range(2000) for d in range(5)])
    assert idx.min() >= 0 and idx.max() <= n - 1
    # roughly uniform: each decile populated
    hist = np.histogram(idx, bins=10, range=(0, n))[0]
    assert hist.min() > 0.07 * len(idx)


def test_irls_and_decompose(golden):
    g = golden("irls.npz")
    for k, c in g.items():
        assert np.array_equal(R.optimise(c["q"], c["qp"], c["E_init"], 0.001, 0.0, 200), c["E_opt"]), k
        assert np.array_equal(R.optimise(c["q"], c["qp"], c["E_init"], 0.002, 1.0, 20), c["E_opt_huber"]), k
        assert np.array_equal(R.decompose(c["E_init"]), c["params"])
        U, V = R.decompose_uv(c["E_init"])
        assert np.array_equal(U, c["U"]) and np.array_equal(V, c["V"])
        # E = U diag(1,1,0) V^T up to scale
        E = c["E_init"] / np.linalg.norm(c["E_init"]) * np.sqrt(2)
        rec = U @ np.diag([1.0, 1.0, 0.0]) @ V.T
        assert min(np.abs(rec - E).max(), np.abs(rec + E).max()) < 1e-9


def test_inverse_warp_oracle(golden):
    g = golden("warp.npz")["warp"]
    K = torch.from_numpy(g["K"]); Ki = torch.from_numpy(g["Kinv"]); f = torch.from_numpy(g["feat"])
    for k in range(g["depth"].shape[0]):
        out = S.inverse_warp(f, torch.from_numpy(g["depth"][k]), torch.from_numpy(g["pose"][k]), K, Ki)
        assert torch.equal(out, torch.from_numpy(g["out"][k]))


def test_cost_volume_oracle(golden):
    g = golden("warp.npz")["cost"]
    cost = S.plane_sweep_cost(torch.from_numpy(g["ref"]), torch.from_numpy(g["tgt"]), torch.from_numpy(g["pose"]),
                              torch.from_numpy(g["K"]), torch.from_numpy(g["Kinv"]), int(g["nlabel"]),
                              float(g["min_depth"]), rescale=float(g["norm_target"]))
    assert torch.equal(cost, torch.from_numpy(g["cost"]))


def test_flow2depth_oracle(golden):
    g = golden("warp.npz")["flow2depth"]
    out = S.flow2depth(torch.from_numpy(g["R"]), torch.from_numpy(g["T"]), torch.zeros(*g["shape"].tolist()),
                       torch.from_numpy(g["K"]))
    assert torch.allclose(out, torch.from_numpy(g["out"]), rtol=0, atol=1e-5)


MODES = ("round", "sample_sp", "sift_pose")


def test_flow_oracle_matches_reference_correspondences(golden):
    """oracle/flow.py vs the float64 correspondences the reference's own
    SFMnet.pose_by_ransac hands to essential_matrix.computeP (corr.npz, made by
    oracle/gen_golden.py:gen_corr): bit-identical in every branch."""
    from oracle import flow as OF
    g = golden("corr.npz")
    inp = g["input"]
    flow, Ki = inp["flow"], inp["Kinv"]
    for name, side in (("dense", None), ("dense_side", inp["side"])):
        f = flow if side is None else np.ascontiguousarray(flow[:, :, :side[0], :side[1]])
        q, qp = OF.dense_correspondences(f, Ki)
        assert np.array_equal(q, g[name]["q"]) and np.array_equal(qp, g[name]["qp"]), name
        assert list(g[name]["num_test"]) == [q.shape[1]] * 2           # SFMnet.py:269: N for both counts
    for mode in MODES:
        for b in range(flow.shape[0]):
            q, qp = OF.keypoint_correspondences(flow[b], Ki[b], inp["kp1"][b], inp["kp2"][b], mode=mode)
            assert np.array_equal(q, g[mode]["q"][b]) and np.array_equal(qp, g[mode]["qp"][b]), (mode, b)


@pytest.mark.parametrize("prec", [32, 16])
def test_lowp_inlier_oracle_matches_numpy(prec):
    """ransac5_oracle.cpp:is_inlier_lp (software half rounding h16) vs numpy's
    own float16 / float32 arithmetic, on geometric and random E of very
    different scales (the power-of-two normalisation) and thresholds."""
    from oracle.gen_golden import geometric_scene
    rng = np.random.default_rng(prec)
    q, qp = geometric_scene(rng, 4000, out_frac=0.3, noise=0.003)
    r = R.ransac5(q, qp, iters=1, thr=1e-3, nchains=32)
    Es = [r["E"], r["E"] * 1e-7, r["E"] * 3e6] + [rng.normal(size=(3, 3)) * s for s in (1e-9, 1.0, 1e9)]
    for E in Es:
        for thr in (1e-4, 1e-3, 1e-2, 0.5):
            a = R.inlier_mask(E, q, qp, thr, prec)
            b = R.inlier_mask_numpy(E, q, qp, thr, prec)
            assert np.array_equal(a, b), (thr, int((a != b).sum()))


@pytest.mark.parametrize("prec", [33, 17])
def test_lowp_template_oracle_matches_numpy(prec):
    """ransac5_oracle.cpp:is_inlier_lp_tpl -- the literal ComputeError<T> with the
    reference's double Ematrix (kernel_functions.cu:231-264, common.h:26) -- vs
    numpy's float64 products / float16|float32 roundings, on geometric and random
    E of very different scales (no normalisation in this form: tiny E underflow
    in half) and thresholds.  In half the two low-precision forms differ.""" 
    from oracle.gen_golden import geometric_scene
    rng = np.random.default_rng(prec)
    q, qp = geometric_scene(rng, 4000, out_frac=0.3, noise=0.003)
    r = R.ransac5(q, qp, iters=1, thr=1e-3, nchains=32)
    Es = [r["E"], r["E"] * 1e-7, r["E"] * 3e6] + [rng.normal(size=(3, 3)) * s for s in (1e-9, 1.0, 1e3)]
    differs = 0
    for E in Es:
        for thr in (1e-4, 1e-3, 1e-2, 0.5):
            a = R.inlier_mask(E, q, qp, thr, prec)
            b = R.inlier_mask_numpy_tpl(E, q, qp, thr, prec)
            assert np.array_equal(a, b), (thr, int((a != b).sum()))
            differs += int((a != R.inlier_mask(E, q, qp, thr, prec - 1)).sum())
    assert prec == 33 or differs > 0


def test_psnet64_fixture_clear_of_border_step_and_oracle_chain(golden):
    """psnet64.npz (the float64 depth bar): every plane-sweep sample stays
    PSNET64_MARGIN clear of the reference's border step (inverse_warp.py:60-66,
    a sample beyond |xn| = 1 is zeroed, so a float32 rounding near it moves
    the depth by percent) and the torch-CPU oracle chain (sweep -> the
    reference's module forward -> head) meets the GPU test's bars against the
    float64 depth: median <= 1e-5, max <= 1e-4 relative."""
    from oracle import regularize as OR
    from oracle.gen_golden import PSNET64_MARGIN, sweep_boundary_margin
    from sfm_amd.regularize import CostRegularization
    g = golden("psnet64.npz")
    inp = g["input"]
    L = int(inp["nlabel"])
    H, W = (int(x) for x in inp["image_hw"])
    m = sweep_boundary_margin(inp["K"], inp["pose_rescaled"][:, 0], L, H // 4, W // 4)
    assert m >= PSNET64_MARGIN and m == float(inp["boundary_margin"])
    mod = CostRegularization(64)
    mod.load_state_dict({k: torch.from_numpy(v) for k, v in g["state"].items()})
    t = lambda k: torch.from_numpy(inp[k])
    cost = S.plane_sweep_cost(t("ref_fea"), t("tgt_fea"), t("pose_rescaled")[:, 0], t("K"), t("Kinv"), L, 1.0)
    dep = S.depth_head(OR.regularize_fp32(mod, cost), L, 1.0, out_hw=(H, W))
    want = torch.from_numpy(g["out64"]["depth"]).double()
    r = ((dep.double() - want).abs() / want.abs()).flatten()
    assert float(r.median()) <= 1e-5 and float(r.max()) <= 1e-4, (float(r.median()), float(r.max()))


def test_lowp_template_half_overflow_makes_every_point_an_inlier():
    """The literal ComputeError<half> with the reference's double Ematrix:
    an unnormalised candidate (|E| in the hundreds, as 5-point roots give)
    overflows half's 65504 in d = sqrt(Ex0^2 + ...), so error = xEx / inf = 0
    and every point counts as an inlier -- the C5 sweep's degenerate winners
    (DESIGN.md §2.3).  The held-in-T form scales E by a power of two first and
    is scale-invariant."""
    rng = np.random.default_rng(0)
    q = rng.uniform(-0.5, 0.5, (1000, 2))
    qp = rng.uniform(-0.5, 0.5, (1000, 2))
    E = rng.normal(size=(3, 3))
    assert not R.inlier_mask_numpy_tpl(E, q, qp, 1e-4, 17).any()
    assert R.inlier_mask_numpy_tpl(E * 1000, q, qp, 1e-4, 17).mean() > 0.99
    assert np.array_equal(R.inlier_mask(E * 1000, q, qp, 1e-4, 17), R.inlier_mask_numpy_tpl(E * 1000, q, qp, 1e-4, 17))
    assert np.array_equal(R.inlier_mask(E * 1000, q, qp, 1e-4, 16), R.inlier_mask(E, q, qp, 1e-4, 16))
