"""k_solve_front with the cooperative equations and reduction (tuning key
solve_coop = 1: build_equations_quad / quad_reduce in five_point.h, one DPP
quad per hypothesis) against the one-lane path it replaces (solve_coop = 0):
the whole RANSAC workspace -- the solve state between the kernels (E basis,
reduced equation blocks, samples, determinant polynomial), every hypothesis'
roots, candidates and scores -- must be byte-identical after a full pose
stage, on the dense bench workload, the sparse keypoint branch, the B=32
batched C3 shape, and with fewer than 16 hypotheses per wave (solve_lanes)
and a hypothesis count that leaves the last wave partly empty.  The one-lane
path is pinned to the reference by test_gpu_ransac.py (golden vectors, the
oracle at H=4096).

Bar: bit-exact (integer and float64 bytes), except the payload and sign of
NaN values: degenerate samples (duplicate keypoints) give NaN determinant
coefficients, and which NaN an operation on NaN inputs returns depends on the
compiler's operand order in each instantiation (IEEE 754 leaves it open).  A
differing 8-byte word passes only if it is a NaN in both runs; every root,
candidate, score, E and P stays byte-identical (scripts/solve_coop_diff.py:
19 of 32,768 sparse hypotheses, all in determinant fields)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pose_workspace(hp, flow, K, coop, lanes):
    from sfm_amd import _lib
    prev = (_lib.tune_get("solve_coop"), _lib.tune_get("solve_lanes"))
    _lib.tune("solve_coop", coop)
    _lib.tune("solve_lanes", lanes)
    try:
        hp.ws.zero_()
        out = hp.pose(flow, K)
        torch.cuda.synchronize()
        return hp.ws.clone(), [t.clone() for t in out if torch.is_tensor(t)]
    finally:
        _lib.tune("solve_coop", prev[0])
        _lib.tune("solve_lanes", prev[1])


@pytest.mark.parametrize("mode,lanes,iters", [("dense", 16, 8), ("sparse", 16, 8), ("batch32", 16, 8),
                                              ("dense", 12, 8), ("sparse", 16, 3)])
def test_solve_coop_bit_identical(cuda, mode, lanes, iters):
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    B = 32 if mode == "batch32" else 8
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000 + B, device=cuda)
    kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=cuda), [2048] * B) if mode == "sparse" else None
    hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, iters, 1e-4, 1.0, True, 0.6, device=cuda,
                        keypoints=kp)
    ws0, out0 = _pose_workspace(hp, flow, K, 0, lanes)
    ws1, out1 = _pose_workspace(hp, flow, K, 1, lanes)
    w0, w1 = ws0.view(torch.float64), ws1.view(torch.float64)
    diff = ws0.view(torch.int64) != ws1.view(torch.int64)
    assert bool((w0[diff].isnan() & w1[diff].isnan()).all()), \
        "workspace bytes differ between the one-lane and the quad solve"
    assert int(diff.sum()) <= 64
    for a, b in zip(out0, out1):
        assert torch.equal(a, b)


def test_pose_workspace_repeatable(cuda):
    """Two identical pose stages leave byte-identical workspaces: nothing
    schedule-dependent survives a launch (k_score_mf2's range-claim counters
    are zeroed by its last block; the float64 drains only add counts)."""
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    B = 8
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=1008, device=cuda)
    hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=cuda)
    ws0, out0 = _pose_workspace(hp, flow, K, 1, 16)
    ws1, out1 = _pose_workspace(hp, flow, K, 1, 16)
    assert torch.equal(ws0, ws1)
    for a, b in zip(out0, out1):
        assert torch.equal(a, b)
