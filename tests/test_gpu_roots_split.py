"""k_roots_split (five_point.h: isolate_p1 / falsi_tasks / bisect_deferred),
with per-wave task lists (roots_split=1) and with one pool per block of four
waves (roots_split=2, the default), against k_roots, the single-loop isolation
it replaces (roots_split=0): the whole RANSAC workspace -- every hypothesis' roots and root
count, its candidates, their scores -- must be byte-identical after a full
pose stage, on the dense bench workload, the sparse keypoint branch and the
B=32 batched C3 shape.  k_roots itself is pinned to the reference by
test_gpu_ransac.py (golden vectors, the oracle at H=4096).

Bar: bit-exact (integer and float64 bytes)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pose_workspace(hp, flow, K, split):
    from sfm_amd import _lib
    prev = _lib.tune_get("roots_split")
    _lib.tune("roots_split", split)
    try:
        hp.ws.zero_()
        out = hp.pose(flow, K)
        torch.cuda.synchronize()
        return hp.ws.clone(), [t.clone() for t in out if torch.is_tensor(t)]
    finally:
        _lib.tune("roots_split", prev)


@pytest.mark.parametrize("mode", ["dense", "sparse", "batch32"])
def test_roots_split_bit_identical(cuda, mode):
    from sfm_amd import synth
    from sfm_amd.pipeline import TwoViewHotPath
    B = 32 if mode == "batch32" else 8
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000 + B, device=cuda)
    kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=cuda), [2048] * B) if mode == "sparse" else None
    hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=cuda, keypoints=kp)
    ws0, out0 = _pose_workspace(hp, flow, K, 0)
    for split in (1, 2):                 # per-wave task lists; one pool per block of four waves
        ws1, out1 = _pose_workspace(hp, flow, K, split)
        assert torch.equal(ws0, ws1), f"workspace bytes differ between k_roots and roots_split={split}"
        for a, b in zip(out0, out1):
            assert torch.equal(a, b)
