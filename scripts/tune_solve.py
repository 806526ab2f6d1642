"""In-process A/B of the solve launch shapes (results must not change)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
flow, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
# --sparse: the SIFT-keypoint branch (bench.py --config sparse, 2,048 keypoints per pair)
kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=dev), [2048] * B) if "--sparse" in sys.argv else None
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev, keypoints=kp)
E0, P0, inl0, _ = hp.pose(flow, K)
E0 = E0.clone(); inl0 = inl0.clone()

def timed(reps=3):
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(reps): hp.pose(flow, K)
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read("ransac_solve")
    return ms / max(n, 1)

res = {}
for rnd in range(3):
    for fl in (4, 8, 12, 16):
        for rl in (4, 8, 16, 32):
            _lib.tune("solve_lanes", fl); _lib.tune("roots_lanes", rl)
            res.setdefault((fl, rl), []).append(timed())
            E, P, inl, _ = hp.pose(flow, K)
            assert torch.equal(E, E0) and torch.equal(inl, inl0)
for k, v in sorted(res.items(), key=lambda t: sorted(t[1])[1]):
    print(f"solve_lanes={k[0]:2d} roots_lanes={k[1]:2d}  median {sorted(v)[1]:.4f} ms")
