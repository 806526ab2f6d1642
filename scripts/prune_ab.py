"""Score-kernel time and skipped evaluations with exact bound pruning on / off
and the MFMA kernel on / off (KITTI B=8, H=4096, the bench workload)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, ransac, synth
from sfm_amd.pipeline import TwoViewHotPath

dev = torch.device("cuda", 0)
B = 8
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
ref = None
for rnd in range(2):
    for prune, mx in ((0, 0), (1, 0), (0, 1), (1, 1)):
        _lib.tune("score_prune", prune)
        _lib.tune("score_mfma", mx)
        hp.pose(flow, K)
        torch.cuda.synchronize()
        _lib.profile_reset(); _lib.profile_enable(True)
        for _ in range(3):
            E, P, inl, win = hp.pose(flow, K)
        torch.cuda.synchronize(); _lib.profile_enable(False)
        ms, n = _lib.profile_read("ransac_score")
        sk = ransac.skipped_evaluations(hp.ws, B, 8)
        out = (E.cpu(), inl.cpu(), win.cpu())
        if ref is None:
            ref = out
        same = all(torch.equal(a, b) for a, b in zip(out, ref))
        print(f"prune={prune} mfma={mx}: score {ms / n:.3f} ms, skipped {sk}, same result {same}", flush=True)
_lib.tune("score_prune", 1)
_lib.tune("score_mfma", 1)
