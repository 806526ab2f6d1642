"""Sweep launch time in the bench context (right after the RANSAC step) vs
after an idle gap, for the per-row, aligned-slab and narrow-window kernels."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath

dev = torch.device("cuda", 0)
B = 8
flow, K, pose_gt, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
ref, tgt = synth.features(B, 32, 94, 311, device=dev)
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
E, P, inl, _ = hp.pose(flow, K)
torch.cuda.synchronize()


def sweep_ms(n):
    ms, k = _lib.profile_read("plane_sweep")
    return ms / max(k, 1)


for rnd in range(2):
    for flat, grp, nj in ((1, 8, 1), (2, 8, 1), (2, 8, 2), (2, 4, 2), (2, 8, 4)):
        _lib.tune("sweep_flat", flat); _lib.tune("sweep_group", grp); _lib.tune("sweep_nj", nj)
        res = {}
        for mode in ("after_ransac", "gap_5ms", "gap_50ms", "sweep_only"):
            for _ in range(2):
                hp.step(flow, K, ref, tgt)
            torch.cuda.synchronize()
            per = []
            for _ in range(6):
                _lib.profile_reset(); _lib.profile_enable(True)
                if mode != "sweep_only":
                    hp.pose(flow, K)
                    if mode.startswith("gap"):
                        torch.cuda.synchronize()
                        time.sleep(0.005 if mode == "gap_5ms" else 0.05)
                hp.sweep(ref, tgt, P.clone(), K)
                torch.cuda.synchronize(); _lib.profile_enable(False)
                per.append(sweep_ms(1))
            res[mode] = per
        print(f"flat={flat} group={grp} nj={nj}: " + "; ".join(f"{m} {[round(x, 3) for x in v]}" for m, v in res.items()),
              flush=True)
_lib.tune("sweep_flat", 2); _lib.tune("sweep_group", 8); _lib.tune("sweep_nj", 1)
