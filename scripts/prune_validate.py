"""Round-5 validation sweep (GPU box): the pruned default scorer against the
unpruned one on full-size batches of the bench workloads over several seeds
-- winner, inlier count, E and P must be identical (exact count-bound
pruning).  Prints one line per (config, seed) and the total.
Usage: python scripts/prune_validate.py [seeds=6]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, ransac, synth
from sfm_amd.pipeline import TwoViewHotPath

SEEDS = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda", 0)
bad = 0
for name, hw, k, iters in (("c2", synth.KITTI_HW, None, 8), ("c4", synth.INDOOR_HW, synth.INDOOR_K, 4),
                           ("c5", synth.KITTI_HW, None, 16)):
    fhw = synth.feature_hw(hw)
    hp = TwoViewHotPath(8, hw, fhw, 32, 8, iters, 1e-4, 1.0, True, 0.6, device=dev)
    for s in range(SEEDS):
        flow, K, _, _ = synth.kitti_pair_batch(8, seed=7000 + 31 * s, hw=hw, device=dev, k=k,
                                               outlier_frac=(0.15, 0.3, 0.5)[s % 3])
        Kinv = hp.k_inverse(K)
        out = {}
        for pm in (880, 0):
            _lib.tune("score_mf_prune", pm)
            E, P, inl, win = hp.pose(flow, K, Kinv)
            torch.cuda.synchronize()
            out[pm] = (E.clone(), P.clone(), inl.clone(), win.clone(), _lib.last_scorer(),
                       int(ransac.skipped_evaluations(hp.ws, 8, iters)))
        _lib.tune("score_mf_prune", 880)
        a, b = out[880], out[0]
        same = all(torch.equal(x, y) for x, y in zip(a[:4], b[:4]))
        bad += not same
        print(f"{name} seed {s}: identical={same} scorers {a[4]} / {b[4]} skipped {a[5]} inliers {a[2].tolist()}",
              flush=True)
print("mismatches", bad)
sys.exit(1 if bad else 0)
