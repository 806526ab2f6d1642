"""Experiment: where k_solve_front's time goes (library built with
-DSFM_FRONT_STATS by scripts/build_exp.sh "FRONTSTATS=-DSFM_FRONT_STATS",
selected with SFM_HIP_LIB).  Per wave: s_memtime stamps at the end of each
phase relative to the wave's start; prints the mean phase durations and the
wave totals.  Usage: front_stats.py [--sparse] [lanes]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import numpy as np
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
lanes = [int(a) for a in sys.argv[1:] if a.isdigit()] or [16]
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=dev), [2048] * B) if "--sparse" in sys.argv else None
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev, keypoints=kp)
lib = _lib.load()
n = 1 << 15
names = ["sample+load", "basis", "equations", "reduce", "determinant", "stores"]
for ln in lanes:
    _lib.tune("solve_lanes", ln)
    hp.pose(flow, K); torch.cuda.synchronize()
    hp.pose(flow, K); torch.cuda.synchronize()
    cy = (ctypes.c_ulonglong * (6 * n))()
    assert lib.sfm_experiment_front_stats(cy, n) == 0
    nw = B * ((4096 + ln - 1) // ln)
    a = np.frombuffer(cy, dtype=np.uint64).astype(np.float64).reshape(6, n)[:, :nw]
    d = np.diff(np.vstack([np.zeros(nw), a]), axis=0)
    print(f"lanes {ln}: {nw} waves, wave total mean {a[5].mean():.0f} p90 {np.percentile(a[5], 90):.0f} "
          f"max {a[5].max():.0f} cycles (s_memtime)")
    for i, nm in enumerate(names):
        print(f"  {nm:12s} mean {d[i].mean():9.0f}  {d[i].mean() / a[5].mean() * 100:5.1f} %")
