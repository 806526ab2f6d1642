"""Experiment: where k_roots_split's time goes (library built with
-DSFM_ROOTS_STATS, selected with SFM_HIP_LIB).  Per hypothesis: Sturm
evaluations (all), single-root bisection steps (modrf failed), the cycles at
the end of phase 1; per wave: phase-1 end of its slowest lane vs the kernel's
end (phases 2 + 3).  Usage: roots_split_stats.py [--sparse]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import numpy as np
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
_lib.tune("roots_split", 1)
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=dev), [2048] * B) if "--sparse" in sys.argv else None
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev, keypoints=kp)
hp.pose(flow, K); torch.cuda.synchronize()
lib = _lib.load()
n = 1 << 17
ev = (ctypes.c_uint * n)(); b1 = (ctypes.c_uint * n)(); cy = (ctypes.c_ulonglong * n)()
ph = (ctypes.c_ulonglong * (4 * n))()   # [0]: cycles at the end of phase 2
lib.sfm_experiment_roots_stats(ev, b1, cy, ph, n, 1)
hp.pose(flow, K); torch.cuda.synchronize()
lib.sfm_experiment_roots_stats(ev, b1, cy, ph, n, 0)
ev = np.frombuffer(ev, dtype=np.uint32)[: 1 << 16].reshape(-1, 64)[:, :32].ravel()
b1 = np.frombuffer(b1, dtype=np.uint32)[: 1 << 16].reshape(-1, 64)[:, :32].ravel()
cy = np.frombuffer(cy, dtype=np.uint64).astype(np.float64)
tot = cy[: 1 << 16].reshape(-1, 64)[:, :32]
p1 = cy[1 << 16:].reshape(-1, 64)[:, :32]
p2 = np.frombuffer(ph, dtype=np.uint64).astype(np.float64)[: 1 << 16].reshape(-1, 64)[:, :32]
live = tot.max(1) > 0
tot, p1, p2 = tot[live], p1[live], p2[live]
for name, a in (("sturm evals", ev), ("bis1 evals (p3)", b1), ("p1 cycles/lane", p1.ravel())):
    q = np.percentile(a, [50, 90, 99, 100])
    print(f"{name:15s} mean {a.mean():10.1f}  p50 {q[0]:9.0f}  p90 {q[1]:9.0f}  p99 {q[2]:9.0f}  max {q[3]:9.0f}")
print(f"hypotheses with a single-root bisection: {(b1 > 0).mean():.3f}; waves with one: "
      f"{(b1.reshape(-1, 32).max(1) > 0).mean():.3f}")
w1 = p1.max(1); w2 = p2.max(1); wt = tot.max(1)
print(f"per wave: phase 1 mean {w1.mean():.0f}  phase 2 mean {(w2 - w1).mean():.0f}  phase 3 mean "
      f"{(wt - w2).mean():.0f}  total mean {wt.mean():.0f}  max {wt.max():.0f} cycles")
print(f"phase 1: mean lane {p1.mean():.0f} vs slowest lane {w1.mean():.0f}")
