"""Experiment: per-hypothesis work of k_roots (library built with
-DSFM_ROOTS_STATS by scripts/build_exp.sh; select with SFM_HIP_LIB): Sturm
sequence evaluations, falsi steps and cycles per thread, and the share of a
wave's time its slowest lane sets."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import numpy as np
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
# --sparse: the SIFT-keypoint branch (bench.py --config sparse, 2,048 keypoints per pair)
kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=dev), [2048] * B) if "--sparse" in sys.argv else None
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev, keypoints=kp)
hp.pose(flow, K); torch.cuda.synchronize()
lib = _lib.load()
n = 1 << 17
ev = (ctypes.c_uint * n)(); fa = (ctypes.c_uint * n)(); cy = (ctypes.c_ulonglong * n)()
ph = (ctypes.c_ulonglong * (4 * n))()
lib.sfm_experiment_roots_stats(ev, fa, cy, ph, n, 1)
hp.pose(flow, K); torch.cuda.synchronize()
lib.sfm_experiment_roots_stats(ev, fa, cy, ph, n, 0)
ph = np.frombuffer(ph, dtype=np.uint64).astype(np.float64).reshape(4, n)
ev = np.frombuffer(ev, dtype=np.uint32).copy(); fa = np.frombuffer(fa, dtype=np.uint32).copy()
cy = np.frombuffer(cy, dtype=np.uint64).astype(np.float64)
ld = cy[1 << 16:].copy(); cy = cy.copy(); cy[1 << 16:] = 0
lanes = _lib.tune_get("roots_lanes")
live = cy > 0
print(f"threads {live.sum()}  (lanes per wave {lanes})")
for name, a in (("sturm evals", ev[live]), ("falsi steps", fa[live]), ("cycles", cy[live])):
    q = np.percentile(a, [50, 90, 99, 99.9, 100])
    print(f"{name:12s} mean {a.mean():10.1f}  p50 {q[0]:9.0f}  p90 {q[1]:9.0f}  p99 {q[2]:9.0f}  "
          f"p99.9 {q[3]:9.0f}  max {q[4]:9.0f}")
w = cy.reshape(-1, 64)[:, :lanes]
wl = w.max(1)
print(f"per wave: mean of slowest lane {wl[wl > 0].mean():.0f} cycles, mean lane {w[w > 0].mean():.0f} "
      f"-> lanes idle {1 - w[w > 0].mean() / wl[wl > 0].mean():.2f} of the wave time")
print(f"correlation cycles ~ evals: {np.corrcoef(cy[live], ev[live])[0, 1]:.3f}, "
      f"cycles per eval (median over threads) {np.median(cy[live] / np.maximum(ev[live] + fa[live], 1)):.0f}")
live = cy > 0
print(f"poly load latency: mean {ld[:live.sum()].mean():.0f} cycles (slots from 2^16, first threads)")
for i, nm in enumerate(["scale (cr_pow)", "sturm build + count", "bracket", "isolate"]):
    a = ph[i][live]
    print(f"{nm:22s} mean {a.mean():10.0f}  p99 {np.percentile(a, 99):10.0f}  max {a.max():10.0f}")
