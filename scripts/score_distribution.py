"""Experiment: distribution of per-hypothesis inlier counts on the bench
workload (fraction of N), and the evaluation fraction an exact
bound-pruning scheme could skip (uniform-arrival model)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import synth, ransac
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
flow, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
Kinv = torch.inverse(K.float())
ransac.flow_to_points(flow, Kinv, hp.H, hp.W, hp.margin, out=hp.pts)
E, P, inl, win, sc = ransac.ransac5_batched(hp.pts, None, None, None, hp.iters, hp.thr, hp.seed, True,
                                           return_scores=True, workspace=hp.ws)
n = hp.n
for b in range(B):
    r = sc[b].double().cpu() / n
    best = r.max().item()
    q = torch.quantile(r, torch.tensor([0.1, 0.5, 0.9, 0.99], dtype=torch.float64)).tolist()
    keep = (1.0 / (1.0 + best - r)).clamp(max=1.0)
    print("pair %d best %.4f q10/50/90/99 %s  prunable-eval fraction %.3f" % (
        b, best, " ".join("%.4f" % v for v in q), 1.0 - keep.mean().item()))
