"""Run the bench RANSAC (KITTI B=8, H=4096) 3x with tuning given as key=value
arguments (for rocprofv3 PMC passes over one score-kernel variant)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath

for kv in sys.argv[1:]:
    k, v = kv.split("=")
    _lib.tune(k, int(v))
dev = torch.device("cuda", 0)
flow, K, _, _ = synth.kitti_pair_batch(8, seed=1000, device=dev)
hp = TwoViewHotPath(8, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
for _ in range(3):
    hp.pose(flow, K)
torch.cuda.synchronize()
print("ok")
