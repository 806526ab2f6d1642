"""Run the KITTI B=8 L=128 sweep 3x with the tuning given as key=value args
(for rocprofv3 PMC passes over one variant); dtype=bf16 selects the bf16 volume."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd import sweep as SW

dtype = torch.float32
for kv in sys.argv[1:]:
    k, v = kv.split("=")
    if k == "dtype":
        dtype = torch.bfloat16 if v == "bf16" else torch.float32
    else:
        _lib.tune(k, int(v))
dev = torch.device("cuda", 0)
B, C, L, h, w = 8, 32, 128, 94, 311
_, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
ref, tgt = synth.features(B, C, h, w, device=dev)
K4, Ki4 = SW.quarter_intrinsics(K, torch.inverse(K))
P = pose[:, :3, :4].float().contiguous().to(dev)
out = torch.empty(B, 2 * C, L, h, w, device=dev, dtype=dtype)
ws = SW.workspace_for(B, C, h, w, dev)
for _ in range(3):
    SW.plane_sweep_cost(ref, tgt, P, K4, Ki4, L, 1.0, dtype=dtype, out=out, workspace=ws)
torch.cuda.synchronize()
print("ok")
