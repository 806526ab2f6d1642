"""Sweep time vs pose source (RANSAC pose rescaled as in the bench, or the
synthetic GT pose), per-row vs aligned-slab kernel."""
import os, sys
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
print("RANSAC P[0]:", P[0].cpu().numpy().round(4).tolist())
print("GT pose[0]:", pose_gt[0].cpu().numpy().round(4).tolist())


def timed(fn, reps=5):
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read("plane_sweep")
    return ms / max(n, 1)


for name, pz in (("ransac", P.clone()), ("gt", pose_gt.double().clone()), ("gt_x0.6", pose_gt.double().clone())):
    if name == "gt_x0.6":
        pz[:, :, 3] = pz[:, :, 3] / pz[:, :, 3].norm(dim=1, keepdim=True)
    for flat in (0, 1):
        _lib.tune("sweep_flat", flat)
        t = [timed(lambda: hp.sweep(ref, tgt, pz.clone(), K)) for _ in range(3)]
        c = hp.cost
        inimg = float((c[:, 32:] != 0).float().mean())
        print(f"pose={name:8s} flat={flat}: {sorted(t)[1]:.4f} ms  nonzero warped frac {inimg:.3f}", flush=True)
_lib.tune("sweep_flat", 1)

# inside the bench loop: RANSAC then sweep, back to back
for flat in (0, 1, 0, 1):
    _lib.tune("sweep_flat", flat)
    for _ in range(2):
        hp.step(flow, K, ref, tgt)
    torch.cuda.synchronize()
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(5):
        hp.step(flow, K, ref, tgt)
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read("plane_sweep")
    ms2, n2 = _lib.profile_read("ransac_score")
    print(f"bench loop flat={flat}: sweep {ms / n:.4f} ms, score {ms2 / n2:.3f} ms", flush=True)
    # the same sweeps back to back right after
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(5):
        hp.sweep(ref, tgt, P.clone(), K)
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read("plane_sweep")
    print(f"   back-to-back flat={flat}: sweep {ms / n:.4f} ms", flush=True)
_lib.tune("sweep_flat", 1)
