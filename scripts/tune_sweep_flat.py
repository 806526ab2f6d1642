"""A/B of the aligned-slab sweep (sweep_flat=1, group 4/8) against the per-row
kernel (sweep_flat=0), fp32 and bf16, with bit-equality of the volumes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd import sweep as SW

dev = torch.device("cuda", 0)
B, C, L, h, w = 8, 32, 128, 94, 311
flow, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
ref, tgt = synth.features(B, C, h, w, device=dev)
K4, Ki4 = SW.quarter_intrinsics(K, torch.inverse(K))
P = pose[:, :3, :4].float().contiguous().to(dev)
res = {}


def timed(name, fn, reps=5):
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read(name)
    return ms / max(n, 1)


for dt in (torch.float32, torch.bfloat16):
    out = torch.empty(B, 2 * C, L, h, w, device=dev, dtype=dt)
    ws = SW.workspace_for(B, C, h, w, dev)
    run = lambda: SW.plane_sweep_cost(ref, tgt, P, K4, Ki4, L, 1.0, dtype=dt, out=out, workspace=ws)
    _lib.tune("sweep_flat", 0); run(); want = out.clone()
    for rnd in range(3):
        for flat, grp in ((0, 4), (1, 4), (1, 8)):
            _lib.tune("sweep_flat", flat); _lib.tune("sweep_group", grp)
            out.zero_()
            res.setdefault(f"{dt} flat={flat} group={grp}", []).append(timed("plane_sweep", run))
            if flat:
                d = (out.float() - want.float()).abs()
                tol = (1e-4 * want.float().abs() + 1e-4) if dt == torch.float32 else (8e-3 * want.float().abs() + 1e-3)
                if rnd == 0:
                    print(f"{dt} flat group={grp} vs per-row kernel: max|diff| {float(d.max()):.3g}, over tol {int((d > tol).sum())}, "
                          f"over 1e-2 {int((d > 1e-2).sum())}", flush=True)
            else:
                assert torch.equal(out, want), f"volume differs: flat={flat} group={grp} {dt}"
    del out, want
_lib.tune("sweep_flat", 1); _lib.tune("sweep_group", 8)
for k, v in res.items():
    gb = B * 2 * C * L * h * w * (4 if "float32" in k else 2) / 1e9
    med = sorted(v)[len(v) // 2]
    print(f"{k:44s} median {med:.4f} ms  {gb / (med * 1e-3):7.1f} GB/s written  all {[round(x, 4) for x in v]}")
