"""A/B of the narrow-window sweep (sweep_flat=2, k_sweep_tile) against the
aligned-slab kernel (sweep_flat=1, k_sweep_flat) at the C2 shape, fp32 and
bf16: bit-equality of the volumes and per-launch time (HIP events)."""
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
variants = [(1, 8, 1), (1, 4, 1), (2, 8, 1), (2, 8, 2), (2, 8, 4), (2, 4, 1), (2, 4, 2), (2, 4, 4)]


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
    _lib.tune("sweep_flat", 1); _lib.tune("sweep_group", 8); run(); want = out.clone()
    for rnd in range(3):
        for flat, grp, nj in variants:
            if dt == torch.bfloat16 and flat == 2 and nj == 1:
                continue
            _lib.tune("sweep_flat", flat); _lib.tune("sweep_group", grp); _lib.tune("sweep_nj", nj)
            out.fill_(7.0)
            res.setdefault(f"{str(dt)[6:]} flat={flat} group={grp} nj={nj}", []).append(timed("plane_sweep", run))
            if rnd == 0 and not torch.equal(out, want):
                d = (out.float() - want.float()).abs()
                print(f"MISMATCH {dt} flat={flat} group={grp} nj={nj}: max|diff| {float(d.max()):.3g} "
                      f"n={int((d > 0).sum())}", flush=True)
    del out, want
_lib.tune("sweep_flat", 1); _lib.tune("sweep_group", 8); _lib.tune("sweep_nj", 1)
for k, v in res.items():
    gb = B * 2 * C * L * h * w * (4 if "float32" in k else 2) / 1e9 + B * 2 * C * h * w * 4 / 1e9
    med = sorted(v)[len(v) // 2]
    print(f"{k:36s} median {med:.4f} ms  {gb / (med * 1e-3):7.1f} GB/s  all {[round(x, 4) for x in v]}", flush=True)
