"""A/B of k_sweep_tile's generic body (sweep_buffer=0) against its
buffer-addressed fast path (sweep_buffer=1, printed as rows=1) and of the
plane-run band sweep (sweep_flat=3, k_sweep_band) against the
narrow-window kernel (sweep_flat=2, k_sweep_tile) at the bench's C2 volume
(B=8, C=32, L=128, 94x311, translation scaled to 0.6 like the bench's
RESCALE_DEPTH pose), fp32 and bf16: bit-equality and per-launch time."""
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
P = pose[:, :3, :4].float().clone()
P[:, :, 3] *= 0.6 / P[:, :, 3].norm(dim=1, keepdim=True)
P = P.contiguous().to(dev)
variants = [(2, 0, 0), (2, 0, 1), (2, -2, 1)] + [(3, r, rows) for r in (int(x) for x in os.environ.get("RUNS", "").split(",") if x)
                                    for rows in (int(x) for x in os.environ.get("ROWS", "16").split(","))]
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
    _lib.tune("sweep_flat", 2); _lib.tune("sweep_buffer", 0); run(); want = out.clone()
    for rnd in range(3):
        for flat, r, rows in variants:
            _lib.tune("sweep_flat", flat)
            _lib.tune("sweep_buffer", rows if flat == 2 else 1)
            if flat == 3:
                _lib.tune("sweep_run", r); _lib.tune("sweep_band_rows", rows)
            else:   # run = -nj (pixels per lane)
                _lib.tune("sweep_nj", -r if r < 0 else 1)
            out.fill_(7.0)
            res.setdefault(f"{str(dt)[6:]} flat={flat} run={r} rows={rows}", []).append(timed("plane_sweep", run))
            if rnd == 0 and not torch.equal(out, want):
                d = (out.float() - want.float()).abs()
                print(f"MISMATCH {dt} flat={flat} run={r} rows={rows}: max|diff| {float(d.max()):.3g} "
                      f"n={int((d > 0).sum())}", flush=True)
    del out, want
_lib.tune("sweep_flat", 2); _lib.tune("sweep_buffer", 1); _lib.tune("sweep_nj", 1)
_lib.tune("sweep_run", 16); _lib.tune("sweep_band_rows", 16)
for k, v in res.items():
    gb = B * 2 * C * L * h * w * (4 if "float32" in k else 2) / 1e9 + B * 2 * C * h * w * 4 / 1e9
    med = sorted(v)[len(v) // 2]
    print(f"{k:36s} median {med:.4f} ms  {gb / (med * 1e-3):7.1f} GB/s  all {[round(x, 4) for x in v]}", flush=True)
