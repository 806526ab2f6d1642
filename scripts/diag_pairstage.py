"""Round-5 diagnostic (GPU box, experiment library built with
-DSFM_SWEEP_PAIRSTAGE, selected with SFM_HIP_LIB): for the wrong words of the
4-byte pair-staged bf16 wide stores, what the wrong value equals -- the same
pixel of another channel row (stale LDS stage), another pixel of the same
row, or nothing."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
from sfm_amd import _lib, synth
from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics
cuda = torch.device("cuda", 0)
B, C, L = 4, 32, 128
h, w = synth.feature_hw()
ref, tgt = synth.features(B, C, h, w, seed=C + L)
K = synth.intrinsics(B)
pose = synth.relative_pose(B, torch.Generator().manual_seed(L))
pose[:, :, 3] *= 0.6 / pose[:, :, 3].norm(dim=1, keepdim=True)
K4, Ki4 = quarter_intrinsics(K, torch.inverse(K))
args = (ref.to(cuda), tgt.to(cuda), pose.to(cuda), K4.to(cuda), Ki4.to(cuda), L, 1.0)
_lib.tune("sweep_store_px", 0)
want = plane_sweep_cost(*args, dtype=torch.bfloat16).view(torch.int16).cpu()
_lib.tune("sweep_store_px", 2)
got = plane_sweep_cost(*args, dtype=torch.bfloat16).view(torch.int16).cpu()
_lib.tune("sweep_store_px", -1)
slab = L * h * w
W = want.reshape(B, 2 * C, slab)
G = got.reshape(B, 2 * C, slab)
bad = (W != G).nonzero()
print("mismatches", len(bad), "channels", sorted(set(bad[:, 1].tolist()))[:40])
print("slab offset mod 128 histogram:", torch.bincount(bad[:, 2] % 128, minlength=128).nonzero().flatten().tolist())
stats = {"zero": 0, "same_pixel_other_row": 0, "same_row_other_pixel": 0, "none": 0}
rel_rows, rel_px = {}, {}
for b, c, o in bad[:4000].tolist():
    g = int(G[b, c, o])
    if g == 0:
        stats["zero"] += 1
        continue
    rows = (W[b, :, o] == g).nonzero().flatten().tolist()
    if rows:
        stats["same_pixel_other_row"] += 1
        for r in rows:
            rel_rows[r - c] = rel_rows.get(r - c, 0) + 1
        continue
    win0 = o - o % 128
    px = (W[b, c, win0:win0 + 128] == g).nonzero().flatten().tolist()
    if px:
        stats["same_row_other_pixel"] += 1
        for p in px:
            rel_px[p - o % 128] = rel_px.get(p - o % 128, 0) + 1
        continue
    stats["none"] += 1
print(stats)
print("other-row offsets (row - own row):", sorted(rel_rows.items(), key=lambda x: -x[1])[:12])
print("same-row pixel offsets:", sorted(rel_px.items(), key=lambda x: -x[1])[:12])
b, c, o = bad[0].tolist()
win0 = o - o % 128
print("window of the first mismatch: b", b, "ch", c, "slab offset", win0)
for r in range(c - 5, c + 2):
    if 0 <= r < 2 * C:
        print(f"row {r:2d} want", W[b, r, win0 + 28:win0 + 44].tolist())
        print(f"row {r:2d} got ", G[b, r, win0 + 28:win0 + 44].tolist())
