"""Diagnostic (GPU box): where the bf16 wide-store sweep (sweep_store_px)
departs from the pair stores -- mismatch positions and what the wrong values
equal elsewhere in the reference volume."""
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
want = plane_sweep_cost(*args, dtype=torch.bfloat16).view(torch.int16)
for px in (2, 4, 8, 2, 8):
    _lib.tune("sweep_store_px", px)
    got = plane_sweep_cost(*args, dtype=torch.bfloat16).view(torch.int16)
    torch.cuda.synchronize()
    d = (got != want).nonzero()
    print(f"px={px}: {len(d)} mismatches", flush=True)
    if len(d) == 0:
        continue
    flat = (got != want).flatten().nonzero().flatten()
    slab = L * h * w
    ch = d[:, 1]
    print("  channels:", torch.bincount(ch, minlength=2 * C).tolist())
    off = flat % slab
    print("  offset mod 8 hist:", torch.bincount(off % 8, minlength=8).tolist(),
          " mod 64:", torch.bincount(off % 64, minlength=64).nonzero().flatten().tolist()[:16])
    wf, gf = want.flatten(), got.flatten()
    for i in flat[:6].tolist():
        g = int(gf[i])
        cands = (wf[max(0, i - 4096):i + 4096] == g).nonzero().flatten()[:6] + max(0, i - 4096) - i
        print(f"   idx {i} (ch {i // slab % (2 * C)}, off {i % slab}) got {g} want {int(wf[i])} "
              f"got-value at relative {cands.tolist()} ; got==0: {g == 0}")
_lib.tune("sweep_store_px", 0)
