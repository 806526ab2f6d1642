"""Store-policy A/B of the cost-volume sweep over feature-map shapes.  For
each (B, h, w, L, dtype) the sweep runs with every store policy of the list
below, interleaved, after a scorer-sized cache-thrash (a 512 MB copy) so the
caches start cold as inside the bench step; prints the median launch time
and the fraction of 8 TB/s.  Round 5: plain / non-temporal 4-byte lane
stores (the question then: by size or by shape?), then the 16-byte stores
with write-through (sc1) policies.
Usage: sweep_shapes_ab.py [rounds=3]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd import sweep as SW

ROUNDS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
dev = torch.device("cuda", 0)
SHAPES = [(8, 94, 311, 128, "fp32"), (8, 120, 160, 64, "fp32"), (8, 120, 161, 64, "fp32"), (8, 120, 160, 128, "fp32"),
          (8, 94, 312, 128, "fp32"), (8, 96, 320, 128, "fp32"), (8, 94, 311, 64, "fp32"), (8, 128, 128, 64, "fp32"),
          (8, 100, 300, 64, "fp32"), (4, 94, 311, 128, "bf16"), (8, 120, 160, 64, "bf16")]
POLS_F32 = (("plain", {"sweep_store_nt": 0, "sweep_store_px": 0, "sweep_store_wt": 0}),
            ("nt", {"sweep_store_nt": 1, "sweep_store_px": 0, "sweep_store_wt": 0}),
            ("w16", {"sweep_store_nt": 0, "sweep_store_px": 1, "sweep_store_wt": 0}),
            ("w16sc1", {"sweep_store_px": 1, "sweep_store_wt": 1}),
            ("w16ntsc1", {"sweep_store_px": 1, "sweep_store_wt": 3}))
POLS_BF16 = (("w16nt", {"sweep_store_nt": 1, "sweep_store_px": 2, "sweep_store_wt": 0}),
             ("w16ntsc1", {"sweep_store_px": 2, "sweep_store_wt": 3}),
             ("w16sc1", {"sweep_store_px": 2, "sweep_store_wt": 1}))
base = _lib.tune_snapshot()
junk = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
junk2 = torch.empty_like(junk)
C = 32
for B, h, w, L, dt in SHAPES:
    dtype = torch.float32 if dt == "fp32" else torch.bfloat16
    _, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
    ref, tgt = synth.features(B, C, h, w, device=dev)
    K4, Ki4 = SW.quarter_intrinsics(K, torch.inverse(K))
    P = pose[:, :3, :4].float().contiguous().to(dev)
    out = torch.empty(B, 2 * C, L, h, w, device=dev, dtype=dtype)
    ws = SW.workspace_for(B, C, h, w, dev)
    nbytes = out.numel() * out.element_size() + ref.numel() * 4 + tgt.numel() * 4
    pols = (POLS_F32 if dt == "fp32" else POLS_BF16)
    res = {name: [] for name, _ in pols}
    for rnd in range(ROUNDS):
        for name, tune in (pols if rnd % 2 == 0 else pols[::-1]):
            for k, v in tune.items():
                _lib.tune(k, v)
            t = 0.0
            for _ in range(6):
                junk2.copy_(junk)
                _lib.profile_reset(); _lib.profile_enable(True)
                SW.plane_sweep_cost(ref, tgt, P, K4, Ki4, L, 1.0, dtype=dtype, out=out, workspace=ws)
                torch.cuda.synchronize(); _lib.profile_enable(False)
                ms, n = _lib.profile_read("plane_sweep")
                t += ms / max(n, 1)
            res[name].append(t / 6)
            _lib.tune_restore(base)
    line = f"B={B} {h}x{w} L={L:3d} {dt} {nbytes / 1e9:5.2f} GB"
    for name, _ in pols:
        m = sorted(res[name])[len(res[name]) // 2]
        line += f" | {name} {m:.4f} {nbytes / (m * 1e-3) / 8e12:.3f}"
    print(line, flush=True)
    del out, ws
