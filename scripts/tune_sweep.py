"""In-process A/B of launch-shape knobs (interleaved rounds, one process)."""
import os, sys, json, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth, ransac
from sfm_amd.pipeline import TwoViewHotPath

dev = torch.device("cuda", 0)
B = 8
flow, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
ref, tgt = synth.features(B, 32, 94, 311, device=dev)
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
hp.step(flow, K, ref, tgt); torch.cuda.synchronize()
E0, P0, inl0, _ = hp.step(flow, K, ref, tgt)
E0 = E0.clone(); inl0 = inl0.clone()

def timed(name, fn, reps=3):
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(reps): fn()
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read(name)
    return ms / max(n, 1)

# warped-only vs full volume, to separate the reference-copy half
from sfm_amd import sweep as SW
K4, Ki4 = SW.quarter_intrinsics(K, torch.inverse(K))
wout = torch.empty(B, 32, 128, 94, 311, device=dev)
res = {}
MODE = os.environ.get("TUNE", "sweep")
c0 = hp.sweep(ref, tgt, P0, K).clone()
for rnd in range(3):
    if MODE in ("all", "solve"):
        for lanes in (8, 12, 16):
            _lib.tune("solve_lanes", lanes)
            res.setdefault(f"solve_lanes={lanes}", []).append(timed("ransac_solve", lambda: hp.pose(flow, K)))
            E, P, inl, _ = hp.pose(flow, K)
            assert torch.equal(E, E0) and torch.equal(inl, inl0), "results changed with solve_lanes"
        _lib.tune("solve_lanes", 16)
    for lp in (0, 1, 2):
        _lib.tune("sweep_lane_pixels", lp)
        for ipb in (1, 2, 4, 8):
            _lib.tune("sweep_items_per_block", ipb)
            res.setdefault(f"sweep_lp={lp}_ipb={ipb}", []).append(timed("plane_sweep", lambda: hp.sweep(ref, tgt, P0, K)))
            assert torch.equal(hp.cost, c0), "results changed with sweep knobs"
        res.setdefault(f"warped_lp={lp}", []).append(timed("plane_sweep_warped", lambda: SW.plane_sweep_cost(None, tgt, P0.float(), K4, Ki4, 128, 1.0, out=wout, warped_only=True, workspace=hp.sweep_ws)))
    _lib.tune("sweep_items_per_block", 4); _lib.tune("sweep_lane_pixels", 0)
    if MODE in ("all", "score"):
        for bpc in (16, 32):
            _lib.tune("score_blocks_per_cu", bpc)
            res.setdefault(f"score_bpc={bpc}", []).append(timed("ransac_score", lambda: hp.pose(flow, K), reps=2))
        _lib.tune("score_blocks_per_cu", 32)
for k, v in res.items():
    print(f"{k:24s} median {sorted(v)[len(v)//2]:.4f} ms  all {[round(x,4) for x in v]}")
res["sweep_tgt_quads"] = [timed("sweep_tgt_quads", lambda: hp.sweep(ref, tgt, P0, K))]
gb = B * 64 * 128 * 94 * 311 * 4 / 1e9
for k in res:
    if k.startswith("sweep_lp"):
        print(f"{k} write rate {gb / (sorted(res[k])[1] * 1e-3):.1f} GB/s")
