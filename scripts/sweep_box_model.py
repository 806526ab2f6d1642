"""CPU model (round 6): what a per-wave LDS stage of the
target-feature footprint would save the bf16 sweep's tap gathers.  For the
C3 geometry (KITTI 94x311 features, L = 128, synthetic poses with |t| = 0.6
as RESCALE_DEPTH leaves the RANSAC pose) it replays every 128-pixel wave
window of k_sweep_tile (NJ = 2), finds the bounding box of the source pixels
its in-image taps touch (per image row the window covers), and compares the
pixels a stage would load with the 4 gathers per sample made today.
Output: profiles/r06_sweep_box_model.txt."""
import sys, numpy as np, torch
sys.path[:0] = ['deep-sfm-revisited_amd', '.']
from sfm_amd import synth
from oracle import sweep as S
B, L = 4, 128
h, w = synth.feature_hw()
K = synth.intrinsics(B); Ki = torch.inverse(K)
pose = synth.relative_pose(B, torch.Generator().manual_seed(3))
pose[:, :, 3] = 0.6 * pose[:, :, 3] / pose[:, :, 3].norm(dim=1, keepdim=True)
K4, Ki4 = S.quarter_intrinsics(K, Ki)
hw = h * w
stats = []
WW = 128
for b in range(B):
    for l in range(L):
        d = torch.full((1, h, w), L * 1.0 / (l + 1 + 1e-16))
        g = S.warp_grid(d, pose[b:b+1], K4[b:b+1], Ki4[b:b+1], h, w)[0].reshape(-1, 2).numpy()
        inside = (g[:, 0] <= 1) & (g[:, 1] <= 1)
        ix = (g[:, 0] + 1) / 2 * (w - 1); iy = (g[:, 1] + 1) / 2 * (h - 1)
        x0 = np.floor(ix).astype(int); y0 = np.floor(iy).astype(int)
        for s in range(0, hw, WW):
            sl = slice(s, min(s + WW, hw))
            m = inside[sl]
            if not m.any():
                stats.append((0, 0, 0, 0)); continue
            rows = np.arange(sl.start, sl.stop) // w
            tot = 0; nb = 0; ntap = 0
            for r in np.unique(rows):
                mm = m & (rows == r)
                if not mm.any(): continue
                xs = x0[sl][mm]; ys = y0[sl][mm]
                nx = min(xs.max() + 1, w - 1) - xs.min() + 1
                ny = min(ys.max() + 1, h - 1) - ys.min() + 1
                tot += nx * ny; nb += 1
            # unique tap pixels
            xs = x0[sl][m]; ys = y0[sl][m]
            taps = set()
            for a, c in zip(xs, ys):
                for dx in (0, 1):
                    for dy in (0, 1):
                        taps.add((min(c + dy, h - 1), min(a + dx, w - 1)))
            stats.append((int(m.sum()), tot, nb, len(taps)))
st = np.array(stats)
act = st[st[:, 0] > 0]
print("windows", len(st), "with samples", len(act))
print("samples/window mean", act[:, 0].mean())
for q in (50, 75, 90, 95, 99):
    print("box px p%d" % q, np.percentile(act[:, 1], q), " unique taps p%d" % q, np.percentile(act[:, 3], q))
for bud in (256, 384, 512, 640, 768):
    ok = act[:, 1] <= bud
    print("budget", bud, "fraction staged", ok.mean(), "staged px / sample", act[ok, 1].sum() / act[ok, 0].sum(),
          "taps/sample(4)", 4.0)
print("unique taps per sample", act[:, 3].sum() / act[:, 0].sum(), "box/sample all", act[:, 1].sum() / act[:, 0].sum())
