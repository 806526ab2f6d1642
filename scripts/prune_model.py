"""Experiment: how much scoring a two-pass exact prune would skip on the bench
RANSAC (KITTI B=8, N=435,032, H=4096).  Pass 1 scores every candidate on the
first f*N points; a candidate whose prefix count + (1-f)*N is below the
largest prefix count of its pair cannot win (nor tie) and skips pass 2.
Prefix and full counts come from one RANSAC call with num_test = f*N,
num_ransac_test = N (cntT / cntR read from the workspace layout of
csrc/ransac5.hip `layout`)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import numpy as np
import torch
from sfm_amd import ransac, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B, iters = 8, 8
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, iters, 1e-4, 1.0, True, 0.6, device=dev)
hp.pose(flow, K)
N = hp.pts.shape[1]
H = 512 * iters
C = H * 10
al = lambda x: (x + 255) & ~255
sizes = [B * H * 4, B * H * 4, B * H * 90 * 8, B * H * 120 * 8, B * H * 12 * 8, 116 * B * H * 8, B * H * 4, 64 * 4,
         B * C * 18 * 8, B * C * 4, B * C * 4]
offs = np.cumsum([0] + [al(s) for s in sizes])
o_tot, o_T, o_R = offs[7], offs[9], offs[10]
for f in (0.3, 0.4, 0.5, 0.6, 0.7, 0.8):
    nt = int(f * N)
    E, P, inl, win = ransac.ransac5_batched(hp.pts, None, nt, N, iters, 1e-4, hp.seed, True, workspace=hp.ws)
    torch.cuda.synchronize()
    ws = hp.ws.cpu().numpy()
    tot = ws[o_tot:o_tot + B * 4].view(np.int32)
    cT = ws[o_T:o_T + B * C * 4].view(np.int32).reshape(B, C)
    cR = ws[o_R:o_R + B * C * 4].view(np.int32).reshape(B, C)
    surv = work = cands = 0
    for b in range(B):
        t, r = cT[b, :tot[b]], cR[b, :tot[b]]
        keep = t + (N - nt) >= t.max()
        assert keep[np.argmax(r)], "the best candidate would be pruned"
        surv += keep.sum(); cands += tot[b]
    print(f"f={f:.1f}: survivors {surv / cands:.3f}  work {f + (1 - f) * surv / cands:.3f} of one pass "
          f"(full-count quartiles {np.percentile(cR[0, :tot[0]] / N, [25, 50, 75, 90, 99]).round(3)})", flush=True)
