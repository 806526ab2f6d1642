"""Diagnostic: where the RANSAC workspace differs between solve_coop = 0 and 1
(and between two solve_coop = 0 runs, the determinism check).  Mirrors
ransac5.hip's layout() for B pairs at iters; prints the differing elements per
region and, for the solve state, the fields and a few hypotheses' values.
Usage: solve_coop_diff.py [--sparse]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import numpy as np
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath

B, iters = 8, 8
H = 512 * iters
C = H * 10
dev = torch.device("cuda", 0)
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000 + B, device=dev)
kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=dev), [2048] * B) if "--sparse" in sys.argv else None
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, iters, 1e-4, 1.0, True, 0.6, device=dev, keypoints=kp)


def run(coop):
    _lib.tune("solve_coop", coop)
    hp.ws.zero_()
    hp.pose(flow, K)
    torch.cuda.synchronize()
    return hp.ws.cpu().numpy().copy()


def regions():
    al = lambda x: (x + 255) & ~255
    off, out = 0, []
    for name, nbytes in (("nroots", B * H * 4), ("ncand", B * H * 4), ("hypE", B * H * 10 * 9 * 8),
                         ("hypP", B * H * 10 * 12 * 8), ("hypP0", B * H * 12 * 8), ("sstate", 116 * B * H * 8),
                         ("cand_off", B * H * 4), ("chain_ref", B * H * 4), ("cand_total", 64 * 4),
                         ("candE", B * C * 18 * 8), ("cntT", B * C * 4), ("cntR", B * C * 4), ("cov", B * C * 8),
                         ("best_lb", 64 * 64 * 4), ("skipped", 8), ("score", B * H * 4), ("candF", B * C * 64 * 2)):
        out.append((name, off, nbytes))
        off += al(nbytes)
    return out


a0 = run(0)
a0b = run(0)
a1 = run(1)
for tag, x, y in (("coop0 vs coop0", a0, a0b), ("coop0 vs coop1", a0, a1)):
    print("==", tag, "total differing bytes", int((x != y).sum()))
    for name, off, nb in regions():
        d = int((x[off:off + nb] != y[off:off + nb]).sum())
        if d:
            print(f"  {name:10s} {d} bytes differ")
    off = dict((n, o) for n, o, _ in regions())["sstate"]
    s0 = x[off:off + 116 * B * H * 8].view(np.float64).reshape(116, B * H)
    s1 = y[off:off + 116 * B * H * 8].view(np.float64).reshape(116, B * H)
    bad = np.nonzero((s0.view(np.uint64) != s1.view(np.uint64)))
    if bad[0].size:
        fields = np.unique(bad[0])
        hyps = np.unique(bad[1])
        print("  sstate fields", fields.tolist()[:40], "hypotheses", hyps.size, hyps[:10].tolist())
        for hb in hyps[:3]:
            f = np.nonzero(s0[:, hb].view(np.uint64) != s1[:, hb].view(np.uint64))[0]
            print(f"   hyp {hb}: fields {f.tolist()[:20]}")
            for fi in f[:6]:
                print(f"     f{fi}: {s0[fi, hb]!r} vs {s1[fi, hb]!r}")
