"""A/B of tuning keys on the bench RANSAC (KITTI B=8, H=4096): per-launch
score-kernel time (HIP events), 5 launches per variant and round, three
interleaved rounds; every variant's outputs must equal the first's.
Usage: mf_ab.py "k=v,k=v" "k=v" ...  (each variant sets every key it names)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath

dev = torch.device("cuda", 0)
flow, K, _, _ = synth.kitti_pair_batch(8, seed=1000, device=dev)
hp = TwoViewHotPath(8, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
names = sys.argv[1:] or [""]
variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in names]
res = {i: [] for i in range(len(variants))}
base = None
for rnd in range(3):
    for i, v in enumerate(variants):
        for k, x in v.items():
            _lib.tune(k, int(x))
        out = [t.clone() for t in hp.pose(flow, K) if torch.is_tensor(t)]
        torch.cuda.synchronize()
        if base is None:
            base = out
        for a, b in zip(base, out):
            assert torch.equal(a, b), f"variant {names[i]} changed the output"
        _lib.profile_reset(); _lib.profile_enable(True)
        for _ in range(5):
            hp.pose(flow, K)
        torch.cuda.synchronize(); _lib.profile_enable(False)
        ms, n = _lib.profile_read("ransac_score")
        res[i].append(ms / max(n, 1))
for i in range(len(variants)):
    r = sorted(res[i])
    print(f"{names[i] or 'default':40s} score median {r[len(r) // 2]:.3f} ms  all {[round(x, 3) for x in res[i]]}",
          flush=True)
