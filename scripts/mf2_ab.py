"""A/B of the RANSAC score kernels on the bench workload (KITTI B=8,
N=435,032, H=4096): per-launch score time from libsfm_hip's HIP events,
5 launches per variant and round, three interleaved rounds; every variant's
outputs (E, P, inliers, winner and the per-hypothesis score vector) must equal
the first variant's bit for bit.  With a library built with -DSFM_MF_STATS
(scripts/build_exp.sh) it also prints k_score_mf2's undecided fraction.
Usage: mf2_ab.py "score_mf=1" "score_mf=2" ...   (SFM_HIP_LIB selects the library;
AB_REF=file compares the outputs across libraries)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch  # noqa: E402
from sfm_amd import _lib, ransac, synth  # noqa: E402

dev = torch.device("cuda", 0)
B = int(os.environ.get("AB_BATCH", "8"))
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
Kinv = torch.linalg.inv_ex(K.float())[0]
pts = ransac.flow_to_points(flow, Kinv)
ws = ransac.workspace_for(B, 8, dev)
names = sys.argv[1:] or [""]
variants = [dict(kv.split("=") for kv in v.split(",") if kv) for v in names]
lib = _lib.load()
stats = getattr(lib, "sfm_experiment_mf_stats", None)
res = {i: [] for i in range(len(variants))}
base = None
for rnd in range(3):
    for i, v in enumerate(variants):
        for k, x in v.items():
            _lib.tune(k, int(x))
        out = ransac.ransac5_batched(pts, None, None, None, 8, 1e-4, workspace=ws, return_scores=True)
        torch.cuda.synchronize()
        out = [t.clone() for t in out]
        if base is None:
            base = out
        if os.environ.get("AB_NOCHECK") != "1":         # timing-only experiment builds: nondeterministic counts
            for a, b in zip(base, out):
                assert torch.equal(a, b), f"variant {names[i]} changed the output"
        if stats is not None:
            stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
            stats(None, 1)
        _lib.profile_reset()
        _lib.profile_enable(True)
        for _ in range(5):
            ransac.ransac5_batched(pts, None, None, None, 8, 1e-4, workspace=ws)
        torch.cuda.synchronize()
        _lib.profile_enable(False)
        ms, n = _lib.profile_read("ransac_score")
        res[i].append(ms / max(n, 1))
        if stats is not None and rnd == 0:
            o = (ctypes.c_ulonglong * 2)()
            stats(o, 0)
            if o[1]:
                print(f"{names[i]:30s} undecided {o[0]} / {o[1]} = {100.0 * o[0] / o[1]:.4f} %", flush=True)
for i in range(len(variants)):
    r = sorted(res[i])
    print(f"{names[i] or 'default':30s} score median {r[len(r) // 2]:.3f} ms  all {[round(x, 3) for x in res[i]]}",
          flush=True)
print("inliers", base[2].tolist())
# across libraries: AB_REF=path saves the first library's outputs there, and
# every later process compares its own with them bit for bit
ref = os.environ.get("AB_REF")
if ref:
    if not os.path.exists(ref):
        torch.save([t.cpu() for t in base], ref)
    else:
        want = torch.load(ref, weights_only=True)
        for a, b in zip(want, base):
            assert torch.equal(a, b.cpu()), "this library changed the output"
        print("outputs equal the reference library's", flush=True)
