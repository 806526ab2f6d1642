"""Per-launch time of one RANSAC phase (HIP events; --phase NAME, default
ransac_solve = k_solve_front + k_roots + k_solve_back; ransac_score = the
scoring kernels) of the loaded library (SFM_HIP_LIB selects an experiment
build) on the bench RANSAC, dense or --sparse; outputs are checked against a
reference file written by the first run (--ref PATH).  Usage:
  solve_time.py [--sparse] [--ref PATH] [--phase NAME] [key=value ...]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
args = [a for a in sys.argv[1:] if not a.startswith("--")]
ref = sys.argv[sys.argv.index("--ref") + 1] if "--ref" in sys.argv else None
phase = sys.argv[sys.argv.index("--phase") + 1] if "--phase" in sys.argv else "ransac_solve"
args = [a for a in args if a not in (ref, phase)]
for kv in args:
    k, v = kv.split("=")
    _lib.tune(k, int(v))
flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
kp = (synth.keypoints(B, 2048, (376, 1242), seed=0, device=dev), [2048] * B) if "--sparse" in sys.argv else None
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev, keypoints=kp)
out = [t.clone().cpu() for t in hp.pose(flow, K) if torch.is_tensor(t)]
if ref:
    if os.path.exists(ref):
        for a, b in zip(torch.load(ref, weights_only=True), out):
            assert torch.equal(a, b), "outputs differ from the reference run"
    else:
        torch.save(out, ref)
res = []
for _ in range(5):
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(3):
        hp.pose(flow, K)
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read(phase)
    res.append(ms / max(n, 1))
res.sort()
print(f"{os.environ.get('SFM_HIP_LIB', 'default')} {' '.join(args)} {'sparse' if kp else 'dense'}: "
      f"{phase} median {res[2]:.4f} ms  min {res[0]:.4f}")
