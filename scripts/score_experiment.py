"""Experiment: score-kernel time with the fp32 pre-decision on/off, and the
undecided statistics (libraries built with -DSFM_SCORE_STATS /
-DSFM_SCORE_NOFALLBACK into scripts/exp/; select with SFM_HIP_LIB)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
flow, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
hp.pose(flow, K); torch.cuda.synchronize()
def timed(reps=3):
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(reps): hp.pose(flow, K)
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read("ransac_score")
    return ms / max(n, 1)
for flag in (0, 1, 0, 1):
    _lib.tune("score_fp32", flag)
    print(os.path.basename(os.environ.get("SFM_HIP_LIB", "default")), "score_fp32", flag, "%.3f ms" % timed())
lib = _lib.load()
if hasattr(lib, "sfm_experiment_score_stats"):
    out = (ctypes.c_ulonglong * 3)()
    lib.sfm_experiment_score_stats(out)
    print("(candidate, point-slot) wave iterations", out[0], "with an undecided lane", out[1],
          "frac %.4f" % (out[1] / max(out[0], 1)), "undecided evaluations", out[2],
          "per evaluation %.6f" % (out[2] / max(out[0] * 64, 1)))
