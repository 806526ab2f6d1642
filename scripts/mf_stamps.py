"""Experiment: per-phase cycle split of k_score_mf / k_score_mf2 (library
built with -DSFM_MF_STAMPS into scripts/exp/, selected with SFM_HIP_LIB;
argument: the score_mf tuning value, default 2).  For k_score_mf2 an "item"
is one (span, candidate tile) run of a wave; "setup+staging" is the span
staging, "block barrier" the span barriers, "prefetch issue" the A rows."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
flow, K, _, _ = synth.kitti_pair_batch(8, seed=1000, device=dev)
hp = TwoViewHotPath(8, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
lib = _lib.load()
_lib.tune("score_mf", int(sys.argv[1]) if len(sys.argv) > 1 else 2)
hp.pose(flow, K); torch.cuda.synchronize()
out = (ctypes.c_ulonglong * 8)()
lib.sfm_experiment_mf_stamps(out, 1)
_lib.profile_reset(); _lib.profile_enable(True)
hp.pose(flow, K); torch.cuda.synchronize(); _lib.profile_enable(False)
ms, n = _lib.profile_read("ransac_score")
lib.sfm_experiment_mf_stamps(out, 0)
names = ["setup+staging", "tile loop", "queue build", "float64 drain", "reduce+atomics", "block barrier", "prefetch issue"]
tot = sum(out[:len(names)])
print("score %.3f ms, items %d" % (ms, out[7]))
for i, nm in enumerate(names):
    print("%-24s %6.1f %%  %.0f cycles/item/wave" % (nm, 100.0 * out[i] / tot, out[i] / max(out[7], 1)))
