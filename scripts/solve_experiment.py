"""Experiment: per-phase cycle breakdown of k_solve (library built with
-DSFM_SOLVE_STATS by scripts/build_exp.sh; select with SFM_HIP_LIB)."""
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
lib = _lib.load()
out = (ctypes.c_ulonglong * 8)()
lib.sfm_experiment_solve_stats(out)
names = ["sample+load", "basis", "equations", "reduce", "determinant", "roots", "E+cheirality"]
tot = sum(out[i] for i in range(7))
for i, nme in enumerate(names):
    print(f"{nme:14s} {out[i] / tot * 100:6.2f} %   {out[i] / (B * 4096):10.0f} cycles/hyp")
