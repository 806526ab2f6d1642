#!/usr/bin/env python3
"""A/B of the HIP-event profiler's cost inside the timed region: the bench step
(TwoViewHotPath.step) timed with libsfm_hip's per-launch events on and off,
alternating, same process.  Usage: python scripts/event_ab.py [c2|sparse|c3] [steps] [rounds]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from sfm_amd import _lib, synth  # noqa: E402
from sfm_amd.pipeline import TwoViewHotPath  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "sparse"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    args = bench.parse(["--config", cfg])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = args.batch
    hw = synth.KITTI_HW if args.hw_name == "kitti" else synth.INDOOR_HW
    kcal = None if args.hw_name == "kitti" else synth.INDOOR_K
    fhw = synth.feature_hw(hw)
    cost_dtype = torch.float32 if args.cost_dtype == "fp32" else torch.bfloat16
    flow, K, _, _ = synth.kitti_pair_batch(B, seed=1000, hw=hw, device=dev, k=kcal)
    ref_fea, tgt_fea = synth.features(B, 32, fhw[0], fhw[1], seed=0, device=dev)
    kp = synth.keypoints(B, args.keypoints, hw, seed=0, device=dev) if args.keypoints else None
    hp = TwoViewHotPath(B, hw, fhw, 32, args.nlabel, args.iters, args.threshold, 1.0, rescale_depth=True,
                        norm_target=0.6, cost_dtype=cost_dtype, device=dev,
                        keypoints=None if kp is None else (kp, [args.keypoints] * B))
    for _ in range(3):
        hp.step(flow, K, ref_fea, tgt_fea)
    torch.cuda.synchronize(dev)
    for r in range(rounds):
        for prof in (True, False):
            _lib.profile_reset()
            _lib.profile_enable(prof)
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                hp.step(flow, K, ref_fea, tgt_fea)
            torch.cuda.synchronize(dev)
            ms = (time.perf_counter() - t0) * 1e3 / steps
            _lib.profile_enable(False)
            ksum = 0.0
            if prof:
                for name in ("flow_to_points", "keypoints_to_points", "ransac_solve", "ransac_chain",
                             "ransac_score", "ransac_select", "plane_sweep"):
                    t, n = _lib.profile_read(name)
                    if n:
                        ksum += t / n
            print(f"{cfg} round {r} events={'on ' if prof else 'off'} {ms:.4f} ms/step  {B / ms * 1e3:9.1f} pairs/s"
                  + (f"  (profiled regions {ksum:.4f} ms)" if prof else ""), flush=True)


if __name__ == "__main__":
    main()
