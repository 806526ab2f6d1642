"""Diagnostic: the shader clock and cycles per tile of the one-sided scorer pass.

Needs a diagnostic build of libsfm_hip.so (SFM_HIP_LIB) whose
k_score_mf2<Src, false, true> stamps s_memtime / s_memrealtime around its unit
loop per block and counts the runs (32 tiles each) its waves executed, read
through sfm_experiment_clk (the product library has neither).  Runs the c2
RANSAC (8 KITTI pairs, H = 4096) back to back for >= 2 s, then reads the last
launch's stamps: clock = d memtime / d memrealtime x 100 MHz (median over
blocks), and shader cycles per 32 x 32 tile per SIMD = d memtime / (tiles / 4)
(16 waves, 4 SIMDs per block, one block per CU)."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-sfm-revisited_amd")]

from sfm_amd import _lib, ransac, synth  # noqa: E402


def main():
    lib = _lib.load()
    fn = lib.sfm_experiment_clk
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    flow, K, _, _ = synth.kitti_pair_batch(8, seed=1000, device=dev)
    pts = ransac.flow_to_points(flow, torch.inverse(K))
    ws = ransac.workspace_for(8, 8, dev)
    t0 = time.time()
    n = 0
    while time.time() - t0 < 3.0:
        ransac.ransac5_batched(pts, None, None, None, 8, 1e-4, workspace=ws)
        n += 1
    torch.cuda.synchronize()
    buf = np.zeros((4096, 3), dtype=np.uint64)
    assert fn(None, 1) == 0
    ransac.ransac5_batched(pts, None, None, None, 8, 1e-4, workspace=ws)
    torch.cuda.synchronize()
    assert fn(buf.ctypes.data, 0) == 0
    used = buf[:, 1] > 0
    cyc, real, runs = (buf[used, i].astype(np.float64) for i in range(3))
    clk = cyc / real * 100.0                                  # MHz
    tiles_per_simd = runs * 32 / 4
    cpt = cyc / np.maximum(tiles_per_simd, 1)
    print(f"warm-up launches {n}; blocks {int(used.sum())}; scorer {_lib.last_scorer()}")
    print(f"clock MHz: median {np.median(clk):.0f}  min {clk.min():.0f}  max {clk.max():.0f}")
    print(f"block time us: median {np.median(real) / 100:.1f}  max {real.max() / 100:.1f}")
    print(f"tiles per block: median {np.median(runs * 32):.0f}  total {int(runs.sum() * 32)}")
    print(f"shader cycles per tile per SIMD: median {np.median(cpt):.1f}  (all blocks: "
          f"{cyc.sum() / tiles_per_simd.sum():.1f})")


if __name__ == "__main__":
    main()
