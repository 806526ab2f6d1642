"""Experiment: cross-block balance of k_score_mf2 (library built with
-DSFM_MF2_BLOCKT, selected with SFM_HIP_LIB): each persistent block's start
and end on the 100 MHz clock.  Prints the kernel span, the spread of block
end times and the idle share (blocks finished while others still ran)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import numpy as np
import torch
from sfm_amd import _lib, synth
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
flow, K, _, _ = synth.kitti_pair_batch(8, seed=1000, device=dev)
hp = TwoViewHotPath(8, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
lib = _lib.load()
for rep in range(4):
    hp.pose(flow, K); torch.cuda.synchronize()
    n = 4096
    out = (ctypes.c_ulonglong * (3 * n))()
    assert lib.sfm_experiment_mf2_blockt(out, n) == 0
    a = np.frombuffer(out, dtype=np.uint64).reshape(n, 3).astype(np.float64)
    a = a[a[:, 1] > 0]
    t0 = a[:, 0].min()
    st = (a[:, 0] - t0) / 100.0   # microseconds (100 MHz)
    en = (a[:, 1] - t0) / 100.0
    span = en.max()
    idle = (span - en).sum() / (len(en) * span)
    q = np.percentile(en, [0, 10, 50, 90, 100])
    print(f"rep {rep}: {len(a)} blocks, span {span:.1f} us; start max {st.max():.1f} us; end p0/10/50/90/100 "
          f"{q[0]:.0f}/{q[1]:.0f}/{q[2]:.0f}/{q[3]:.0f}/{q[4]:.0f} us; idle share {idle * 100:.1f} %; "
          f"units min/max {a[:, 2].min():.0f}/{a[:, 2].max():.0f}")
    xcd = np.arange(len(a)) % 8
    print("   per-XCD mean end (us):", " ".join(f"{en[xcd == x].mean():.0f}" for x in range(8)))
