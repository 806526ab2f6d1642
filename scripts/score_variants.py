"""Experiment: time the score kernel of one library build (SFM_HIP_LIB) on the
bench workload and check that its per-hypothesis inlier counts equal the
float64 scorer's (score_fp32=0) exactly.  One JSON line per run; run once per
build (scripts/build_exp.sh NAME=FLAGS)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
import torch
from sfm_amd import _lib, synth, ransac
from sfm_amd.pipeline import TwoViewHotPath
dev = torch.device("cuda", 0)
B = 8
flow, K, pose, _ = synth.kitti_pair_batch(B, seed=1000, device=dev)
hp = TwoViewHotPath(B, (376, 1242), (94, 311), 32, 128, 8, 1e-4, 1.0, True, 0.6, device=dev)
Kinv = torch.inverse(K.float())
ransac.flow_to_points(flow, Kinv, hp.H, hp.W, hp.margin, out=hp.pts)
def run(scores=False):
    return ransac.ransac5_batched(hp.pts, None, None, None, hp.iters, hp.thr, hp.seed, True, return_scores=scores,
                                  workspace=hp.ws)
out = {"lib": os.path.basename(os.environ.get("SFM_HIP_LIB", "default"))}
_lib.tune("score_fp32", 0)
ref = run(True)[-1].clone()
_lib.tune("score_fp32", 1)
got = run(True)[-1]
out["exact"] = bool(torch.equal(ref, got))
run(); torch.cuda.synchronize()
for rep in range(2):
    _lib.profile_reset(); _lib.profile_enable(True)
    for _ in range(5):
        run()
    torch.cuda.synchronize(); _lib.profile_enable(False)
    ms, n = _lib.profile_read("ransac_score")
    out["score_ms_%d" % rep] = round(ms / max(n, 1), 4)
print(json.dumps(out), flush=True)
