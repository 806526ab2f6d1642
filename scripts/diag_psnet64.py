"""Diagnostic (GPU box): where the fp32 PSNet path departs from the float64
reference on tests/golden/psnet64.npz -- each stage on the GPU against the
torch-CPU oracle of the same stage fed the same input."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deep-sfm-revisited_amd")]
from oracle import regularize as OR  # noqa: E402
from oracle import sweep as S  # noqa: E402
from sfm_amd.depth import depth_head  # noqa: E402
from sfm_amd.regularize import CostRegularization  # noqa: E402
from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics  # noqa: E402

dev = torch.device("cuda", 0)
g = np.load(os.path.join(ROOT, "tests", "golden", "psnet64.npz"))
inp = {k.split("/", 1)[1]: g[k] for k in g.files if k.startswith("input/")}
st = {k.split("/", 1)[1]: torch.from_numpy(g[k]) for k in g.files if k.startswith("state/")}
ref = torch.from_numpy(inp["ref_fea"])
tgt = torch.from_numpy(inp["tgt_fea"])
K = torch.from_numpy(inp["K"])
Ki = torch.from_numpy(inp["Kinv"])
P = torch.from_numpy(inp["pose_rescaled"])[:, 0]
L = int(inp["nlabel"])
hw = tuple(int(x) for x in inp["image_hw"])
m = CostRegularization(64)
m.load_state_dict(st)
m.eval()


def report(name, got, want):
    d = (got.double() - want.double()).abs()
    i = int(d.argmax())
    idx = np.unravel_index(i, tuple(d.shape))
    print(f"{name:34s} max abs {float(d.max()):.3e} at {idx} got {float(got.flatten()[i]):.7g} "
          f"want {float(want.flatten()[i]):.7g}; entries > 1e-3 x scale: "
          f"{int((d > 1e-3 * float(want.abs().max())).sum())}", flush=True)


cost_cpu = S.plane_sweep_cost(ref, tgt, P, K, Ki, L, 1.0)
K4, Ki4 = quarter_intrinsics(K.to(dev), Ki.to(dev))
cost_gpu = plane_sweep_cost(ref.to(dev), tgt.to(dev), P.to(dev), K4, Ki4, L, 1.0).cpu()
report("sweep (GPU vs oracle)", cost_gpu, cost_cpu)
cls_cpu = OR.regularize_fp32(m, cost_cpu)
cls_gpu = m.to(dev)(cost_cpu.to(dev), precision="fp32").cpu()
report("regularize fp32 (same cost)", cls_gpu, cls_cpu)
dep_cpu = S.depth_head(cls_cpu, L, 1.0, out_hw=hw)
dep_gpu = depth_head(cls_cpu.to(dev), L, 1.0, out_hw=hw).cpu()
report("depth head (same logits)", dep_gpu, dep_cpu)
want = torch.from_numpy(g["out64/depth"])
for nm, d in (("oracle chain", dep_cpu), ("GPU head on GPU logits", depth_head(cls_gpu.to(dev), L, 1.0, out_hw=hw).cpu())):
    r = ((d.double() - want.double()).abs() / want.double().abs()).flatten()
    print(f"{nm:34s} vs float64 depth: median {float(r.median()):.3e} max {float(r.max()):.3e} "
          f"at {np.unravel_index(int(r.argmax()), tuple(d.shape))}", flush=True)
