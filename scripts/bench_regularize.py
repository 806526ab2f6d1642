"""Time the PSNet cost-regularisation stack (12 x sfm_conv3_bf16) on the GPU at
BASELINE config C2's geometry: B pairs, 2C=64 channels, L=128, 94x311.

Algorithmic work per 32-cout layer: 2 * B*L*h*w * 27 * Cin * 32 FLOP (the
final 32->1 conv counts its one real output channel).  Peak: 2.5 PFLOP/s dense
bf16 (MI355X_MICROARCH.md).  Prints one JSON line."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))

from sfm_amd import _lib  # noqa: E402
from sfm_amd.regularize import CostRegularization  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--nlabel", type=int, default=128)
ap.add_argument("--hw", type=int, nargs=2, default=[94, 311])
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--precision", choices=["bf16", "fp32"], default="bf16")
a = ap.parse_args()

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = CostRegularization(64).to(dev).eval()
B, L, (h, w) = a.batch, a.nlabel, a.hw
cost = torch.randn(B, 64, L, h, w, device=dev)
m(cost, precision=a.precision)
torch.cuda.synchronize()
_lib.profile_enable(True)
_lib.profile_reset()
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
t0.record()
for _ in range(a.steps):
    m(cost, precision=a.precision)
t1.record()
torch.cuda.synchronize()
ms_total = t0.elapsed_time(t1) / a.steps
conv_ms, conv_n = _lib.profile_read("conv3" if a.precision == "bf16" else "conv3_f32")
cl_ms, cl_n = _lib.profile_read("to_channels_last")
vox = B * L * h * w
flop = 2 * vox * 27 * (64 * 32 + 10 * 32 * 32 + 32 * 1)
per_step_conv = conv_ms / a.steps
peak = 2.5e15 if a.precision == "bf16" else 157.3e12
print(json.dumps({"what": f"psnet cost regularisation (12 conv3d 3x3x3, {a.precision} MFMA)", "B": B, "L": L, "h": h, "w": w,
                  "ms_per_stack": round(ms_total, 4), "conv_ms": round(per_step_conv, 4),
                  "to_channels_last_ms": round(cl_ms / a.steps, 4),
                  "tflops": round(flop / (per_step_conv * 1e-3) / 1e12, 1), "peak_tflops": peak / 1e12,
                  "frac": round(flop / (per_step_conv * 1e-3) / peak, 4), "gflop_per_stack": round(flop / 1e9, 1)}))
