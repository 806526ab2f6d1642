"""Per-layer timing of sfm_conv3_bf16 at C2 geometry (1 pair, L=128, 94x311):
cin 64 (k_conv3) and cin 32 (k_conv3r) with / without ReLU, residual, cout 1."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deep-sfm-revisited_amd"))
from sfm_amd import _lib  # noqa: E402
from sfm_amd.regularize import conv3_bf16  # noqa: E402

dev = torch.device("cuda", 0)
L, h, w = 128, 94, 311
res = {}
for name, cin, relu, resid, cout in (("cin64_relu", 64, True, False, 32), ("cin32_relu", 32, True, False, 32),
                                     ("cin32_resid", 32, False, True, 32), ("cin32_plain", 32, False, False, 32),
                                     ("cin32_cout1", 32, False, False, 1)):
    x = torch.randn(1, L, h, w, cin, device=dev).to(torch.bfloat16)
    wp = (torch.randn(27, 32, cin, device=dev) * 0.05).to(torch.bfloat16)
    sc, bi = torch.ones(32, device=dev), torch.zeros(32, device=dev)
    r = torch.randn(1, L, h, w, 32, device=dev).to(torch.bfloat16) if resid else None
    conv3_bf16(x, wp, sc, bi, r, relu, cout)
    torch.cuda.synchronize()
    _lib.profile_reset()
    _lib.profile_enable(True)
    for _ in range(5):
        conv3_bf16(x, wp, sc, bi, r, relu, cout)
    torch.cuda.synchronize()
    _lib.profile_enable(False)
    ms, n = _lib.profile_read("conv3")
    flop = 2 * L * h * w * 27 * cin * 32
    res[name] = {"ms": round(ms / n, 4), "tflops_mfma_issue": round(flop / (ms / n * 1e-3) / 1e12, 1)}
print(json.dumps(res))
