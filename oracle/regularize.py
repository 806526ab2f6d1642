"""ORACLE (test infrastructure only): torch-CPU restatement of PSNet's 3-D cost
regularisation, models/PSNet.py:159-165 over the modules of PSNet.py:79-102
(convbn_3d = Conv3d(3, 1, 1, bias=False) + BatchNorm3d, submodule.py:17-20),
evaluated with BatchNorm in eval mode (running statistics).

* ``regularize_fp32``  — the reference arithmetic: every layer in fp32.
* ``regularize_bf16``  — the same stack with the weights, the input and every
  layer output rounded to bf16, i.e. the storage precision of the HIP path
  (``sfm_conv3_bf16``); fp32 accumulation.  The HIP result differs from this
  only by summation order (and the rare bf16 rounding flip it causes), so
  tests compare against it tightly and against ``regularize_fp32`` with the
  bf16 storage tolerance.
* ``regularize_f16``   — the same with float16 storage (``sfm_conv3_f16``;
  the precision of the reference's Conv3d layers under cfg.MIXED_PREC
  autocast, models/SFMnet.py:164).

Parity unpinned by the reference: it holds no fixtures for this stack; the
oracle is the reference's own module code run in fp32 (the nn.Conv3d /
nn.BatchNorm3d definitions above, copied in structure by
``sfm_amd.regularize.CostRegularization``).
"""
import torch
import torch.nn.functional as F


def _bf16(t):
    return t.to(torch.bfloat16).to(torch.float32)


def _f16(t):
    return t.to(torch.float16).to(torch.float32)


def _conv_bn(x, conv, bn, wrnd=lambda t: t):
    y = F.conv3d(x, wrnd(conv.weight.detach().float()), None, stride=1, padding=1)
    if bn is not None:
        scale = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
        bias = bn.bias.detach().float() - bn.running_mean.detach().float() * scale
        y = y * scale.view(1, -1, 1, 1, 1) + bias.view(1, -1, 1, 1, 1)
    return y


def _run(mod, cost, rnd):
    """PSNet.py:159-165: cost0 = dres0(cost); cost0 = dres_i(cost0) + cost0
    (i = 1..4); classify(cost0)."""
    x = rnd(cost.float())
    plan = mod.layer_plan()
    keep = None
    for li, (conv, bn, relu, resid) in enumerate(plan):
        y = _conv_bn(x, conv, bn, rnd)
        if relu:
            y = torch.relu(y)
        if resid:
            y = y + keep
        last = li == len(plan) - 1
        y = y if last else rnd(y)
        if li == 1 or resid:
            keep = y
        x = y
    return x


def regularize_fp32(mod, cost):
    """The reference's own forward of the modules (PSNet.py:160-165), in eval mode."""
    was = mod.training
    mod.eval()
    try:
        with torch.no_grad():
            cost0 = mod.dres0(cost.float())
            cost0 = mod.dres1(cost0) + cost0
            cost0 = mod.dres2(cost0) + cost0
            cost0 = mod.dres3(cost0) + cost0
            cost0 = mod.dres4(cost0) + cost0
            return mod.classify(cost0)
    finally:
        mod.train(was)


def regularize_fp32_plan(mod, cost):
    """``regularize_fp32`` through the folded layer plan (checks the plan)."""
    with torch.no_grad():
        return _run(mod, cost, lambda t: t)


def regularize_bf16(mod, cost):
    with torch.no_grad():
        return _run(mod, cost, _bf16)


def regularize_f16(mod, cost):
    with torch.no_grad():
        return _run(mod, cost, _f16)
