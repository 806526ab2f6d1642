"""PSNet 3-D cost regularisation on the gfx950 matrix cores.

Mirrors the cost-filtering stack of models/PSNet.py:79-102 (module layout,
so a PSNet state_dict's ``dres*`` / ``classify`` entries load unchanged) and
its application at PSNet.py:159-165:

    cost0 = dres0(cost)
    cost0 = dres1(cost0) + cost0   ... dres4
    cost0 = classify(cost0)                      # [B, 1, L, h, w]

``CostRegularization.forward`` runs the 12 Conv3d layers as
``sfm_conv3_f32x3`` launches (default ``precision="fp32x3"``: the
reference's fp32 activations and weights, each product formed from split-f16
operands on the f16 matrix cores; ``precision="fp32"`` is the same on the
f32 matrix cores, ``sfm_conv3_f32``), with
``precision="fp16"`` as ``sfm_conv3_f16`` launches (float16 channels-last
activations and weights, fp32 accumulation: the precision of the reference's
Conv3d layers under ``cfg.MIXED_PREC`` autocast, SFMnet.py:164) or, with
``precision="bf16"``, as ``sfm_conv3_bf16`` launches (the fastest opt-in,
8-bit mantissa).  BatchNorm3d is folded in eval mode, ReLU
and residual are fused into the epilogue.  There is no PyTorch fallback: without libsfm_hip.so or a GPU
the call raises.
"""
import math

import torch
import torch.nn as nn

from . import _lib
from .depth import depth_head
from .sweep import plane_sweep_cost, quarter_intrinsics


_ACT_DTYPE = {"fp32": torch.float32, "fp32x3": torch.float32, "fp16": torch.float16, "bf16": torch.bfloat16}


def weight_exponent(w):
    """sfm_conv3_f32x3's weight scale: the power of two 2^e with 2^e max|w| in
    [2^13, 2^14) (the lo terms of the split stay in the f16 normal range, the
    hi terms far from its maximum), clamped to the ABI's [-24, 24]."""
    m = float(w.abs().max())
    if not (m > 0.0 and math.isfinite(m)):
        return 0
    return max(-24, min(24, 13 - math.frexp(m)[1] + 1))


def convbn_3d(in_planes, out_planes, kernel_size=3, stride=1, pad=1):
    """models/submodule.py:17-20."""
    return nn.Sequential(nn.Conv3d(in_planes, out_planes, kernel_size=kernel_size, padding=pad, stride=stride,
                                   bias=False),
                         nn.BatchNorm3d(out_planes))


_LP_NAME = {torch.bfloat16: "bf16", torch.float16: "f16"}


def to_channels_last(cost, dtype=torch.bfloat16):
    """[B, C, L, h, w] fp32/bf16 (device) -> [B, L, h, w, C] ``dtype`` (bf16 or
    fp16, round to nearest even)."""
    if not (isinstance(cost, torch.Tensor) and cost.is_cuda) or cost.dtype not in (torch.float32, torch.bfloat16):
        raise RuntimeError("to_channels_last needs a float32 / bfloat16 device tensor")
    if dtype not in _LP_NAME:
        raise RuntimeError("to_channels_last writes bfloat16 or float16")
    cost = cost.contiguous()
    B, C = cost.shape[:2]
    P = cost[0, 0].numel()
    out = torch.empty((B,) + tuple(cost.shape[2:]) + (C,), dtype=dtype, device=cost.device)
    fn = "sfm_to_channels_last_" + _LP_NAME[dtype]
    with torch.cuda.device(cost.device):
        _lib.check(getattr(_lib.load(), fn)(_lib.ptr(cost), 0 if cost.dtype == torch.float32 else 1,
                                            B, C, P, _lib.ptr(out), _lib.stream_ptr(cost.device)), fn)
    return out


def _conv3_lp(x, weights, scale, bias, residual, relu, cout, dtype):
    name = {torch.bfloat16: "bfloat16", torch.float16: "float16"}[dtype]
    for t, n in ((x, "x"), (weights, "weights")):
        if not (t.is_cuda and t.dtype == dtype and t.is_contiguous()):
            raise RuntimeError(f"{n} must be a contiguous {name} device tensor")
    B, L, h, w, cin = x.shape
    if tuple(weights.shape) != (27, 32, cin):
        raise RuntimeError(f"weights must be [27, 32, {cin}]")
    if residual is not None and (residual.dtype != dtype or tuple(residual.shape) != (B, L, h, w, 32)):
        raise RuntimeError(f"residual must be {name} [B, L, h, w, 32]")
    if cout == 32:
        out = torch.empty((B, L, h, w, 32), dtype=dtype, device=x.device)
    else:
        out = torch.empty((B, L, h, w), dtype=torch.float32, device=x.device)
    scale = scale.to(device=x.device, dtype=torch.float32).contiguous()
    bias = bias.to(device=x.device, dtype=torch.float32).contiguous()
    fn = "sfm_conv3_" + _LP_NAME[dtype]
    with torch.cuda.device(x.device):
        rc = getattr(_lib.load(), fn)(_lib.ptr(x), B, cin, L, h, w, _lib.ptr(weights), _lib.ptr(scale),
                                      _lib.ptr(bias), None if residual is None else _lib.ptr(residual.contiguous()),
                                      1 if relu else 0, cout, _lib.ptr(out), _lib.stream_ptr(x.device))
        _lib.check(rc, fn)
    return out


def conv3_bf16(x, weights, scale, bias, residual=None, relu=False, cout=32):
    """One fused layer: x [B, L, h, w, Cin] bf16, weights [27, 32, Cin] bf16,
    scale/bias [32] fp32 -> [B, L, h, w, 32] bf16 (cout 32) or [B, L, h, w]
    fp32 (cout 1)."""
    return _conv3_lp(x, weights, scale, bias, residual, relu, cout, torch.bfloat16)


def conv3_f16(x, weights, scale, bias, residual=None, relu=False, cout=32):
    """``conv3_bf16`` with float16 activations, weights and residual
    (sfm_conv3_f16)."""
    return _conv3_lp(x, weights, scale, bias, residual, relu, cout, torch.float16)


class CostRegularization(nn.Module):
    """dres0..dres4 + classify of PSNet (PSNet.py:79-102), initialised as
    PSNet.py:104-118 (Conv3d ~ N(0, sqrt(2 / (27 * out_channels))), BN = 1 / 0)."""

    def __init__(self, in_channels=64):
        super().__init__()
        if in_channels not in (32, 64):
            raise ValueError("in_channels must be 32 or 64 (2 x feature channels)")
        self.dres0 = nn.Sequential(convbn_3d(in_channels, 32), nn.ReLU(inplace=True),
                                   convbn_3d(32, 32), nn.ReLU(inplace=True))
        for i in range(1, 5):
            setattr(self, f"dres{i}", nn.Sequential(convbn_3d(32, 32), nn.ReLU(inplace=True), convbn_3d(32, 32)))
        self.classify = nn.Sequential(convbn_3d(32, 32), nn.ReLU(inplace=True),
                                      nn.Conv3d(32, 1, kernel_size=3, padding=1, stride=1, bias=False))
        for m in self.modules():
            if isinstance(m, nn.Conv3d):
                n = m.kernel_size[0] * m.kernel_size[1] * m.kernel_size[2] * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2. / n))
            elif isinstance(m, nn.BatchNorm3d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()
        self._packed = None
        self._packed_key = None

    # (conv, bn, relu, residual-from) per layer, in execution order
    def layer_plan(self):
        plan = [(self.dres0[0][0], self.dres0[0][1], True, False),
                (self.dres0[2][0], self.dres0[2][1], True, False)]
        for i in range(1, 5):
            blk = getattr(self, f"dres{i}")
            plan.append((blk[0][0], blk[0][1], True, False))
            plan.append((blk[2][0], blk[2][1], False, True))
        plan.append((self.classify[0][0], self.classify[0][1], True, False))
        plan.append((self.classify[2], None, False, False))
        return plan

    def _key(self, device):
        return (str(device),) + tuple((t.data_ptr(), t._version) for t in list(self.parameters()) + list(self.buffers()))

    def pack(self, device, precision="bf16"):
        """Packed weights [27][32][Cin] in the precision's type (fp32 / fp16 /
        bf16) and folded fp32 scale/bias per layer."""
        key = self._key(device) + (precision,)
        if self._packed is not None and self._packed_key == key:
            return self._packed
        wdt = _ACT_DTYPE[precision]
        packed = []
        with torch.no_grad():
            for conv, bn, relu, resid in self.layer_plan():
                w = conv.weight.detach().float()                    # [Cout, Cin, 3, 3, 3]
                cout, cin = w.shape[:2]
                wp = torch.zeros(27, 32, cin, dtype=torch.float32, device=w.device)
                wp[:, :cout] = w.permute(2, 3, 4, 0, 1).reshape(27, cout, cin)
                if bn is not None:
                    scale = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
                    bias = bn.bias.detach().float() - bn.running_mean.detach().float() * scale
                else:
                    scale = torch.ones(cout)
                    bias = torch.zeros(cout)
                sc = torch.ones(32)
                bi = torch.zeros(32)
                sc[:cout] = scale.cpu()
                bi[:cout] = bias.cpu()
                packed.append(dict(w=wp.to(device=device, dtype=wdt).contiguous(),
                                   scale=sc.to(device), bias=bi.to(device), cin=cin, cout=cout, relu=relu,
                                   resid=resid, wexp=weight_exponent(wp)))
        self._packed, self._packed_key = packed, key
        return packed

    def forward(self, cost, precision="fp32x3"):
        """cost [B, Cin, L, h, w] fp32 or bf16 (the sweep's volume) -> [B, 1, L, h, w] fp32.
        ``precision``: "fp32x3" (default: the reference's fp32 activations
        and weights, each product formed from a two-term f16 split of both
        operands on the f16 matrix cores, sfm_conv3_f32x3: ~2^-21 per product,
        within the float64 depth bars at 3x the speed of "fp32"; a layer whose
        input holds an activation beyond the f16 maximum 65504 is re-run as
        "fp32" on the device, see sfm_hip.h), "fp32"
        (fp32 operands on the f32 matrix cores, sfm_conv3_f32: float32
        arithmetic exactly, in another summation order),
        "fp16" (fp16
        activations and weights, fp32 accumulation: sfm_conv3_f16, the
        reference's precision under cfg.MIXED_PREC) or "bf16" (bf16, fp32
        accumulation: sfm_conv3_bf16, the fastest opt-in)."""
        if precision not in _ACT_DTYPE:
            raise ValueError(f"unknown conv precision {precision!r}")
        if not (isinstance(cost, torch.Tensor) and cost.is_cuda):
            raise RuntimeError("CostRegularization.forward needs a device tensor (HIP path, no CPU fallback)")
        if cost.dtype not in (torch.float32, torch.bfloat16) or cost.dim() != 5:
            raise RuntimeError("cost must be a [B, C, L, h, w] float32 or bfloat16 tensor")
        cost = cost.contiguous()
        B, C, L, h, w = cost.shape
        packed = self.pack(cost.device, precision)
        if C != packed[0]["cin"]:
            raise RuntimeError(f"cost has {C} channels, the first layer expects {packed[0]['cin']}")
        lib = _lib.load()
        dev = cost.device
        adt = _ACT_DTYPE[precision]
        suffix = {"fp32": "f32", "fp32x3": "f32", "fp16": "f16", "bf16": "bf16"}[precision]
        to_cl = getattr(lib, "sfm_to_channels_last_" + suffix)
        if precision == "fp32x3":
            # the split-f16 kernel takes the weights' power-of-two exponent after them
            x3 = lib.sfm_conv3_f32x3
            fn_name = "sfm_conv3_f32x3"
        else:
            conv = getattr(lib, "sfm_conv3_" + suffix)
            fn_name = "sfm_conv3_" + suffix
        with torch.cuda.device(dev):
            stream = _lib.stream_ptr(dev)
            x = torch.empty((B, L, h, w, C), dtype=adt, device=dev)
            _lib.check(to_cl(_lib.ptr(cost), 0 if cost.dtype == torch.float32 else 1, B, C, L * h * w, _lib.ptr(x),
                             stream), "sfm_to_channels_last")
            bufs = [torch.empty((B, L, h, w, 32), dtype=adt, device=dev) for _ in range(3)]
            out = torch.empty((B, 1, L, h, w), dtype=torch.float32, device=dev)
            # fp32x3: one range flag per layer -- a layer whose input leaves the
            # f16 range is re-run by sfm_conv3_f32 inside the same call, stream-ordered
            flags = torch.empty(len(packed), dtype=torch.int32, device=dev) if precision == "fp32x3" else None
            cur, keep = x, None           # keep: the block input of a residual pair (cost0)
            for li, lay in enumerate(packed):
                if lay["cout"] == 1:
                    dst = out
                else:
                    dst = next(bb for bb in bufs if bb is not cur and bb is not keep)
                res = keep if lay["resid"] else None
                if precision == "fp32x3":
                    rc = x3(_lib.ptr(cur), B, lay["cin"], L, h, w, _lib.ptr(lay["w"]), lay["wexp"],
                            _lib.ptr(lay["scale"]), _lib.ptr(lay["bias"]), None if res is None else _lib.ptr(res),
                            1 if lay["relu"] else 0, lay["cout"], _lib.ptr(dst), flags[li].data_ptr(), stream)
                else:
                    rc = conv(_lib.ptr(cur), B, lay["cin"], L, h, w, _lib.ptr(lay["w"]), _lib.ptr(lay["scale"]),
                              _lib.ptr(lay["bias"]), None if res is None else _lib.ptr(res), 1 if lay["relu"] else 0,
                              lay["cout"], _lib.ptr(dst), stream)
                _lib.check(rc, fn_name)
                # cost0 after dres0 (layer 1) and after every residual add is the next block's input
                if li == 1 or lay["resid"]:
                    keep = dst
                cur = dst
        return out


def psnet_depth(ref_fea, tgt_fea, pose, intrinsics, intrinsics_inv, regularizer, nlabel, min_depth=1.0,
                out_hw=None, predict_by_depth=False, cost_dtype=torch.float32, precision=None):
    """PSNet's single-target depth path at feature resolution, PSNet.py:130-216
    without the context network (cfg.PSNET_CONTEXT off): plane sweep ->
    dres/classify -> trilinear upsample, softmax, disparity regression.
    ``pose`` [B,3,4] already rescaled; full-resolution intrinsics.
    Returns depth [B, 1, H, W] fp32."""
    K4, Ki4 = quarter_intrinsics(intrinsics, intrinsics_inv)
    cost = plane_sweep_cost(ref_fea, tgt_fea, pose, K4, Ki4, nlabel, min_depth, dtype=cost_dtype,
                            predict_by_depth=predict_by_depth)
    costs = regularizer(cost) if precision is None else regularizer(cost, precision=precision)
    B = costs.shape[0]
    h, w = costs.shape[-2:]
    H, W = out_hw if out_hw is not None else (4 * h, 4 * w)
    return depth_head(costs.view(B, int(nlabel), h, w), nlabel, min_depth, out_hw=(H, W),
                      predict_by_depth=predict_by_depth)
