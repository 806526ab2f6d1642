"""PSNet-layout depth estimator: SFMnet's default ``depth_estimator``.

The reference builds ``PSNet(nlabel, min_depth)`` inside ``SFMnet.__init__``
(models/SFMnet.py:57-58; PSNet models/PSNet.py:40-227).  This module keeps
PSNet's module names and constructor, so a PSNet state_dict loads unchanged,
and runs its forward with the hot path on libsfm_hip:

  feature_extraction  2-D CNN at 1/4 resolution, 32 channels         torch (MIOpen)
                      (PSMNet SPP layout, models/submodule.py:108-184)
  plane sweep         cost [B, 64, L, h, w] (PSNet.py:130-158)        sfm_plane_sweep (HIP)
  dres0..4, classify  3-D cost regularisation (PSNet.py:79-102, 159-165)  sfm_conv3_* (HIP MFMA)
  convs               per-plane context CNN (PSNET_CONTEXT, 175-192)   torch (MIOpen)
  head                trilinear up, softmax, disparity regression     sfm_depth_head (HIP)
  dep_convs           full-resolution depth refinement (PSNET_DEP_CONTEXT, 218-225)  torch (MIOpen)

The 2-D CNNs are outside the measured path (feature CNN and
context networks are out of scope); they are plain torch modules here so the
estimator is complete and a reference checkpoint's weights apply.  The
``COST_BY_COLOR`` ablations (PSNet.py:75-78, 181-188) are not built.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import cfg as _default_cfg
from .depth import depth_head
from .regularize import CostRegularization
from .sweep import plane_sweep_cost, quarter_intrinsics


def _conv_bn(cin, cout, k, stride, pad, dilation):
    """Conv2d (no bias) + BatchNorm2d; a dilated conv pads by its dilation
    (models/submodule.py:11-15)."""
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride=stride, padding=dilation if dilation > 1 else pad,
                                   dilation=dilation, bias=False),
                         nn.BatchNorm2d(cout))


class _Residual(nn.Module):
    """Two 3x3 conv-BN stages with a ReLU between, plus the (projected) input."""

    def __init__(self, cin, cout, stride, pad, dilation):
        super().__init__()
        self.conv1 = nn.Sequential(_conv_bn(cin, cout, 3, stride, pad, dilation), nn.ReLU(inplace=True))
        self.conv2 = _conv_bn(cout, cout, 3, 1, pad, dilation)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = self.conv2(self.conv1(x))
        return y + (x if self.downsample is None else self.downsample(x))


class FeatureExtraction(nn.Module):
    """PSNet's feature CNN (layout of models/submodule.py:108-184): stride-2
    stem, four residual stages (the second stride 2, the last dilated), four
    average-pool pyramid branches upsampled back, and a 320 -> 32 fusion."""

    # (attribute, channels, blocks, stride, dilation)
    STAGES = (("layer1", 32, 3, 1, 1), ("layer2", 64, 16, 2, 1), ("layer3", 128, 3, 1, 1), ("layer4", 128, 3, 1, 2))
    POOLS = (32, 16, 8, 4)      # branch1..branch4

    def __init__(self):
        super().__init__()
        self.firstconv = nn.Sequential(_conv_bn(3, 32, 3, 2, 1, 1), nn.ReLU(inplace=True),
                                       _conv_bn(32, 32, 3, 1, 1, 1), nn.ReLU(inplace=True),
                                       _conv_bn(32, 32, 3, 1, 1, 1), nn.ReLU(inplace=True))
        cin = 32
        for name, ch, blocks, stride, dil in self.STAGES:
            mods = [_Residual(cin, ch, stride, 1, dil)] + [_Residual(ch, ch, 1, 1, dil) for _ in range(blocks - 1)]
            setattr(self, name, nn.Sequential(*mods))
            cin = ch
        for i, p in enumerate(self.POOLS):
            setattr(self, f"branch{i + 1}", nn.Sequential(nn.AvgPool2d((p, p), stride=(p, p)),
                                                          _conv_bn(128, 32, 1, 1, 0, 1), nn.ReLU(inplace=True)))
        self.lastconv = nn.Sequential(_conv_bn(320, 128, 3, 1, 1, 1), nn.ReLU(inplace=True),
                                      nn.Conv2d(128, 32, kernel_size=1, padding=0, stride=1, bias=False))

    def forward(self, x):
        x = self.layer1(self.firstconv(x))
        raw = self.layer2(x)
        skip = self.layer4(self.layer3(raw))
        size = skip.shape[2:]
        pyr = [F.interpolate(getattr(self, f"branch{i}")(skip), size, mode="bilinear", align_corners=True)
               for i in (4, 3, 2, 1)]
        return self.lastconv(torch.cat([raw, skip] + pyr, 1))


def _context_conv(cin, cout, k=3, stride=1, dilation=1, bn=False):
    """PSNet.py:17-26 (convtext)."""
    conv = nn.Conv2d(cin, cout, kernel_size=k, stride=stride, dilation=dilation,
                     padding=((k - 1) * dilation) // 2, bias=False)
    return nn.Sequential(conv, nn.BatchNorm2d(cout), nn.ReLU(inplace=True)) if bn else \
        nn.Sequential(conv, nn.ReLU(inplace=True))


def _context_stack(cin, bn):
    """Seven dilated 3x3 stages cin -> 128 -> ... -> 1 (PSNet.py:54-70)."""
    plan = ((cin, 128, 1), (128, 128, 2), (128, 128, 4), (128, 96, 8), (96, 64, 16), (64, 32, 1), (32, 1, 1))
    return nn.Sequential(*[_context_conv(a, b, 3, 1, d, bn) for a, b, d in plan])


class PSNet(CostRegularization):
    """``PSNet(nlabel, mindepth)`` with the reference's module names
    (feature_extraction, dres0..4, classify, convs, dep_convs, context_net)
    and forward signature / return value ``(depth_init, depth)``
    (PSNet.py:128, 214-227).

    ``feature_fn`` replaces the feature CNN (any callable image -> [B, 32,
    H/4, W/4]); ``conv_precision`` selects the regularisation arithmetic
    (CostRegularization): "auto" (default) follows the reference --
    PSNet.py:159-165 in float32, or in float16 under cfg.MIXED_PREC, the
    autocast SFMnet.py:164 wraps the depth estimator in (cfgs/kitti.yml:10) --
    so it resolves to "fp32x3" (fp32 operands, each product from a two-term
    f16 split on the f16 matrix cores: within the float64 fixture's depth bars
    at 3x the speed of "fp32", the f32-MFMA path, which stays selectable) or
    "fp16"; "bf16" is the fastest opt-in path;
    ``cost_dtype`` the sweep volume's storage."""

    def __init__(self, nlabel, mindepth=None, cfg=None, feature_fn=None, cost_dtype=torch.float32,
                 conv_precision="auto"):
        super().__init__(64)
        c = _default_cfg if cfg is None else cfg
        if c.get("COST_BY_COLOR", False) or c.get("COST_BY_COLOR_WITH_FEAT", False):
            raise RuntimeError("PSNet: the COST_BY_COLOR ablations (PSNet.py:75-78) are not built")
        self.cfg = c
        self.nlabel = int(nlabel)
        self.mindepth = float(c.MIN_DEPTH)            # the reference reads cfg.MIN_DEPTH too (PSNet.py:44)
        self.cost_dtype = cost_dtype
        if conv_precision == "auto":
            conv_precision = "fp16" if c.get("MIXED_PREC", False) else "fp32x3"
        if conv_precision not in ("fp32", "fp32x3", "fp16", "bf16"):
            raise ValueError(f"unknown conv precision {conv_precision!r}")
        self.conv_precision = conv_precision
        self.feature_extraction = FeatureExtraction() if feature_fn is None else feature_fn
        if c.get("IND_CONTEXT", False):
            self.context_net = FeatureExtraction()
        bn = bool(c.get("CONTEXT_BN", False))
        self.convs = _context_stack(33, bn)
        if c.get("PSNET_DEP_CONTEXT", False):
            self.dep_convs = _context_stack(36, bn)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def regularize(self, cost):
        return CostRegularization.forward(self, cost, precision=self.conv_precision)

    def forward(self, ref, targets, pose, intrinsics, intrinsics_inv, pose_gt=None, depth_gt=None, E_mat=None):
        c = self.cfg
        K4, Ki4 = quarter_intrinsics(intrinsics.float(), intrinsics_inv.float())
        if c.get("RESCALE_DEPTH", False):
            pose[:, 0, :, -1:] = pose[:, 0, :, -1:] * c.NORM_TARGET      # in place, PSNet.py:135-136
        pbd = bool(c.get("PREDICT_BY_DEPTH", False))
        ref_fea = self.feature_extraction(ref).float()
        costs = None
        for j, target in enumerate(targets):
            tgt_fea = self.feature_extraction(target).float()
            cost = plane_sweep_cost(ref_fea.contiguous(), tgt_fea.contiguous(), pose[:, j].float().contiguous(),
                                    K4, Ki4, self.nlabel, self.mindepth, dtype=self.cost_dtype,
                                    predict_by_depth=pbd)
            c0 = self.regularize(cost)
            costs = c0 if costs is None else costs + c0
        costs = costs / len(targets)                                   # [B, 1, L, h, w]
        B, _, L, h, w = costs.shape
        H, W = ref.shape[2], ref.shape[3]
        costss = costs
        if c.get("PSNET_CONTEXT", True):
            if c.get("IND_CONTEXT", False):
                ref_fea = self.context_net(ref).float()        # PSNet.py:177-178 reassigns refimg_fea
            ctx = ref_fea
            # every plane through the same 2-D stack: one batch of B*L images
            planes = costs[:, 0].permute(1, 0, 2, 3).reshape(L * B, 1, h, w)
            x = torch.cat([ctx.unsqueeze(0).expand(L, B, ctx.shape[1], h, w).reshape(L * B, -1, h, w), planes], 1)
            costss = (self.convs(x) + planes).reshape(L, B, h, w).permute(1, 0, 2, 3).unsqueeze(1)
        # PREDICT_BY_DEPTH: depth_init is depthregression's output unscaled,
        # depth is scaled by mindepth (PSNet.py:200-202 vs 209-210)
        depth_init = depth_head(costs.reshape(B, L, h, w).contiguous(), self.nlabel, self.mindepth, (H, W), pbd,
                                scale=1.0 if pbd else None)
        depth = depth_head(costss.reshape(B, L, h, w).contiguous(), self.nlabel, self.mindepth, (H, W), pbd)
        if c.get("PSNET_DEP_CONTEXT", False):
            up = F.interpolate(ref_fea, [H, W], mode="bilinear", align_corners=True)
            feat = torch.cat((depth.detach(), up, ref.float()), dim=1)
            return depth, self.dep_convs(feat) + depth
        return depth_init, depth


def default_feature_hw(image_hw):
    """Feature map size of FeatureExtraction for an image (two stride-2 convs)."""
    H, W = image_hw
    h = (H - 1) // 2 + 1
    w = (W - 1) // 2 + 1
    return (h - 1) // 2 + 1, (w - 1) // 2 + 1

