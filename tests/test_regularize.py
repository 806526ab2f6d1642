"""CPU checks of the PSNet cost-regularisation mirror (no compute on a GPU):
module layout matches PSNet.py:79-102, the folded layer plan reproduces the
modules' own forward, and the product path refuses CPU tensors."""
import numpy as np
import pytest
import torch

from oracle import regularize as R


def _module(seed, cin=64, random_bn=True):
    from sfm_amd.regularize import CostRegularization
    torch.manual_seed(seed)
    m = CostRegularization(cin)
    if random_bn:
        g = torch.Generator().manual_seed(seed + 1)
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm3d):
                n = mod.num_features
                mod.weight.data = 0.5 + torch.rand(n, generator=g)
                mod.bias.data = 0.2 * torch.randn(n, generator=g)
                mod.running_mean.data = 0.1 * torch.randn(n, generator=g)
                mod.running_var.data = 0.5 + torch.rand(n, generator=g)
    return m.eval()


def test_state_dict_keys_match_psnet():
    m = _module(0)
    keys = set(m.state_dict().keys())
    # PSNet.py:79-102: dres0 = Seq(convbn_3d, ReLU, convbn_3d, ReLU); convbn_3d = Seq(Conv3d, BN3d)
    for k in ("dres0.0.0.weight", "dres0.0.1.running_var", "dres0.2.0.weight", "dres4.2.1.bias",
              "classify.0.0.weight", "classify.2.weight"):
        assert k in keys, k
    assert m.dres0[0][0].weight.shape == (32, 64, 3, 3, 3)
    assert m.classify[2].weight.shape == (1, 32, 3, 3, 3)
    assert len(m.layer_plan()) == 12


@pytest.mark.parametrize("cin", [64, 32])
def test_layer_plan_equals_module_forward(cin):
    m = _module(3, cin)
    cost = torch.randn(1, cin, 5, 6, 7, generator=torch.Generator().manual_seed(9))
    a = R.regularize_fp32(m, cost)
    b = R.regularize_fp32_plan(m, cost)
    assert a.shape == (1, 1, 5, 6, 7)
    # folding BN into scale/bias reorders fp32 rounding only
    rel = float((a - b).norm() / a.norm())
    assert rel < 1e-5, rel


def test_bf16_storage_stays_within_tolerance_of_fp32():
    # the storage-precision tolerance the GPU tests use against the fp32 stack
    m = _module(5)
    cost = torch.randn(2, 64, 6, 9, 11, generator=torch.Generator().manual_seed(2))
    a = R.regularize_fp32(m, cost)
    b = R.regularize_bf16(m, cost)
    rel = float((a - b).norm() / a.norm())
    assert rel < 2e-2, rel


def test_product_path_refuses_cpu_tensors():
    m = _module(1)
    with pytest.raises(RuntimeError):
        m(torch.randn(1, 64, 3, 4, 5))


def _psnet_module(g):
    from sfm_amd.regularize import CostRegularization
    m = CostRegularization(64)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in g["state"].items()})
    return m.eval()


def test_oracles_match_reference_psnet(golden):
    """psnet.npz (SURVEY §8(c) golden #5, the reference PSNet's own forward at
    seed 0): the sweep oracle rebuilds its cost volume from its features, the
    regularisation oracle its classify output, the head oracle its depth."""
    from oracle import regularize as R
    from oracle import sweep as S
    g = golden("psnet.npz")
    inp, out = g["input"], g["out"]
    L = int(inp["nlabel"])
    K = torch.from_numpy(inp["K"]); Ki = torch.from_numpy(inp["Kinv"])
    pose = torch.from_numpy(inp["pose_rescaled"])[:, 0]
    cost = S.plane_sweep_cost(torch.from_numpy(out["ref_fea"]), torch.from_numpy(out["tgt_fea"]), pose, K, Ki, L,
                              float(inp["min_depth"]))
    want = torch.from_numpy(out["cost"])
    assert float((cost - want).abs().max()) <= 1e-5
    m = _psnet_module(g)
    cls = R.regularize_fp32_plan(m, want)          # folded-BN plan == the reference's module forward
    ref_cls = torch.from_numpy(out["classify"])
    assert float((cls - ref_cls).abs().max()) <= 1e-4 * float(ref_cls.abs().max())
    depth = S.depth_head(ref_cls, L, float(inp["min_depth"]), out_hw=tuple(inp["ref_img"].shape[2:]))
    assert float(((depth - torch.from_numpy(out["depth_init"])).abs() / depth.abs()).max()) <= 1e-6
    # PSNET_CONTEXT off: the refined depth equals depth_init
    assert np.array_equal(out["depth"], out["depth_init"])
