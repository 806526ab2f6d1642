"""The aligned-slab sweep kernels (k_sweep_tile, the default, sweep_flat=2;
k_sweep_flat, sweep_flat=1) against the per-row kernel (sweep_flat=0) and the
oracle: both group sizes, every window width of k_sweep_tile (bit-identical to
k_sweep_flat of the same group),
edge windows, feature maps under one 1024-pixel window, odd slabs and output
pointers off the 256-byte grid; and the plane-run kernel k_sweep_band
(sweep_flat=3: target band in LDS, bit-identical to k_sweep_tile) at several
run lengths and LDS band heights, down to a 2-row band whose taps mostly take
the global-gather path.  Sample positions are bit-identical
(warp.h sample_pos_nr); the 4-tap sum differs by FMA rounding only."""
import pytest
import torch

from oracle import sweep as S

pytestmark = pytest.mark.gpu

RTOL, FLOOR = 1e-4, 1.0    # the tolerance of test_gpu_sweep.py: 1e-4 * max(|b|, feature RMS)


@pytest.mark.parametrize("B,C,L,h,w,dtype,offset", [
    (2, 32, 16, 47, 156, torch.float32, 0),    # slab % 64 != 0: per-row misaligned groups
    (1, 6, 5, 13, 21, torch.float32, 1),       # hw < 1024: windows span several planes; out 4 B off
    (1, 10, 4, 20, 64, torch.float32, 3),      # slab % 64 == 0, output pointer misaligned
    (1, 5, 3, 11, 19, torch.bfloat16, 1),      # odd slab: bf16 element stores
    (2, 12, 6, 16, 40, torch.bfloat16, 0),     # bf16 pair stores, partial group of 8
    (1, 8, 4, 9, 13, torch.bfloat16, 2),       # even slab, output 4 B off: pair stores
    (1, 8, 8, 12, 25, torch.bfloat16, 4),      # even slab, output 8 B off
])
def test_aligned_slab_kernels_match_per_row(cuda, B, C, L, h, w, dtype, offset):
    from sfm_amd import _lib, synth
    from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics
    ref, tgt = synth.features(B, C, h, w, seed=C * L + w)
    K = synth.intrinsics(B, 4.0 * w, 4.0 * w, 2.0 * w, 2.0 * h)
    Ki = torch.inverse(K)
    pose = synth.relative_pose(B, torch.Generator().manual_seed(L + h))
    K4, Ki4 = quarter_intrinsics(K, Ki)
    args = (ref.to(cuda), tgt.to(cuda), pose.to(cuda), K4.to(cuda), Ki4.to(cuda), L, 0.8)
    n = B * 2 * C * L * h * w
    outs = {}
    try:
        for flat, group, nj in ((0, 4, 1), (1, 4, 1), (1, 8, 1), (2, 4, 1), (2, 4, 2), (2, 4, 4),
                                (2, 8, 1), (2, 8, 2), (2, 8, 4),
                                # k_sweep_band: (3, planes per block, LDS band rows); 2 rows
                                # sends most taps down the global-gather path
                                (3, 16, 16), (3, 3, 16), (3, 1, 2), (3, 5, 3),
                                # k_sweep_tile without its buffer-addressed interior path
                                (2, 8, -1), (2, 4, -2)):
            _lib.tune("sweep_flat", flat)
            _lib.tune("sweep_buffer", 0 if nj < 0 else 1)
            nj = abs(nj)
            if flat == 3:
                _lib.tune("sweep_run", group)
                _lib.tune("sweep_band_rows", nj)
            else:
                _lib.tune("sweep_group", group)
                _lib.tune("sweep_nj", nj)
            buf = torch.full((n + offset,), float("nan"), dtype=dtype, device=cuda)
            out = buf[offset:].view(B, 2 * C, L, h, w)
            plane_sweep_cost(*args, dtype=dtype, out=out)
            outs[(flat, group, nj) if _lib.tune_get("sweep_buffer") else (flat, group, -nj)] = out.float().cpu()
    finally:
        _lib.tune("sweep_flat", 2)
        _lib.tune("sweep_group", 8)
        _lib.tune("sweep_nj", 1)
        _lib.tune("sweep_run", 16)
        _lib.tune("sweep_band_rows", 16)
        _lib.tune("sweep_buffer", 1)
    base = outs[(0, 4, 1)]
    assert not torch.isnan(base).any()
    tol = 2e-6 if dtype == torch.float32 else 1e-2
    for key, got in outs.items():
        if key[0] == 0:
            continue
        assert not torch.isnan(got).any(), key            # every element written
        assert torch.equal(got[:, :C], base[:, :C]), key  # reference half: exact copy
        assert float((got - base).abs().max()) <= tol, (key, float((got - base).abs().max()))
        if key[0] == 2:                                   # same arithmetic as k_sweep_flat
            assert torch.equal(got, outs[(1, key[1], 1)]), key
        if key[0] == 3 or key[2] < 0:                     # same arithmetic as k_sweep_tile
            assert torch.equal(got, outs[(2, 8, 1)]), key
    if dtype == torch.float32:
        want = S.plane_sweep_cost(ref, tgt, pose, K, Ki, L, 0.8)
        got = outs[(2, 8, 1)]
        err = (got - want).abs() - RTOL * torch.clamp(want.abs(), min=FLOOR)
        assert float(err.max()) <= 0.0, float((got - want).abs().max())


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("run,rows", [(16, 16), (32, 6), (128, 16)])
def test_band_kernel_full_size_kitti(cuda, dtype, run, rows):
    """k_sweep_band at the bench's volume (94x311, L=128, C=32, B=2, translation
    scaled to 0.6 as the bench's RESCALE_DEPTH pose): bit-identical to
    k_sweep_tile for run lengths whose bands fit the LDS and ones that do not
    (6 rows, a 128-plane run: clipped bands, global gathers for the rest)."""
    from sfm_amd import _lib, synth
    from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics
    B, C, L = 2, 32, 128
    h, w = synth.feature_hw()
    ref, tgt = synth.features(B, C, h, w, seed=11)
    K = synth.intrinsics(B)
    Ki = torch.inverse(K)
    pose = synth.relative_pose(B, torch.Generator().manual_seed(3))
    pose[:, :, 3] *= 0.6 / pose[:, :, 3].norm(dim=1, keepdim=True)
    K4, Ki4 = quarter_intrinsics(K, Ki)
    args = (ref.to(cuda), tgt.to(cuda), pose.to(cuda), K4.to(cuda), Ki4.to(cuda), L, 1.0)
    try:
        _lib.tune("sweep_flat", 2)
        want = plane_sweep_cost(*args, dtype=dtype)
        _lib.tune("sweep_buffer", 0)                  # the generic k_sweep_tile body
        assert torch.equal(plane_sweep_cost(*args, dtype=dtype), want)
        _lib.tune("sweep_buffer", 1)
        _lib.tune("sweep_flat", 3)
        _lib.tune("sweep_run", run)
        _lib.tune("sweep_band_rows", rows)
        got = plane_sweep_cost(*args, dtype=dtype)
    finally:
        _lib.tune("sweep_flat", 2)
        _lib.tune("sweep_run", 16)
        _lib.tune("sweep_band_rows", 16)
    assert torch.equal(got, want)
    assert float(want[:, C:].float().abs().sum()) > 0.0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,L,hw,tscale,by_depth", [
    (2, 32, 128, None, 0.6, False),     # the bench's volume (94x311, RESCALE_DEPTH pose)
    (1, 32, 64, None, 3.0, True),       # large baseline, depth planes: taps far apart
    (2, 16, 8, (40, 300), 0.6, False),  # windows across row and plane ends
    (1, 8, 5, (13, 64), 1.0, False),    # hw < 256: windows span several planes
])
def test_shared_taps_equal_gathered(cuda, dtype, B, C, L, hw, tscale, by_depth):
    """sweep_share=1 (k_sweep_tile's interior path takes each lane's right-hand
    taps from the next lane where the tap offsets are equal) writes the same
    bits as the gathering path, whatever the share rate; so do the
    non-temporal volume stores (sweep_store_nt; by default bf16 only) and
    plain ones."""
    from sfm_amd import _lib, synth
    from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics
    h, w = hw or synth.feature_hw()
    ref, tgt = synth.features(B, C, h, w, seed=C + L)
    K = synth.intrinsics(B, 4.0 * w, 4.0 * w, 2.0 * w, 2.0 * h) if hw else synth.intrinsics(B)
    Ki = torch.inverse(K)
    pose = synth.relative_pose(B, torch.Generator().manual_seed(L))
    pose[:, :, 3] *= tscale / pose[:, :, 3].norm(dim=1, keepdim=True)
    K4, Ki4 = quarter_intrinsics(K, Ki)
    args = (ref.to(cuda), tgt.to(cuda), pose.to(cuda), K4.to(cuda), Ki4.to(cuda), L, 1.0)
    old = _lib.tune_get("sweep_share"), _lib.tune_get("sweep_store_nt")
    try:
        outs = []
        for share, nt in ((0, 0), (1, 0), (0, 1), (1, 1)):
            _lib.tune("sweep_share", share)
            _lib.tune("sweep_store_nt", nt)
            outs.append(plane_sweep_cost(*args, dtype=dtype, predict_by_depth=by_depth))
    finally:
        _lib.tune("sweep_share", old[0])
        _lib.tune("sweep_store_nt", old[1])
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    assert float(outs[0][:, C:].float().abs().sum()) > 0.0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,C,L,hw,tscale,by_depth", [
    (4, 32, 128, None, 0.6, False),     # the C3 volume (94x311, RESCALE_DEPTH pose)
    (1, 32, 64, None, 3.0, True),       # large baseline, depth planes
    (2, 16, 8, (40, 300), 0.6, False),  # windows across row and plane ends
    (1, 8, 5, (13, 64), 1.0, False),    # hw < 256: windows span several planes
    (1, 8, 5, (13, 61), 1.0, False),    # odd slab: wide stores fall back to the plain path
    (1, 8, 8, (13, 61), 1.0, False),    # odd h*w, slab a multiple of 8: wide stores
    (2, 12, 6, (20, 96), 0.8, False),   # a partial channel group (C = 12, groups of 8)
])
def test_wide_stores_equal_plain(cuda, dtype, B, C, L, hw, tscale, by_depth):
    """sweep_store_px (16-byte lane stores of 8 bf16 / 4 fp32 consecutive
    pixels, transposed through a per-wave LDS stage, with px pixels per lane
    for the taps) writes the same bits as the plain 4-byte lane stores, with
    and without non-temporal stores, under every write-through policy
    (sweep_store_wt)."""
    from sfm_amd import _lib, synth
    from sfm_amd.sweep import plane_sweep_cost, quarter_intrinsics
    h, w = hw or synth.feature_hw()
    ref, tgt = synth.features(B, C, h, w, seed=C + L)
    K = synth.intrinsics(B, 4.0 * w, 4.0 * w, 2.0 * w, 2.0 * h) if hw else synth.intrinsics(B)
    Ki = torch.inverse(K)
    pose = synth.relative_pose(B, torch.Generator().manual_seed(L))
    pose[:, :, 3] *= tscale / pose[:, :, 3].norm(dim=1, keepdim=True)
    K4, Ki4 = quarter_intrinsics(K, Ki)
    args = (ref.to(cuda), tgt.to(cuda), pose.to(cuda), K4.to(cuda), Ki4.to(cuda), L, 1.0)
    # (store_px, store_nt, store_wt); the autouse fixture restores the tuning
    if dtype == torch.bfloat16:
        cases = ((0, 2, 0), (-1, 2, -1), (2, 2, 1), (2, 2, 3), (4, 2, -1), (4, 2, 2), (8, 2, -1), (8, 0, 3),
                 (2, 0, 0))
    else:
        cases = ((0, 2, 0), (-1, 2, -1), (1, 2, 0), (1, 2, 1), (1, 2, 2), (2, 2, -1), (4, 2, 3), (1, 1, 0),
                 (2, 1, 0))
    outs = []
    for px, nt, wt in cases:
        _lib.tune("sweep_store_px", px)
        _lib.tune("sweep_store_nt", nt)
        _lib.tune("sweep_store_wt", wt)
        outs.append(plane_sweep_cost(*args, dtype=dtype, predict_by_depth=by_depth))
    bad = {}
    iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
    for case, o in zip(cases[1:], outs[1:]):
        d = (outs[0].view(iv) != o.view(iv)).nonzero()
        if len(d):
            bad[case] = (len(d), d[:4].tolist())
    assert not bad, bad
    assert float(outs[0][:, C:].float().abs().sum()) > 0.0
