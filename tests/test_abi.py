"""CPU-side checks of the C ABI: the library loads and exports every symbol
include/sfm_hip.h declares; host-only entry points (IRLS, decompose) match the
reference's host code bit-for-bit; argument validation fails loudly."""
import ctypes
import os
import re
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "sfm_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(sfm_\w+)\s*\(", hdr, re.M)))


def test_header_symbols_exported():
    from sfm_amd import _lib
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SYMBOLS)
    assert lib.sfm_abi_version() == 1


def test_integration_indexes_every_entry_point():
    """INTEGRATION.md's entry-point index names every declared function (the
    bindings a maintainer writes against the reference's interface)."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    missing = [n for n in _declared() if f"`{n}`" not in doc]
    assert not missing, missing


def test_workspace_query():
    from sfm_amd import _lib
    lib = _lib.load()
    a = lib.sfm_ransac5_workspace_bytes(1, 0, 8)
    b = lib.sfm_ransac5_workspace_bytes(8, 0, 8)
    c = lib.sfm_ransac5_workspace_bytes(8, 435032, 8)
    assert 0 < a < b < c
    assert c - b >= 435032 * 32
    assert lib.sfm_ransac5_workspace_bytes(0, 0, 8) == 0


def test_host_entry_points_match_reference(golden):
    import essential_matrix
    for k, c in golden("irls.npz").items():
        q = torch.from_numpy(c["q"]); qp = torch.from_numpy(c["qp"]); E = torch.from_numpy(c["E_init"])
        assert np.array_equal(essential_matrix.optimise(q, qp, E, 0.001, 0.0, 200).numpy(), c["E_opt"]), k
        assert np.array_equal(essential_matrix.optimise(q, qp, E, 0.002, 1.0, 20).numpy(), c["E_opt_huber"]), k
        assert np.array_equal(essential_matrix.decompose(E).numpy(), c["params"])
        U, V = essential_matrix.decomposeUV(E)
        assert np.array_equal(U.numpy(), c["U"]) and np.array_equal(V.numpy(), c["V"])


def test_argument_validation_is_loud():
    from sfm_amd import _lib
    lib = _lib.load()
    # null pointers / bad sizes are rejected before touching the device
    rc = lib.sfm_ransac5(None, None, 10, 10, 10, 1, 1e-3, 1234, 1, None, 0, None, None, None, None, None)
    assert rc == 1 and b"null" in lib.sfm_last_error()
    n = (ctypes.c_int64 * 1)(5)
    rc = lib.sfm_ransac5_packed(ctypes.c_void_p(8), 5, n, 1, 10, 10, 1, 1e-3, 1234, 1, None, 0,
                                ctypes.c_void_p(8), ctypes.c_void_p(8), ctypes.c_void_p(8), None, None, None)
    assert rc == 1 and b"exceed" in lib.sfm_last_error()
    rc = lib.sfm_plane_sweep(None, None, 1, 32, 10, 10, None, None, None, 8, 1.0, 0, None, None, 0, None)
    assert rc == 1
    rc = lib.sfm_plane_sweep(ctypes.c_void_p(8), ctypes.c_void_p(8), 1, 32, 10, 10, ctypes.c_void_p(8),
                             ctypes.c_void_p(8), ctypes.c_void_p(8), 8, 1.0, 0, ctypes.c_void_p(8), None, 0, None)
    assert rc == 3 and b"workspace" in lib.sfm_last_error()
    import essential_matrix
    with pytest.raises(RuntimeError, match="double"):
        essential_matrix.optimise(torch.zeros(4, 2), torch.zeros(4, 2), torch.eye(3), 1e-3, 0.0, 5)


def test_product_does_not_import_oracle():
    pkg = os.path.join(ROOT, "deep-sfm-revisited_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                src = open(os.path.join(dp, f)).read()
                assert "oracle" not in re.sub(r"#.*|//.*", "", src).lower().replace("oracle/", ""), f


def test_new_entry_points_validate_arguments():
    """Argument checks of the later entry points fail loudly without touching
    the device (no GPU here)."""
    from sfm_amd import _lib
    lib = _lib.load()
    v = ctypes.c_void_p(8)
    n = (ctypes.c_int64 * 2)(5, 7)
    # keypoints: bad mode, SIFT_POSE without target keypoints, counts beyond the stride
    assert lib.sfm_keypoints_to_points(v, 2, 10, 10, 10, 10, v, None, 8, n, 3, v, v, 8, None) == 1
    assert lib.sfm_keypoints_to_points(None, 2, 10, 10, 10, 10, v, None, 8, n, 2, v, v, 8, None) == 1
    assert b"target" in lib.sfm_last_error()
    assert lib.sfm_keypoints_to_points(v, 2, 10, 10, 10, 10, v, None, 6, n, 0, v, v, 8, None) == 1
    # correlation: workspace query and missing workspace
    assert lib.sfm_correlation_workspace_bytes(2, 32, 10, 20) > 0
    assert lib.sfm_correlation_workspace_bytes(0, 32, 10, 20) == 0
    rc = lib.sfm_plane_sweep_correlation(v, v, 1, 4, 8, 8, v, v, v, 4, 1.0, 0, v, None, 0, None)
    assert rc == 3 and b"workspace" in lib.sfm_last_error()
    assert lib.sfm_plane_sweep_correlation(v, v, 1, 4, 8, 8, v, v, v, 4, 1.0, 2, v, v, 1 << 20, None) == 1
    # depth head: PREDICT_BY_DEPTH needs a positive step; bad mode
    assert lib.sfm_depth_head(v, 1, 8, 4, 4, 16, 16, 1, 1.0, 0.0, v, None) == 1
    assert lib.sfm_depth_head(v, 1, 8, 4, 4, 16, 16, 5, 1.0, 1.0, v, None) == 1
    # GPU IRLS: counts beyond the stride, negative reps, too-small workspace
    assert lib.sfm_essential_optimise_workspace_bytes(2, 1000) > 0
    assert lib.sfm_essential_optimise_batched(v, 6, n, 2, v, 1e-3, 0.0, 10, v, v, 1 << 20, None) == 1
    assert lib.sfm_essential_optimise_batched(v, 8, n, 2, v, 1e-3, 0.0, -1, v, v, 1 << 20, None) == 1
    rc = lib.sfm_essential_optimise_batched(v, 8, n, 2, v, 1e-3, 0.0, 10, v, v, 16, None)
    assert rc == 3 and b"workspace" in lib.sfm_last_error()
    # plane sweep ex: bad depth mode, non-positive min depth
    assert lib.sfm_plane_sweep_ex(v, v, 1, 4, 8, 8, v, v, v, 4, 1.0, 2, 0, v, v, 1 << 20, None) == 1
    assert lib.sfm_plane_sweep_ex(v, v, 1, 4, 8, 8, v, v, v, 4, 0.0, 0, 0, v, v, 1 << 20, None) == 1
    # plane sweep psnet: bad pose dtype, depth mode, min depth, null K, small workspace
    ws = lib.sfm_plane_sweep_workspace_bytes(1, 4, 8, 8)
    assert lib.sfm_plane_sweep_psnet(v, v, 1, 4, 8, 8, v, 2, v, v, 0.6, 4, 1.0, 0, 0, v, v, ws, None) == 1
    assert lib.sfm_plane_sweep_psnet(v, v, 1, 4, 8, 8, v, 1, v, v, 0.6, 4, 1.0, 2, 0, v, v, ws, None) == 1
    assert lib.sfm_plane_sweep_psnet(v, v, 1, 4, 8, 8, v, 1, v, v, 0.6, 4, 0.0, 0, 0, v, v, ws, None) == 1
    assert lib.sfm_plane_sweep_psnet(v, v, 1, 4, 8, 8, v, 1, None, v, 0.6, 4, 1.0, 0, 0, v, v, ws, None) == 1
    rc = lib.sfm_plane_sweep_psnet(v, v, 1, 4, 8, 8, v, 1, v, v, 0.6, 4, 1.0, 0, 0, v, v, ws - 1, None)
    assert rc == 3 and b"workspace" in lib.sfm_last_error()
    # tuning knobs: unknown key / out of range
    assert lib.sfm_tune_set(b"no_such_knob", 1) == 1
    assert lib.sfm_tune_set(b"sweep_items_per_block", 3) == 1


def test_regularisation_and_flow2depth_validate_arguments():
    """sfm_conv3_bf16 / sfm_to_channels_last_bf16 / sfm_flow2depth refuse bad
    shapes before any device work (no GPU here)."""
    from sfm_amd import _lib
    lib = _lib.load()
    v = ctypes.c_void_p(16)
    o = ctypes.c_void_p(4096)
    # cin must be 32 or 64, cout 32 or 1, residual only with cout 32
    assert lib.sfm_conv3_bf16(v, 1, 16, 4, 4, 4, v, v, v, None, 0, 32, o, None) == 1
    assert b"cin" in lib.sfm_last_error()
    assert lib.sfm_conv3_bf16(v, 1, 32, 4, 4, 4, v, v, v, None, 0, 8, o, None) == 1
    assert lib.sfm_conv3_bf16(v, 1, 32, 4, 4, 4, v, v, v, v, 0, 1, o, None) == 1
    # output aliasing the input, misaligned operands, empty shapes
    assert lib.sfm_conv3_bf16(v, 1, 32, 4, 4, 4, v, v, v, None, 0, 32, v, None) == 1
    assert lib.sfm_conv3_bf16(ctypes.c_void_p(18), 1, 32, 4, 4, 4, v, v, v, None, 0, 32, o, None) == 1
    assert lib.sfm_conv3_bf16(v, 1, 32, 0, 4, 4, v, v, v, None, 0, 32, o, None) == 1
    # channels-last: dtype code, channel multiple of 8
    assert lib.sfm_to_channels_last_bf16(v, 2, 1, 64, 100, o, None) == 1
    assert lib.sfm_to_channels_last_bf16(v, 0, 1, 12, 100, o, None) == 1
    # flow2depth: empty image
    assert lib.sfm_flow2depth(v, v, v, 1, 0, 10, o, None) == 1
    assert lib.sfm_tune_set(b"conv_rolling", 2) == 1


def test_tuning_keys_round_trip():
    """Every key the header documents can be read back; set values stick;
    out-of-range values are refused and leave the key unchanged."""
    import re
    from sfm_amd import _lib
    doc = open(os.path.join(ROOT, "include", "sfm_hip.h")).read()
    block = doc[doc.index("Tuning knobs"):doc.index("int sfm_tune_set")]
    keys = re.findall(r'"([a-z0-9_]+)"', block)
    assert set(keys) == set(_lib.tune_keys())           # documented == exported (sfm_tune_key)
    assert len(set(keys)) == 31 and "score_mf_prune" in keys and "score_lowp_template" in keys
    assert "score_mf_prune_upper" in keys
    assert "sweep_ref16" not in keys          # the bf16 reference-row copy experiment is gone
    for k in keys:
        _lib.tune_get(k)
    old = _lib.tune_get("sweep_nj")
    try:
        _lib.tune("sweep_nj", 4)
        assert _lib.tune_get("sweep_nj") == 4
        with pytest.raises(Exception):
            _lib.tune("sweep_nj", 3)
        assert _lib.tune_get("sweep_nj") == 4
    finally:
        _lib.tune("sweep_nj", old)
    with pytest.raises(Exception):
        _lib.tune_get("no_such_knob")
    snap = _lib.tune_snapshot()
    assert snap["score_mf"] == 2 and snap["score_mf_prune"] == 880 and snap["score_mf_chunk"] == 64
    _lib.tune_restore(snap)
    assert _lib.load().sfm_tune_key(-1) is None and _lib.last_scorer() == ""


def test_profile_select_filters_names():
    """sfm_profile_select parses its comma list (CPU: no launches, so every
    named slot reads zero) and NULL restores recording of every kernel."""
    from sfm_amd import _lib
    _lib.profile_select(["ransac_score", "plane_sweep"])
    _lib.profile_enable(True)
    _lib.profile_enable(False)
    assert _lib.profile_read("ransac_score") == (0.0, 0)
    _lib.profile_select(None)
    assert _lib.load().sfm_profile_select(b",,ransac_score,") == 0
    _lib.profile_select(None)


def test_score_fence_reference_counted():
    """sfm_score_fence_enable is reference-counted (TwoViewHotPath enables it
    for its lifetime); waiting with no enable left is refused before any HIP
    call (CPU-safe)."""
    from sfm_amd import _lib
    lib = _lib.load()
    assert lib.sfm_score_fence_enable(0) == 0            # never below zero
    assert lib.sfm_score_fence_wait(None) == 1
    assert lib.sfm_score_fence_enable(1) == 0 and lib.sfm_score_fence_enable(1) == 0
    assert lib.sfm_score_fence_enable(0) == 0 and lib.sfm_score_fence_enable(0) == 0
    assert lib.sfm_score_fence_wait(None) == 1 and b"not enabled" in lib.sfm_last_error()


def test_no_store_data_overwrite_hazard():
    """Round-5 finding (the round-4 sweep miscompute): on gfx950 a 128-bit VMEM
    store followed directly by a VALU write of one of its data VGPRs stores the
    new value for some lanes, and LLVM only guards stores without an SGPR
    soffset.  The product's 128-bit stores use a literal-0 soffset so the
    compiler inserts the wait state; this checks the built library's machine
    code for any unguarded pair (scripts/store_hazard_check.py)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import store_hazard_check as H
    from sfm_amd import _lib
    lines = H.library_device_code(_lib.LIB_PATH)
    assert sum("buffer_store_dwordx4" in l for l in lines) > 0      # the sweep's wide stores are in there
    hits = H.check(_lib.LIB_PATH, lines)
    assert hits == [], hits[:3]


def test_store_hazard_check_sees_vgpr_and_agpr_data():
    """The checker itself on synthetic assembly: a 128-bit store whose data
    VGPRs or AGPRs the next VALU instruction overwrites (v_mov / v_accvgpr_write
    / v_mfma) is reported; a guarded pair (s_nop between) and a write to
    other registers are not."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import store_hazard_check as H
    asm = """_Z1kv:
        buffer_store_dwordx4 v[4:7], v1, s[0:3], s4 offen
        v_mov_b32_e32 v5, 0
        buffer_store_dwordx4 a[8:11], v1, s[0:3], s4 offen
        v_accvgpr_write_b32 a9, v2
        global_store_dwordx4 v0, a[12:15], s[6:7]
        v_mfma_f32_32x32x16_f16 a[0:15], v[20:23], v[24:27], a[0:15]
        buffer_store_dwordx4 a[16:19], v1, s[0:3], s4 offen
        s_nop 0
        v_accvgpr_write_b32 a17, v2
        buffer_store_dwordx4 v[8:11], v1, s[0:3], s4 offen
        v_accvgpr_write_b32 a8, v2
    """.split("\n")
    hits = H.check(None, asm)
    assert [h[2].split()[0] for h in hits] == ["v_mov_b32_e32", "v_accvgpr_write_b32", "v_mfma_f32_32x32x16_f16"]


def test_reference_built_code_stays_in_the_build_container():
    """oracle/_ref (the reference's own sources compiled here, for golden
    generation only) never travels to the GPU box: .gpurunignore excludes it,
    and excludes neither the product library nor the checker the GPU tests load."""
    pats = [l.strip() for l in open(os.path.join(ROOT, ".gpurunignore")) if l.strip() and not l.startswith("#")]
    assert "./oracle/_ref" in pats
    for keep in ("./deep-sfm-revisited_amd", "./oracle", "*.so", "./oracle/liboracle_ransac.so", "./tests"):
        assert keep not in pats, keep
