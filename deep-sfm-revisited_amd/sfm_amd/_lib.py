"""ctypes binding of libsfm_hip.so (the C ABI declared in include/sfm_hip.h).

The product path has no CPU fallback: if the library cannot be loaded every
entry point raises.  Tensors cross the boundary as raw device pointers plus
sizes; work is enqueued on torch's current HIP stream.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFM_HIP_LIB") or os.path.join(_HERE, "libsfm_hip.so")   # override: A/B of library builds

_c_dp = ctypes.c_void_p
_i64p = ctypes.POINTER(ctypes.c_int64)

# (name, restype, argtypes)
_SIGS = [
    ("sfm_abi_version", ctypes.c_int, []),
    ("sfm_last_error", ctypes.c_char_p, []),
    ("sfm_ransac5_workspace_bytes", ctypes.c_size_t, [ctypes.c_int, ctypes.c_int64, ctypes.c_int]),
    ("sfm_ransac5", ctypes.c_int,
     [_c_dp, _c_dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
      ctypes.c_uint64, ctypes.c_int, _c_dp, ctypes.c_size_t, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp]),
    ("sfm_ransac5_packed", ctypes.c_int,
     [_c_dp, ctypes.c_int64, _i64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
      ctypes.c_double, ctypes.c_uint64, ctypes.c_int, _c_dp, ctypes.c_size_t, _c_dp, _c_dp, _c_dp, _c_dp,
      _c_dp, _c_dp]),
    ("sfm_ransac5_inlier_mask", ctypes.c_int,
     [_c_dp, ctypes.c_int64, _i64p, ctypes.c_int, _c_dp, ctypes.c_double, _c_dp, _c_dp]),
    ("sfm_flow_to_points", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp,
      _c_dp]),
    ("sfm_ransac5_candidate_counts", ctypes.c_int,
     [_c_dp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]),
    ("sfm_ransac5_kept_candidates", ctypes.c_int,
     [_c_dp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp]),
    ("sfm_ransac5_skipped_evaluations", ctypes.c_int,
     [_c_dp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64)]),
    ("sfm_pack_points", ctypes.c_int, [_c_dp, _c_dp, ctypes.c_int64, _c_dp, _c_dp]),
    ("sfm_essential_optimise", ctypes.c_int,
     [_c_dp, _c_dp, ctypes.c_int64, _c_dp, ctypes.c_double, ctypes.c_double, ctypes.c_int, _c_dp]),
    ("sfm_essential_decompose", ctypes.c_int, [_c_dp, _c_dp]),
    ("sfm_essential_decompose_uv", ctypes.c_int, [_c_dp, _c_dp, _c_dp]),
    ("sfm_plane_sweep_workspace_bytes", ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("sfm_plane_sweep", ctypes.c_int,
     [_c_dp, _c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, ctypes.c_int,
      ctypes.c_float, ctypes.c_int, _c_dp, _c_dp, ctypes.c_size_t, _c_dp]),
    ("sfm_plane_sweep_ex", ctypes.c_int,
     [_c_dp, _c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, ctypes.c_int,
      ctypes.c_float, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, ctypes.c_size_t, _c_dp]),
    ("sfm_plane_sweep_psnet", ctypes.c_int,
     [_c_dp, _c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, ctypes.c_int, _c_dp, _c_dp,
      ctypes.c_float, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, ctypes.c_size_t,
      _c_dp]),
    ("sfm_score_fence_enable", ctypes.c_int, [ctypes.c_int]),
    ("sfm_score_fence_wait", ctypes.c_int, [_c_dp]),
    ("sfm_score_gate", ctypes.c_int, [_c_dp, _c_dp, ctypes.c_int]),
    ("sfm_plane_sweep_ref_planes_workspace_bytes", ctypes.c_size_t,
     [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("sfm_plane_sweep_ref_planes", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp,
      ctypes.c_size_t, _c_dp]),
    ("sfm_plane_sweep_psnet_warped_half", ctypes.c_int,
     [_c_dp, _c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, ctypes.c_int, _c_dp, _c_dp,
      ctypes.c_float, ctypes.c_int, ctypes.c_float, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, ctypes.c_size_t,
      _c_dp]),
    ("sfm_plane_sweep_warped", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, ctypes.c_int,
      ctypes.c_float, ctypes.c_int, _c_dp, _c_dp, ctypes.c_size_t, _c_dp]),
    ("sfm_ransac5_flow", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp,
      ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.c_int, _c_dp,
      ctypes.c_size_t, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp]),
    ("sfm_keypoints_to_points", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, ctypes.c_int64,
      _c_dp, ctypes.c_int, _c_dp, _c_dp, ctypes.c_int64, _c_dp]),
    ("sfm_essential_optimise_workspace_bytes", ctypes.c_size_t, [ctypes.c_int, ctypes.c_int64]),
    ("sfm_essential_optimise_batched", ctypes.c_int,
     [_c_dp, ctypes.c_int64, _c_dp, ctypes.c_int, _c_dp, ctypes.c_double, ctypes.c_double, ctypes.c_int, _c_dp,
      _c_dp, ctypes.c_size_t, _c_dp]),
    ("sfm_correlation_workspace_bytes", ctypes.c_size_t, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    ("sfm_plane_sweep_correlation", ctypes.c_int,
     [_c_dp, _c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, ctypes.c_int,
      ctypes.c_float, ctypes.c_int, _c_dp, _c_dp, ctypes.c_size_t, _c_dp]),
    ("sfm_depth_head", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
      ctypes.c_float, ctypes.c_float, _c_dp, _c_dp]),
    ("sfm_inverse_warp", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp]),
    ("sfm_kinv3x3", ctypes.c_int, [_c_dp, ctypes.c_int, _c_dp, _c_dp]),
    ("sfm_flow2depth", ctypes.c_int, [_c_dp, _c_dp, _c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp]),
    ("sfm_conv3_bf16", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, _c_dp,
      ctypes.c_int, ctypes.c_int, _c_dp, _c_dp]),
    ("sfm_to_channels_last_bf16", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp]),
    ("sfm_conv3_f16", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, _c_dp,
      ctypes.c_int, ctypes.c_int, _c_dp, _c_dp]),
    ("sfm_to_channels_last_f16", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp]),
    ("sfm_conv3_f32", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp, _c_dp,
      ctypes.c_int, ctypes.c_int, _c_dp, _c_dp]),
    ("sfm_conv3_f32x3", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _c_dp, ctypes.c_int, _c_dp, _c_dp,
      _c_dp, ctypes.c_int, ctypes.c_int, _c_dp, _c_dp, _c_dp]),
    ("sfm_to_channels_last_f32", ctypes.c_int,
     [_c_dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int64, _c_dp, _c_dp]),
    ("sfm_score_essentials_workspace_bytes", ctypes.c_size_t, [ctypes.c_int, ctypes.c_int]),
    ("sfm_score_essentials", ctypes.c_int,
     [_c_dp, ctypes.c_int64, _i64p, ctypes.c_int, _c_dp, ctypes.c_int, ctypes.c_double, _c_dp, _c_dp,
      ctypes.c_size_t, _c_dp]),
    ("sfm_tune_set", ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    ("sfm_tune_get", ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    ("sfm_tune_key", ctypes.c_char_p, [ctypes.c_int]),
    ("sfm_last_scorer", ctypes.c_char_p, []),
    ("sfm_profile_enable", ctypes.c_int, [ctypes.c_int]),
    ("sfm_profile_select", ctypes.c_int, [ctypes.c_char_p]),
    ("sfm_profile_reset", ctypes.c_int, []),
    ("sfm_profile_read", ctypes.c_int,
     [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]),
]

SYMBOLS = [s[0] for s in _SIGS]

_lib = None
_load_error = None


class SfmError(RuntimeError):
    pass


def load():
    """Load libsfm_hip.so (once).  Raises SfmError if it is missing."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SfmError(f"libsfm_hip.so not found at {LIB_PATH}: build it with "
                       f"`make -C deep-sfm-revisited_amd/csrc` (or __graft_entry__.build())")
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the runtime
        _load_error = e
        raise SfmError(f"cannot load {LIB_PATH}: {e}") from e
    for name, res, args in _SIGS:
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if lib.sfm_abi_version() != 1:
        raise SfmError("libsfm_hip ABI version mismatch")
    _lib = lib
    return lib


def check(rc, what):
    if rc != 0:
        msg = load().sfm_last_error().decode("utf-8", "replace")
        raise SfmError(f"{what} failed (code {rc}): {msg}")


def ptr(t):
    """Raw data pointer of a tensor (None -> NULL)."""
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def i64_array(values):
    arr = (ctypes.c_int64 * len(values))(*[int(v) for v in values])
    return arr


def profile_enable(on=True):
    check(load().sfm_profile_enable(1 if on else 0), "sfm_profile_enable")


def profile_select(names=None):
    """Record only the named kernels (None / empty: all) while profiling is on."""
    arg = None if not names else ",".join(names).encode()
    check(load().sfm_profile_select(arg), "sfm_profile_select")


def profile_reset():
    check(load().sfm_profile_reset(), "sfm_profile_reset")


def profile_read(name):
    ms = ctypes.c_double(0.0)
    n = ctypes.c_int(0)
    check(load().sfm_profile_read(name.encode(), ctypes.byref(ms), ctypes.byref(n)), "sfm_profile_read")
    return ms.value, n.value


def tune(key, value):
    """Set a launch-shape knob of libsfm_hip (see sfm_tune_set in include/sfm_hip.h)."""
    check(load().sfm_tune_set(key.encode(), int(value)), "sfm_tune_set")


def tune_get(key):
    """The current value of a tuning knob (sfm_tune_get)."""
    v = ctypes.c_int(0)
    check(load().sfm_tune_get(key.encode(), ctypes.byref(v)), "sfm_tune_get")
    return v.value


def tune_keys():
    """Every tuning key of the library, in its own order (sfm_tune_key)."""
    keys, i = [], 0
    while True:
        k = load().sfm_tune_key(i)
        if k is None:
            return keys
        keys.append(k.decode())
        i += 1


def tune_snapshot():
    """{key: value} of every tuning knob (restore with tune_restore)."""
    return {k: tune_get(k) for k in tune_keys()}


def tune_restore(snap):
    for k, v in snap.items():
        tune(k, v)


def last_scorer():
    """The score kernel the last RANSAC / score call dispatched (sfm_last_scorer)."""
    return load().sfm_last_scorer().decode()
