"""ORACLE (test infrastructure only): ctypes bindings of the C++ restatement
(oracle/ransac5_oracle.cpp) and, when built, of the reference solver
(oracle/_ref/libref_ransac.so, see oracle/Makefile)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle_ransac.so")
_REF = os.path.join(_HERE, "_ref", "libref_ransac.so")

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build(ref=False):
    """Compile the oracle (and, if asked and the reference tree exists, _ref)."""
    targets = ["all"] + (["ref"] if ref else [])
    subprocess.run(["make", "-s", "-C", _HERE] + targets, check=True)


def _ptr(a, t=_dp):
    return a.ctypes.data_as(t)


def _load(path, prefix):
    lib = ctypes.CDLL(path)
    f = getattr(lib, prefix + "solve5")
    f.argtypes = [_dp, _dp, ctypes.c_int, _dp, _ip, _dp, _dp, _ip]
    f.restype = ctypes.c_int
    f = getattr(lib, prefix + "decompose")
    f.argtypes = [_dp, _dp]
    f.restype = None
    f = getattr(lib, prefix + "decompose_uv")
    f.argtypes = [_dp, _dp, _dp]
    f.restype = None
    f = getattr(lib, prefix + "optimise")
    f.argtypes = [_dp, _dp, ctypes.c_int64, _dp, ctypes.c_double, ctypes.c_double, ctypes.c_int, _dp]
    f.restype = None
    return lib


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        _lib = _load(_LIB, "orc_")
        _lib.orc_ransac5.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                     _dp, _dp, _ip, _ip, _ip, _ip, _ip]
        _lib.orc_ransac5.restype = ctypes.c_int
        _lib.orc_ransac5_prec.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, _dp, _dp, _ip, _ip, _ip, _ip, _ip]
        _lib.orc_ransac5_prec.restype = ctypes.c_int
        _lib.orc_inlier_mask_prec.argtypes = [_dp, _dp, _dp, ctypes.c_int64, ctypes.c_double, ctypes.c_int, _u8p]
        _lib.orc_inlier_mask_prec.restype = None
        _lib.orc_inlier_mask.argtypes = [_dp, _dp, _dp, ctypes.c_int64, ctypes.c_double, _u8p]
        _lib.orc_inlier_mask.restype = None
        _lib.orc_sample_index.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64]
        _lib.orc_sample_index.restype = ctypes.c_int64
        _lib.orc_philox_u32.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        _lib.orc_philox_u32.restype = ctypes.c_uint32
    return _lib


def ref_available():
    return os.path.exists(_REF)


def ref():
    """The reference's own solver (host-compiled). Only present where it was built."""
    global _ref
    if _ref is None:
        if not os.path.exists(_REF):
            raise FileNotFoundError("oracle/_ref/libref_ransac.so not built (needs /root/reference)")
        _ref = _load(_REF, "ref_")
        _ref.ref_ransac5.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_double, ctypes.c_uint64, ctypes.c_int,
                                     _dp, _dp, _ip, _ip, _ip, _ip]
        _ref.ref_ransac5.restype = ctypes.c_int
    return _ref


def _solve5(L, prefix, q5, qp5, cheir=True):
    q5 = np.ascontiguousarray(q5, dtype=np.float64).reshape(5, 2)
    qp5 = np.ascontiguousarray(qp5, dtype=np.float64).reshape(5, 2)
    er = np.zeros((10, 9)); eo = np.zeros((10, 9)); po = np.zeros((10, 12))
    nr = ctypes.c_int(0); npp = ctypes.c_int(0)
    getattr(L, prefix + "solve5")(_ptr(q5), _ptr(qp5), int(cheir), _ptr(er), ctypes.byref(nr),
                                  _ptr(eo), _ptr(po), ctypes.byref(npp))
    return dict(nroots=nr.value, E_roots=er, nP=npp.value, E=eo, P=po)


def solve5(q5, qp5, cheir=True):
    """Five-point solve (+cheirality) of one 5-tuple: the oracle restatement."""
    return _solve5(lib(), "orc_", q5, qp5, cheir)


def ref_solve5(q5, qp5, cheir=True):
    """Same, through the reference's own host-compiled solver."""
    return _solve5(ref(), "ref_", q5, qp5, cheir)


def sample_index(seed, h, d, n):
    return lib().orc_sample_index(seed, h, d, n)


def philox_u32(seed, h, d):
    return lib().orc_philox_u32(seed, h, d)


def ransac5(q, qp, num_test=None, num_ransac_test=None, iters=5, thr=1e-4, seed=1234, cheir=True,
            nchains=512, nthreads=0, use_ref=False, prec=64):
    """Full RANSAC emulation for one pair. Returns dict(E, P, inliers, winner,
    hyp_score, hyp_ncand).  prec: 64 (the reference's ComputeError<double>),
    33 / 17 (the literal ComputeError<float> / <half> template form),
    32 / 16 (ComputeError<float> / <half>, ransac5_oracle.cpp:is_inlier_lp)."""
    q = np.ascontiguousarray(q, dtype=np.float64)
    qp = np.ascontiguousarray(qp, dtype=np.float64)
    n = q.shape[0]
    num_test = n if num_test is None else num_test
    num_ransac_test = n if num_ransac_test is None else num_ransac_test
    H = nchains * iters
    E = np.zeros(9); P = np.zeros(12)
    inl = ctypes.c_int(0); win = ctypes.c_int(0)
    score = np.zeros(H, dtype=np.int32); ncand = np.zeros(H, dtype=np.int32)
    best = np.zeros(H, dtype=np.int32)
    if use_ref:
        rc = ref().ref_ransac5(_ptr(q), _ptr(qp), n, num_test, num_ransac_test, nchains, iters, thr, seed,
                               int(cheir), _ptr(E), _ptr(P), ctypes.byref(inl), ctypes.byref(win),
                               _ptr(score, _ip), _ptr(ncand, _ip))
    else:
        rc = lib().orc_ransac5_prec(_ptr(q), _ptr(qp), n, num_test, num_ransac_test, nchains, iters, thr, seed,
                                    int(cheir), nthreads, int(prec), _ptr(E), _ptr(P), ctypes.byref(inl),
                                    ctypes.byref(win), _ptr(score, _ip), _ptr(ncand, _ip), _ptr(best, _ip))
    if rc != 0:
        raise RuntimeError("oracle ransac5: invalid arguments")
    return dict(E=E.reshape(3, 3), P=P.reshape(3, 4), inliers=inl.value, winner=win.value,
                hyp_score=score, hyp_ncand=ncand, hyp_best=best)


def inlier_mask(E, q, qp, thr, prec=64):
    E = np.ascontiguousarray(E, dtype=np.float64).reshape(9)
    q = np.ascontiguousarray(q, dtype=np.float64)
    qp = np.ascontiguousarray(qp, dtype=np.float64)
    m = np.zeros(q.shape[0], dtype=np.uint8)
    if prec == 64:
        lib().orc_inlier_mask(_ptr(E), _ptr(q), _ptr(qp), q.shape[0], thr, _ptr(m, _u8p))
    else:
        lib().orc_inlier_mask_prec(_ptr(E), _ptr(q), _ptr(qp), q.shape[0], thr, int(prec), _ptr(m, _u8p))
    return m.astype(bool)


def inlier_mask_numpy(E, q, qp, thr, prec):
    """numpy restatement of ransac5_oracle.cpp:is_inlier_lp (checks the C++
    half rounding): numpy float16 / float32 arithmetic rounds every operation
    to the type; float16 ops are computed in float32 and rounded once, which
    is the correctly rounded half result (24 >= 2*11 + 2 bits)."""
    T = np.float16 if prec == 16 else np.float32
    c = lambda v: np.asarray(np.asarray(v, np.float64).astype(np.float32)).astype(T)
    E = np.asarray(E, np.float64).reshape(9)
    m = float(np.abs(E).max())
    ex = int(np.frexp(m)[1]) if 0.0 < m < 2.0 ** 1000 else 0
    e = c(np.ldexp(E, -ex))                 # exact power-of-two scaling to max |E_ij| in [0.5, 1)
    x, y, xp, yp = c(q[:, 0]), c(q[:, 1]), c(qp[:, 0]), c(qp[:, 1])
    with np.errstate(all="ignore"):
        ex0 = (e[0] * x + e[1] * y) + e[2]
        ex1 = (e[3] * x + e[4] * y) + e[5]
        ex2 = (e[6] * x + e[7] * y) + e[8]
        xe0 = (xp * e[0] + yp * e[3]) + e[6]
        xe1 = (xp * e[1] + yp * e[4]) + e[7]
        a = (xp * ex0 + yp * ex1) + ex2
        D = ((ex0 * ex0 + ex1 * ex1) + xe0 * xe0) + xe1 * xe1
        d = np.sqrt(D.astype(np.float32)).astype(T)
        err = np.abs((a.astype(np.float32) / d.astype(np.float32)).astype(T))
    return err.astype(np.float64) <= thr


def inlier_mask_numpy_tpl(E, q, qp, thr, prec):
    """numpy restatement of ransac5_oracle.cpp:is_inlier_lp_tpl (prec 33 = float,
    17 = half): the literal ComputeError<T> with a double Ematrix (double
    products and adds, each sum rounded to T; xEx, D, sqrt, division in T).
    numpy's float64 -> float16 conversion rounds once, like h16d."""
    T = np.float16 if prec == 17 else np.float32
    E = np.asarray(E, np.float64).reshape(3, 3)
    q = [np.asarray(q[:, 0], np.float64).astype(T), np.asarray(q[:, 1], np.float64).astype(T),
         np.ones(len(q), T)]
    qp = [np.asarray(qp[:, 0], np.float64).astype(T), np.asarray(qp[:, 1], np.float64).astype(T),
          np.ones(len(qp), T)]
    with np.errstate(all="ignore"):
        Ex, xE = [], []
        for k in range(3):
            s_ = np.zeros(len(q[0]), T)
            for l in range(3):
                s_ = (s_.astype(np.float64) + E[k, l] * q[l].astype(np.float64)).astype(T)
            Ex.append(s_)
        for k in range(3):
            s_ = np.zeros(len(q[0]), T)
            for l in range(3):
                s_ = (s_.astype(np.float64) + qp[l].astype(np.float64) * E[l, k]).astype(T)
            xE.append(s_)
        xEx = np.zeros(len(q[0]), T)
        for k in range(3):
            xEx = xEx + qp[k] * Ex[k]
        D = ((Ex[0] * Ex[0] + Ex[1] * Ex[1]) + xE[0] * xE[0]) + xE[1] * xE[1]
        d = np.sqrt(D.astype(np.float32)).astype(T)
        err = np.abs((xEx.astype(np.float32) / d.astype(np.float32)).astype(T))
    return err.astype(np.float64) <= thr


def _decomp(L, prefix, E):
    E = np.ascontiguousarray(E, dtype=np.float64).reshape(9)
    out = np.zeros(5)
    getattr(L, prefix + "decompose")(_ptr(E), _ptr(out))
    return out


def decompose(E, use_ref=False):
    return _decomp(ref() if use_ref else lib(), "ref_" if use_ref else "orc_", E)


def decompose_uv(E, use_ref=False):
    L, prefix = (ref(), "ref_") if use_ref else (lib(), "orc_")
    E = np.ascontiguousarray(E, dtype=np.float64).reshape(9)
    U = np.zeros(9); V = np.zeros(9)
    getattr(L, prefix + "decompose_uv")(_ptr(E), _ptr(U), _ptr(V))
    return U.reshape(3, 3), V.reshape(3, 3)


def optimise(q, qp, E_init, delta=0.001, alpha=0.0, max_reps=200, use_ref=False):
    L, prefix = (ref(), "ref_") if use_ref else (lib(), "orc_")
    q = np.ascontiguousarray(q, dtype=np.float64)
    qp = np.ascontiguousarray(qp, dtype=np.float64)
    E = np.ascontiguousarray(E_init, dtype=np.float64).reshape(9)
    out = np.zeros(9)
    getattr(L, prefix + "optimise")(_ptr(q), _ptr(qp), q.shape[0], _ptr(E), delta, alpha, max_reps, _ptr(out))
    return out.reshape(3, 3)
