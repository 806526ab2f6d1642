"""Drop-in for the reference's `essential_matrix` PyTorch extension
(RANSAC_FiveP/essential_matrix/essential_matrix_wrapper.cpp:102-108), backed
by libsfm_hip.so on MI355X.

Same functions, argument meaning, return types and checks:

    initialise(input1, input2, num_test_points, num_ransac_test_points,
               num_ransac_iterations, inlier_threshold) -> E [3,3] f64 (device)
    computeP(...same...)          -> (E [3,3] f64, P [3,4] f64, max_inliers: int)
    optimise(input1, input2, E_init, delta, alpha, MaxReps) -> E [3,3] f64 (CPU)
    decompose(Emat)               -> [5] f64 (CPU)   angles (x, y, z, u, v)
    decomposeUV(Emat)             -> (U [3,3], V [3,3]) (CPU)

input1/input2 are [N,2] correspondences (normalised coordinates), float64,
contiguous, on the GPU for initialise/computeP (RuntimeError otherwise, as the
TORCH_CHECKs of essential_matrix_wrapper.cpp:36-43).  Deviations, all
documented in DESIGN.md: launch errors raise instead of exit(); hypothesis
sampling uses the build's Philox sampler (cuRAND XORWOW is unavailable); the
indeterminate outputs of the reference (no inlier anywhere) are zeros.
"""
import torch

from sfm_amd import _lib
from sfm_amd import ransac as _ransac

SEED = _ransac.DEFAULT_SEED


def _check_opt(t, name):
    if t.dtype != torch.float64:
        raise RuntimeError(f"{name} must be a double tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def initialise(input1, input2, num_test_points, num_ransac_test_points, num_ransac_iterations, inlier_threshold):
    """EssentialMatrixInitialise (essential_matrix.cu:110-184): RANSAC without
    the cheirality test."""
    E, _, inl, _ = _ransac.ransac5(input1, input2, num_test_points, num_ransac_test_points, num_ransac_iterations,
                                   inlier_threshold, SEED, cheirality=False)
    print("The number of inliers: " + str(int(inl.item())))   # essential_matrix.cu:170
    return E


def computeP(input1, input2, num_test_points, num_ransac_test_points, num_ransac_iterations, inlier_threshold):
    """ProjectionMatrixRansac (essential_matrix.cu:190-280)."""
    E, P, inl, _ = _ransac.ransac5(input1, input2, num_test_points, num_ransac_test_points, num_ransac_iterations,
                                   inlier_threshold, SEED, cheirality=True)
    return E, P, int(inl.item())


def optimise(input1, input2, E_init, delta, alpha, MaxReps):
    """EssentialMatrixOptimise (essential_matrix.cu:76-105): host IRLS."""
    _check_opt(input1, "input1")
    _check_opt(input2, "input2")
    _check_opt(E_init, "E_init")
    q = input1.cpu().contiguous()
    qp = input2.cpu().contiguous()
    Ei = E_init.cpu().contiguous()
    out = torch.empty(3, 3, dtype=torch.float64)
    rc = _lib.load().sfm_essential_optimise(_lib.ptr(q), _lib.ptr(qp), q.shape[0], _lib.ptr(Ei), float(delta),
                                            float(alpha), int(MaxReps), _lib.ptr(out))
    _lib.check(rc, "optimise")
    return out.to(E_init.device)


def decompose(Emat):
    """EssentialMatrixDecompose (essential_matrix.cu:29-43)."""
    E = Emat.detach().to("cpu", torch.float64).contiguous()
    out = torch.empty(5, dtype=torch.float64)
    _lib.check(_lib.load().sfm_essential_decompose(_lib.ptr(E), _lib.ptr(out)), "decompose")
    return out


def decomposeUV(Emat):
    """EssentialMatrixDecomposeUV (essential_matrix.cu:48-70)."""
    E = Emat.detach().to("cpu", torch.float64).contiguous()
    U = torch.empty(3, 3, dtype=torch.float64)
    V = torch.empty(3, 3, dtype=torch.float64)
    _lib.check(_lib.load().sfm_essential_decompose_uv(_lib.ptr(E), _lib.ptr(U), _lib.ptr(V)), "decomposeUV")
    return U, V

