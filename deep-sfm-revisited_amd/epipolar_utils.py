"""Drop-in for the hot-path functions of the reference's epipolar_utils.py
(epipolar_utils.py:8-135): the glue between the correspondences and the
`essential_matrix` extension.  The unused bilevel-optimisation helpers
(epipolar_utils.py:139-357) are out of scope."""
import torch

import essential_matrix


def flow2coord(flow):
    """epipolar_utils.py:8-28: flow [b,2,h,w] -> homogeneous coords [b,3,h*w] (x2)."""
    b, _, h, w = flow.size()
    coord1 = torch.zeros_like(flow)
    coord1[:, 0, :, :] += torch.arange(w, dtype=flow.dtype, device=flow.device)
    coord1[:, 1, :, :] += torch.arange(h, dtype=flow.dtype, device=flow.device)[:, None]
    coord2 = coord1 + flow
    ones = torch.ones((b, 1, h * w), dtype=torch.float32, device=flow.device)
    return (torch.cat((coord1.reshape(b, 2, h * w), ones), dim=1),
            torch.cat((coord2.reshape(b, 2, h * w), ones), dim=1))


def coord2flow(coord1, coord2, b, h, w):
    """epipolar_utils.py:32-46"""
    return (coord2[:, :2, :] - coord1[:, :2, :]).reshape(b, 2, h, w)


def compute_P_matrix_ransac(coord1, coord2, intrinsic_inv, delta, alpha, maxreps, num_test_points,
                            ransac_test_points, ransac_iter, ransac_threshold):
    """epipolar_utils.py:112-135 -> (E f32 [3,3], P f64 [3,4], F f32 [3,3], inliers int)"""
    E_init, P_init, inlier_num = essential_matrix.computeP(coord1.double(), coord2.double(), num_test_points,
                                                           ransac_test_points, ransac_iter, ransac_threshold)
    E_init = E_init.float()
    F_init = intrinsic_inv.transpose(0, 1).mm(E_init).mm(intrinsic_inv)
    return E_init, P_init, F_init, inlier_num


def compute_E_matrix_ransac(coord1, coord2, intrinsic_inv, delta, alpha, maxreps, num_test_points,
                            ransac_test_points, ransac_iter, ransac_threshold):
    """epipolar_utils.py:87-110 -> (E f32, F f32)"""
    E_init = essential_matrix.initialise(coord1.double(), coord2.double(), num_test_points, ransac_test_points,
                                         ransac_iter, ransac_threshold)
    E_init = E_init.float()
    F_init = intrinsic_inv.transpose(0, 1).mm(E_init).mm(intrinsic_inv)
    return E_init, F_init


def compute_E_matrix(coord1_hom, coord2_hom, intrinsic_inv, delta, alpha, maxreps, num_test_points,
                     ransac_test_points, ransac_iter, ransac_threshold):
    """epipolar_utils.py:49-85: RANSAC initialisation + host IRLS refinement.
    (The reference passes [1,N,2] tensors here, which its extension reads as
    N = 1; this build passes the [N,2] correspondences.)"""
    c1 = coord1_hom.mm(intrinsic_inv.transpose(0, 1))[:, :2].contiguous().cuda()
    c2 = coord2_hom.mm(intrinsic_inv.transpose(0, 1))[:, :2].contiguous().cuda()
    E_init = essential_matrix.initialise(c1.double(), c2.double(), num_test_points, ransac_test_points,
                                         ransac_iter, ransac_threshold)
    E_opt = essential_matrix.optimise(c1.double().cpu(), c2.double().cpu(), E_init.double().cpu(), delta, alpha,
                                      maxreps)
    E_init = E_init.float()
    E_opt = E_opt.float().to(c1.device)
    Ki = intrinsic_inv.to(c1.device)
    F_init = Ki.transpose(0, 1).mm(E_init).mm(Ki)
    F_opt = Ki.transpose(0, 1).mm(E_opt).mm(Ki)
    return E_init, E_opt, F_init, F_opt
