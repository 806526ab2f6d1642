"""SFMnet with the MI355X hot path (models/SFMnet.py:33-274 of the reference).

Same constructor arguments, ``forward`` signature, control flow and return
tuples as the reference, so main.py's ``model(input1, input0, K, pose_gt_bw,
pred_pose_bw, cfg.GT_POSE, H_raw, W_raw)`` (main.py:533) drops in.  The pose
branch (``pose_by_ransac``) runs on libsfm_hip for the whole batch at once:

  correspondences   dense flow crop (sfm_flow_to_points) or, for pairs with
                    >= min_matches keypoint matches, the sparse gather
                    (sfm_keypoints_to_points: round / SAMPLE_SP / SIFT_POSE)
  RANSAC            one batched sfm_ransac5_packed launch over all pairs
                    (the reference loops over pairs, SFMnet.py:216-272)

Default construction follows SFMnet.__init__ (SFMnet.py:33-75): with
cfg.DEPTH_EST == 'PSNET' (the default) ``SFMnet(nlabel)`` builds
``sfm_amd.psnet.PSNet(nlabel, min_depth)`` -- PSNet's module layout with the
sweep, the 3-D regularisation and the head on libsfm_hip -- so
``SFMnet(args.nlabel)`` (main.py:198) runs as it stands.  Out of scope
(tier framing) and therefore injected: the flow estimator (RAFT /
DICL: ``flow_estimator=``; its absence is a named RuntimeError when forward
needs a flow), the other depth estimators (CVP, PANet, REGNet, REG2D,
DISPNET: a named RuntimeError at construction unless ``depth_estimator=`` is
given), the keypoint matcher (cv2 SIFT/SURF + FLANN, absent here) and
PoseNet.
"""
import time

import numpy as np
import torch

from sfm_amd import ransac as _ransac
from sfm_amd.config import cfg as _default_cfg

time_dict = {}


class SFMnet(torch.nn.Module):
    def __init__(self, nlabel=64, min_depth=0.5, flow_estimator=None, depth_estimator=None, matcher=None,
                 cfg=None, feature_fn=None):
        super().__init__()
        self.cfg = _default_cfg if cfg is None else cfg
        c = self.cfg
        # SFMnet.py:35-42
        self.delta = 0.001
        self.alpha = 0.0
        self.maxreps = 200
        self.min_matches = c.min_matches
        self.ransac_iter = c.ransac_iter
        self.ransac_threshold = c.ransac_threshold
        self.nlabel = nlabel
        self.min_depth = min_depth
        self.flow_estimator = flow_estimator
        if depth_estimator is None:
            kind = c.get("DEPTH_EST", "PSNET")
            if kind != "PSNET":
                raise RuntimeError(f"SFMnet: cfg.DEPTH_EST={kind!r} is not built here (only PSNET, SFMnet.py:57-58); "
                                   f"pass depth_estimator= (a module with PSNet.forward's signature)")
            from sfm_amd.psnet import PSNet
            depth_estimator = PSNet(nlabel, min_depth, cfg=c, feature_fn=feature_fn)
        self.depth_estimator = depth_estimator
        # matcher(ref_img_hwc_uint8, tgt_img_hwc_uint8) -> (pts1 [n,2], pts2 [n,2]) or None;
        # stands in for SIFT/SURF detectAndCompute + FLANN ratio test (SFMnet.py:190-214)
        self.matcher = matcher
        if c.POSE_EST != "RANSAC":
            raise NotImplementedError("only POSE_EST='RANSAC' is on the hot path (PoseNet is out of scope)")
        self._ws = None

    def forward(self, ref, target, intrinsic, pose_gt=None, pred_pose=None, use_gt_pose=False,
                h_side=None, w_side=None, logger=None, depth_gt=None, img_path=None):
        c = self.cfg
        if self.training and c.get("TRAIN_FLOW", False):
            return self._flow()(torch.cat((ref, target), dim=1))

        intrinsic_gpu = intrinsic.float().cuda()
        intrinsic_inv_gpu = torch.inverse(intrinsic_gpu)

        if use_gt_pose is False:
            if c.PRED_POSE_ONLINE:
                flow_start = time.time()
                with torch.autocast("cuda", enabled=bool(c.MIXED_PREC)):
                    flow_2D, conf = self._flow()(torch.cat((ref, target), dim=1))
                time_dict["flow"] = time.time() - flow_start
                if h_side is not None or w_side is not None:
                    flow_2D = flow_2D[:, :, :h_side, :w_side]
                    try:
                        conf = conf[:, :, :h_side, :w_side]
                    except Exception:
                        pass
                P_mat, E_mat = self.pose_by_ransac(flow_2D, ref, target, intrinsic_inv_gpu, h_side, w_side,
                                                   pose_gt=pose_gt, img_path=img_path)
                rot_and_trans = None
            else:
                P_mat = pred_pose
                E_mat = None
                flow_2D = None
                rot_and_trans = None
            if c.PRED_POSE_GT_SCALE:
                scale = torch.norm(pose_gt[:, :3, 3], dim=1, p=2).unsqueeze(1).unsqueeze(1)
                P_mat[:, :, -1:] = P_mat[:, :, -1:] * scale
            P_mat.unsqueeze_(1)
        else:
            E_mat = None
            rot_and_trans = None
            P_mat = pose_gt.clone()
            if c.GT_POSE_NORMALIZED:
                scale = torch.norm(P_mat[:, :3, 3], dim=1, p=2).unsqueeze(1).unsqueeze(1)
                P_mat[:, :, -1:] = P_mat[:, :, -1:] / scale
            P_mat.unsqueeze_(1)
            flow_2D = torch.zeros([ref.shape[0], 2, ref.shape[2], ref.shape[3]], device=ref.device).type_as(ref)

        if c.RECORD_POSE or (c.RECORD_POSE_EVAL and not self.training):
            return P_mat, flow_2D

        if h_side is not None or w_side is not None:
            ref = ref[:, :, :h_side, :w_side]
            target = target[:, :, :h_side, :w_side]

        depth_start = time.time()
        with torch.autocast("cuda", enabled=bool(c.MIXED_PREC)):
            depth_init, depth = self.depth_estimator(ref, [target], P_mat, intrinsic_gpu, intrinsic_inv_gpu,
                                                     pose_gt=pose_gt, depth_gt=depth_gt, E_mat=E_mat)
        time_dict["depth"] = time.time() - depth_start
        if self.training:
            return flow_2D, P_mat, depth, depth_init, rot_and_trans
        return flow_2D, P_mat, depth, time_dict

    def _flow(self):
        if self.flow_estimator is None:
            raise RuntimeError(f"SFMnet: this forward needs optical flow, and cfg.FLOW_EST="
                               f"{self.cfg.get('FLOW_EST', 'DICL')!r} (RAFT / DICL) is out of scope here: pass "
                               f"flow_estimator= (images [B,6,H,W] -> (flow [B,2,H,W], conf)), or use GT / "
                               f"predicted poses")
        return self.flow_estimator

    # ------------------------------------------------------------------
    def _matches(self, ref, target, h_side, w_side):
        """Per-pair keypoint matches (PTS1, PTS2) as SFMnet.py:186-214 builds them."""
        b = ref.shape[0]
        if self.matcher is None:
            return [None] * b, [None] * b
        P1, P2 = [], []
        for i in range(b):
            r = ref[i, :, :h_side, :w_side] if (h_side is not None or w_side is not None) else ref[i]
            t = target[i, :, :h_side, :w_side] if (h_side is not None or w_side is not None) else target[i]
            r = ((r.cpu().numpy().transpose(1, 2, 0)[:, :, ::-1] * 0.5 + 0.5) * 255).astype(np.uint8)
            t = ((t.cpu().numpy().transpose(1, 2, 0)[:, :, ::-1] * 0.5 + 0.5) * 255).astype(np.uint8)
            try:
                m = self.matcher(r, t)
            except Exception:
                m = None
            if m is None:
                P1.append(None); P2.append(None)
            else:
                P1.append(np.asarray(m[0], np.float64).reshape(-1, 2))
                P2.append(np.asarray(m[1], np.float64).reshape(-1, 2))
        return P1, P2

    def pose_by_ransac(self, flow_2D, ref, target, intrinsic_inv_gpu, h_side, w_side, pose_gt=False,
                       img_path=None):
        """SFMnet.py:176-274 for the whole batch: returns P_mat [B,3,4], E_mat [B,3,3] (float32)."""
        c = self.cfg
        b, _, h, w = flow_2D.size()
        margin = 10
        PTS1, PTS2 = self._matches(ref, target, h_side, w_side)
        flow = flow_2D.float().contiguous()
        Ki = intrinsic_inv_gpu.float().contiguous()
        sift_pose = bool(c.get("SIFT_POSE", False))
        sparse = [(p is not None) and (sift_pose or (len(p) >= self.min_matches and len(PTS2[i]) >= self.min_matches))
                  for i, p in enumerate(PTS1)]
        if sift_pose and not all(sparse):
            raise RuntimeError("SIFT_POSE needs keypoint matches for every pair (the reference fails too)")
        n_dense = (h - 2 * margin) * (w - 2 * margin)
        n = [len(PTS1[i]) if sparse[i] else n_dense for i in range(b)]
        n_stride = max(n)
        pts = torch.zeros(b, n_stride, 4, dtype=torch.float64, device=flow.device)
        dense_idx = [i for i in range(b) if not sparse[i]]
        if dense_idx:
            d = torch.tensor(dense_idx, device=flow.device)
            dp = _ransac.flow_to_points(flow[d], Ki[d], h, w, margin)
            pts[d, :n_dense] = dp
        sp_idx = [i for i in range(b) if sparse[i]]
        if sp_idx:
            mode = "sift_pose" if sift_pose else ("sample_sp" if c.get("SAMPLE_SP", False) else "round")
            s = torch.tensor(sp_idx, device=flow.device)
            sp, ns = _ransac.keypoints_to_points(flow[s], Ki[s], [PTS1[i] for i in sp_idx],
                                                 [PTS2[i] for i in sp_idx] if sift_pose else None, mode, h, w)
            for j, i in enumerate(sp_idx):
                pts[i, :ns[j]] = sp[j, :ns[j]]
        if self._ws is None or self._ws[0] != (b, self.ransac_iter) or self._ws[1].device != flow.device:
            self._ws = ((b, self.ransac_iter), _ransac.workspace_for(b, self.ransac_iter, flow.device))
        E, P, _, _ = _ransac.ransac5_batched(pts, n, None, None, self.ransac_iter, self.ransac_threshold,
                                             workspace=self._ws[1])
        # E_i.float(), P_i (f64) assigned into float32 E_mat / P_mat (SFMnet.py:266-272)
        return P.float(), E.float()
